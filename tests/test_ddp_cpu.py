"""Flat-buffer DDP over gloo (world_size 2): gradient equivalence with a single-process run on the
global batch, gradient accumulation (no_sync), direct-write weight gradients, param broadcast."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, accum):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gke_ray_train_amd.models import build_llama
        from gke_ray_train_amd.parallel import DistributedDataParallel
        torch.manual_seed(100 + rank)  # different init per rank: broadcast must fix it
        m = build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=None)
        m.init_weights(seed=None)
        ddp = DistributedDataParallel(m, bucket_cap_mb=0.05)
        assert ddp.num_buckets() > 2
        g = torch.Generator().manual_seed(0)
        ids = torch.randint(0, 512, (4 * accum, 32), generator=g)
        mine = ids.view(world, -1, 32)[rank]
        micro = mine.view(accum, -1, 32)
        for j in range(accum):
            with ddp.no_sync(j < accum - 1):
                loss = m(micro[j], labels=micro[j])["loss"] / accum
                loss.backward()
        ddp.finish_gradient_sync()
        grads = {n: (p.grad / world).numpy().copy() for n, p in m.named_parameters()}
        params = {n: p.detach().numpy().copy() for n, p in m.named_parameters()}
        q.put((rank, grads, params))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("accum", [1, 2])
def test_ddp_matches_single_process(accum):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, accum)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, g, prm = q.get(timeout=300)
        res[r] = ({k: torch.from_numpy(v) for k, v in g.items()}, {k: torch.from_numpy(v) for k, v in prm.items()})
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g0, p0 = res[0]
    g1, p1 = res[1]
    for n in g0:
        assert torch.equal(p0[n], p1[n]), f"param {n} not broadcast"
        assert torch.allclose(g0[n], g1[n], atol=1e-7), f"grad {n} differs across ranks"
    # single process, global batch, same (broadcast) weights
    from gke_ray_train_amd.models import build_llama
    m = build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=None)
    m.load_state_dict(p0)
    gen = torch.Generator().manual_seed(0)
    ids = torch.randint(0, 512, (4 * accum, 32), generator=gen)
    # per-rank losses are means over equal-size micro-batches -> global mean of micro means
    micro = ids.view(world * accum, -1, 32)
    for j in range(world * accum):
        (m(micro[j], labels=micro[j])["loss"] / (world * accum)).backward()
    for n, p in m.named_parameters():
        assert torch.allclose(p.grad, g0[n], atol=1e-5, rtol=1e-4), f"{n}: max {(p.grad - g0[n]).abs().max()}"


def _zero_worker(rank, world, port, q, zero, tensor_coll=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if tensor_coll:  # the RCCL code path (reduce_scatter_tensor / all_gather_into_tensor) over gloo
        os.environ["GRT_GLOO_TENSOR_COLLECTIVES"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gke_ray_train_amd.models import build_llama
        from gke_ray_train_amd.ops import FusedAdamW
        from gke_ray_train_amd.parallel import DistributedDataParallel
        m = build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=3)
        ddp = DistributedDataParallel(m, bucket_cap_mb=0.1, shard_optimizer=zero)
        assert ddp.zero == zero
        # ZeRO marks the projection weights for the forward-time W^T (TN dX GEMM on GPU)
        from gke_ray_train_amd.ops.linear import Linear
        marked = [getattr(mm.weight, "_grt_fwd_transpose", False) for mm in m.modules() if isinstance(mm, Linear)]
        assert marked and all(x == zero for x in marked)
        opt = FusedAdamW(ddp.optimizer_param_groups(0.1), lr=3e-3)
        if zero:  # the optimizer holds only this rank's shard
            n_opt = sum(p.numel() for gp in opt.param_groups for p in gp["params"])
            assert n_opt * world <= sum(g.flat.numel() for g in ddp.groups) + 1
        g = torch.Generator().manual_seed(1)
        norms = []
        for step in range(3):
            ids = torch.randint(0, 512, (world * 2, 32), generator=g).view(world, 2, 32)[rank]
            loss = ddp(ids, labels=ids)["loss"]
            loss.backward()
            ddp.finish_gradient_sync()
            st = ddp.clip_grad_norm_(0.5)
            norms.append(float(st.buf[0]))
            opt.step(grad_scale=st)
            ddp.after_optimizer_step()
            ddp.zero_grad()
        ddp.wait_params()
        q.put((rank, {n: p.detach().numpy().copy() for n, p in m.named_parameters()}, norms))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("tensor_coll", [False, True])
def test_zero_sharded_optimizer_matches_ddp(tensor_coll):
    """ZeRO-1/2 mode (reduce-scatter + sharded AdamW + async all-gather) == plain DDP, 3 steps.
    tensor_coll=True runs the exact collective calls of the RCCL path (reduce_scatter_tensor into
    the shard views, all_gather_into_tensor into the flat buckets) over gloo."""
    world = 2
    ctx = mp.get_context("spawn")
    out = {}
    for zero in (False, True):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_zero_worker, args=(r, world, port, q, zero, tensor_coll)) for r in range(world)]
        for p in procs:
            p.start()
        res = {}
        for _ in range(world):
            r, prm, norms = q.get(timeout=300)
            res[r] = (prm, norms)
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        for n in res[0][0]:
            assert (res[0][0][n] == res[1][0][n]).all(), f"zero={zero}: ranks diverged on {n}"
        out[zero] = res[0]
    (p_ref, n_ref), (p_zero, n_zero) = out[False], out[True]
    assert max(abs(a - b) for a, b in zip(n_ref, n_zero)) < 1e-4 * max(n_ref), (n_ref, n_zero)
    for n in p_ref:
        d = abs(p_ref[n] - p_zero[n]).max()
        assert d < 1e-5, f"{n}: {d}"


def test_proxy_world_lays_out_rank0_of_an_n_rank_zero_job():
    """DistributedDataParallel(proxy_world=8) on one process (no process group): buckets and ZeRO
    shards exactly as rank 0 of 8 (1/8 of the optimizer state), collectives replaced by local copies
    of rank 0's chunk; a step runs end to end (bench.py --proxy-world)."""
    import torch
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.ops import FusedAdamW
    from gke_ray_train_amd.parallel import DistributedDataParallel
    m = build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=0)
    eng = DistributedDataParallel(m, shard_optimizer=True, proxy_world=8)
    assert eng.proxy and eng.zero and eng.world_size == 8 and eng.rank == 0
    for g in eng.groups:
        assert g.shard_grad.numel() * 8 == g.grad.numel()
    opt = FusedAdamW(eng.optimizer_param_groups(0.0), lr=1e-3)
    assert sum(p.numel() for grp in opt.param_groups for p in grp["params"]) * 8 == sum(g.flat.numel() for g in eng.groups)
    ids = torch.randint(0, m.config.vocab_size, (2, 32))
    before = [g.flat.clone() for g in eng.groups]
    loss = m(ids, labels=ids)["loss"]
    loss.backward()
    eng.finish_gradient_sync()
    st = eng.clip_grad_norm_(1.0)
    opt.step(grad_scale=st)
    eng.after_optimizer_step()
    eng.wait_params()
    for g, b0 in zip(eng.groups, before):
        for b in g.buckets:
            c = (b.end - b.start) // 8
            assert not torch.equal(g.flat[b.start:b.start + c], b0[b.start:b.start + c])  # rank 0's chunk updated
            assert torch.equal(g.flat[b.start + c:b.end], b0[b.start + c:b.end])          # the rest: other ranks'
