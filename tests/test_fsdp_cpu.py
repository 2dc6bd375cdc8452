"""FSDP full-shard over gloo (world 2): gradients equal a single-process run on the global batch,
with and without activation checkpointing and gradient accumulation; optimizer step keeps ranks
consistent; meta-device init; full / sharded state dicts."""
import os
import socket

import numpy as np
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


def _worker(rank, world, port, q, ckpt, accum, tensor_coll=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if tensor_coll:  # the RCCL code path (reduce_scatter_tensor / all_gather_into_tensor) over gloo
        os.environ["GRT_GLOO_TENSOR_COLLECTIVES"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gke_ray_train_amd.models import build_llama
        from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel
        from gke_ray_train_amd.ops import FusedAdamW
        m = build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=5)
        if ckpt:
            m.gradient_checkpointing_enable()
        f = FullyShardedDataParallel(m)
        opt = FusedAdamW(f.optimizer_param_groups(0.01), lr=1e-3)
        g = torch.Generator().manual_seed(0)
        ids = torch.randint(0, 512, (4 * accum, 32), generator=g)
        micro = ids.view(world, -1, 32)[rank].view(accum, -1, 32)
        for j in range(accum):
            with f.no_sync(j < accum - 1):
                loss = f(micro[j], labels=micro[j])["loss"] / accum
                loss.backward()
        f.finish_gradient_sync()
        grads = {k: (v / world).numpy().copy() for k, v in f.full_grad_dict().items()}
        st = f.clip_grad_norm_(1.0)
        opt.step(grad_scale=st)
        f.zero_grad()
        sd = {k: v.numpy().copy() for k, v in f.full_state_dict().items()}
        q.put((rank, grads, sd, float(st.buf[0])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ckpt,accum,tensor_coll", [(False, 1, False), (True, 2, False), (True, 2, True)])
def test_fsdp_matches_single_process(ckpt, accum, tensor_coll):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, ckpt, accum, tensor_coll)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, g, sd, norm = q.get(timeout=300)
        res[r] = (g, sd, norm)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    g0, sd0, n0 = res[0]
    g1, sd1, n1 = res[1]
    for k in sd0:
        assert np.array_equal(sd0[k], sd1[k]), f"{k} diverged across ranks"
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.ops import FusedAdamW, clip_grad_norm_
    m = build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=5)
    gen = torch.Generator().manual_seed(0)
    ids = torch.randint(0, 512, (4 * accum, 32), generator=gen)
    micro = ids.view(world * accum, -1, 32)
    for j in range(world * accum):
        (m(micro[j], labels=micro[j])["loss"] / (world * accum)).backward()
    for n, p in m.named_parameters():
        assert np.allclose(p.grad.numpy(), g0[n], atol=2e-5, rtol=1e-4), f"{n}"
    ref_norm = torch.sqrt(sum(p.grad.pow(2).sum() for p in m.parameters())).item()
    assert abs(ref_norm - n0) < 1e-4 * max(1, ref_norm)


def test_fsdp_world1_meta_init_and_step():
    from gke_ray_train_amd.models.llama import LlamaForCausalLM, RMSNorm, get_config
    from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel
    from gke_ray_train_amd.ops import FusedAdamW
    cfg = get_config("llama-tiny")
    m = LlamaForCausalLM(cfg, device="meta", dtype=torch.float32)

    def init(mod):
        with torch.no_grad():
            if isinstance(mod, (torch.nn.Linear, torch.nn.Embedding)):
                mod.weight.normal_(0, 0.02)
            elif isinstance(mod, RMSNorm):
                mod.weight.fill_(1.0)
    f = FullyShardedDataParallel(m, param_init_fn=init, device="cpu")
    opt = FusedAdamW(f.optimizer_param_groups(0.0), lr=1e-2)
    ids = torch.randint(0, 512, (2, 16))
    losses = []
    for _ in range(3):
        loss = f(ids, labels=ids)["loss"]
        loss.backward()
        f.finish_gradient_sync()
        opt.step(grad_scale=f.clip_grad_norm_(1.0))
        f.zero_grad()
        losses.append(loss.item())
    assert losses[-1] < losses[0]
    sd = f.full_state_dict()
    assert sd["model.layers.0.self_attn.qkv_proj.weight"].shape == (768, 256)
    zero = {k: torch.zeros_like(v) for k, v in sd.items()}
    f.load_full_state_dict(zero)
    assert all(v.abs().sum() == 0 for v in f.full_state_dict().values())
    f.load_full_state_dict(sd)
    assert all(torch.equal(sd[k], v) for k, v in f.full_state_dict().items())


def _ckpt_worker(rank, world, port, path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gke_ray_train_amd.models import build_llama
        from gke_ray_train_amd.ops import FusedAdamW
        from gke_ray_train_amd.parallel.checkpoint import AsyncCheckpointer, load_fsdp_sharded, save_fsdp_sharded
        from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel
        m = build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=5)
        f = FullyShardedDataParallel(m)
        opt = FusedAdamW(f.optimizer_param_groups(0.0), lr=1e-3)
        ids = torch.randint(0, 512, (2, 16), generator=torch.Generator().manual_seed(rank))
        loss = f(ids, labels=ids)["loss"]
        loss.backward()
        f.finish_gradient_sync()
        opt.step(grad_scale=f.clip_grad_norm_(1.0))
        f.zero_grad()
        save_fsdp_sharded(f, path, optimizer=opt, async_ckpt=AsyncCheckpointer())
        full = {k: v.numpy().copy() for k, v in f.full_state_dict().items()}
        # reload into a fresh engine of the same world size (own shard files + optimizer state)
        m2 = build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=99)
        f2 = FullyShardedDataParallel(m2)
        opt2 = FusedAdamW(f2.optimizer_param_groups(0.0), lr=1e-3)
        load_fsdp_sharded(f2, path, optimizer=opt2)
        same = all(np.array_equal(full[k], v.numpy()) for k, v in f2.full_state_dict().items())
        st1 = opt.state[opt.param_groups[0]["params"][0]]["exp_avg"]
        st2 = opt2.state[opt2.param_groups[0]["params"][0]]["exp_avg"]
        q.put((rank, full, same and torch.equal(st1, st2)))
    finally:
        dist.destroy_process_group()


def test_fsdp_sharded_checkpoint_roundtrip_consolidate_and_reshard(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    path = str(tmp_path / "ckpt")
    ps = [ctx.Process(target=_ckpt_worker, args=(r, world, port, path, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, full, ok = q.get(timeout=300)
        res[r] = (full, ok)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] and res[1][1], "same-world reload (params + optimizer state) mismatch"
    import os as _os
    assert sorted(_os.listdir(path)) == ["fsdp_layout.json", "optim-00000-of-00002.safetensors",
                                         "optim-00001-of-00002.safetensors", "shard-00000-of-00002.safetensors",
                                         "shard-00001-of-00002.safetensors"]
    from gke_ray_train_amd.parallel.checkpoint import consolidate_fsdp_checkpoint, export_hf, load_fsdp_sharded
    full = consolidate_fsdp_checkpoint(path)
    for k, v in res[0][0].items():
        assert np.array_equal(full[k].numpy(), v), k
    # resharding: world-size-1 engine loads the 2-rank checkpoint
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel
    f1 = FullyShardedDataParallel(build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=1))
    load_fsdp_sharded(f1, path)
    for k, v in f1.full_state_dict().items():
        assert np.array_equal(v.numpy(), res[0][0][k]), k
    # HF export loads back through from_pretrained
    out = export_hf(path, str(tmp_path / "hf"), dtype=torch.float32)
    from gke_ray_train_amd.models.hub import from_pretrained
    m = from_pretrained(out, device="cpu", torch_dtype=torch.float32)
    sd = m.state_dict()
    for k, v in res[0][0].items():
        assert np.array_equal(sd[k].numpy(), v), k


def test_fsdp_proxy_world_lays_out_rank0_of_n():
    """FullyShardedDataParallel(proxy_world=4) on one process (no process group): every unit holds
    1/4 of its flat parameters (rank 0's shard), gathers / reduce-scatters run as local copies of
    rank 0's part, and a full step (with accumulation and the optimizer on the shards) runs
    (bench.py --parallel fsdp --proxy-world N)."""
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.ops import FusedAdamW
    from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel
    m = build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=5)
    n_total = sum(p.numel() for p in m.parameters() if p.dim() >= 2)
    f = FullyShardedDataParallel(m, proxy_world=4)
    assert f.proxy and f.world == 4 and f.rank == 0 and f.comm
    assert all(u.total == 4 * u.shard_numel for u in f.units)
    assert f.shard_store.numel() * 4 >= n_total and f.shard_store.numel() * 4 < n_total + 4 * 4096 * len(f.units)
    opt = FusedAdamW(f.optimizer_param_groups(0.01), lr=1e-3)
    assert sum(p.numel() for g in opt.param_groups for p in g["params"]) <= f.shard_store.numel() + f.rep_flat.numel()
    ids = torch.randint(0, 512, (4, 32))
    before = f.shard_store.clone()
    for j in range(2):
        with f.no_sync(j < 1):
            f(ids[2 * j:2 * j + 2], labels=ids[2 * j:2 * j + 2])["loss"].backward()
    f.finish_gradient_sync()
    assert f.grad_store.abs().sum() > 0  # rank 0's chunk of the (local) gradient arrived
    st = f.clip_grad_norm_(1.0)
    opt.step(grad_scale=st)
    f.zero_grad()
    assert not torch.equal(before, f.shard_store)
    # units are resharded after their forward / backward: no full buffer stays bound
    assert all(u.full is None for u in f.units if u.module is not f.module)
