"""Ulysses sequence parallelism (parallel/sequence.py) over gloo: 2 and 4 ranks each hold S/P
tokens of the same sequences; loss and DDP-averaged gradients equal a single-process run on the
full sequences. World 4 with 2 KV heads exercises the KV-head repetition (GQA, P > Hkv)."""
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


def _ids():
    g = torch.Generator().manual_seed(0)
    return torch.randint(0, 512, (2, 64), generator=g)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GRT_GLOO_TENSOR_COLLECTIVES="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gke_ray_train_amd.models import build_llama
        from gke_ray_train_amd.parallel import DistributedDataParallel
        from gke_ray_train_amd.parallel.sequence import enable_sequence_parallel, shard_sequence
        m = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32, seed=3)
        enable_sequence_parallel(m)
        ddp = DistributedDataParallel(m)
        ids_loc, lab_loc, w = shard_sequence(_ids())
        loss = ddp(ids_loc, shifted_labels=lab_loc)["loss"] * w
        loss.backward()
        ddp.finish_gradient_sync()
        tot = loss.detach().clone()
        dist.all_reduce(tot)
        grads = {n: (p.grad / world).numpy().copy() for n, p in m.named_parameters()}
        q.put((rank, float(tot) / world, grads))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ulysses_matches_full_sequence(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, loss, grads = q.get(timeout=300)
        res[r] = (loss, grads)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    from gke_ray_train_amd.models import build_llama
    m = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32, seed=3)
    ids = _ids()
    loss = m(ids, labels=ids)["loss"]
    loss.backward()
    ref = float(loss.detach())
    assert abs(res[0][0] - ref) < 1e-5 * max(1.0, abs(ref)), (res[0][0], ref)
    for n, p in m.named_parameters():
        g = torch.from_numpy(res[0][1][n])
        assert torch.allclose(g, p.grad, atol=2e-6, rtol=1e-4), f"{n}: {(g - p.grad).abs().max()}"
