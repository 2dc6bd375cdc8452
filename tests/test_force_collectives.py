"""Forced-collective rehearsal at world size 1.

``force_collectives=True`` (``GRT_FORCE_COLLECTIVES=1``) makes the DDP/ZeRO and FSDP engines issue
the multi-rank collectives — ``reduce_scatter_tensor`` into the flat-buffer shard views, async
``Work.wait()`` from autograd hooks, ``all_gather_into_tensor`` waited by forward pre-hooks, the
per-unit FSDP gathers into pooled buffers — on a one-rank process group. A sum over one rank is a
copy, so the parameters after 3 optimizer steps must be BIT-IDENTICAL to the engine's
no-collective one-GPU path. The CPU variant runs it over gloo's tensor collectives; the GPU
variant over RCCL (``nccl``), so a one-GPU box executes the exact calls an 8-GPU node issues.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train(kind, force, dev, dtype, steps=3):
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.ops import FusedAdamW
    from gke_ray_train_amd.parallel import DistributedDataParallel
    from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel
    model = build_llama("llama-tiny-gqa", device=dev, dtype=dtype, seed=11)
    if kind == "fsdp":
        eng = FullyShardedDataParallel(model, force_collectives=force)
        opt = eng.build_optimizer(lr=1e-3)
        assert eng.comm == force
    else:
        eng = DistributedDataParallel(model, shard_optimizer=True, force_collectives=force, bucket_cap_mb=1.0)
        opt = FusedAdamW(eng.optimizer_param_groups(weight_decay=0.0), lr=1e-3)
        assert eng.zero == force and eng.num_buckets() > 1
    g = torch.Generator(device=dev).manual_seed(3)
    losses = []
    for _ in range(steps):
        ids = torch.randint(0, model.config.vocab_size, (2, 128), device=dev, generator=g)
        loss = eng(ids, labels=ids)["loss"]
        loss.backward()
        eng.finish_gradient_sync()
        st = eng.clip_grad_norm_(1e9)  # no clipping: the coefficient is exactly 1 on both paths
        opt.step(grad_scale=st)
        if kind == "ddp":
            eng.after_optimizer_step()
        eng.zero_grad()
        losses.append(float(loss.detach()))
    if kind == "ddp":
        eng.wait_params()
        sd = {k: v.detach().float().cpu().clone() for k, v in model.state_dict().items()}
        eng.remove_hooks()
    else:
        sd = {k: v.float().cpu() for k, v in eng.full_state_dict().items()}
    return losses, sd


def _run(kind, backend, dev, dtype, monkeypatch):
    monkeypatch.setenv("GRT_ZERO_FWD_TRANSPOSE", "0")  # same dX GEMM form on both paths
    if backend == "gloo":
        monkeypatch.setenv("GRT_GLOO_TENSOR_COLLECTIVES", "1")
    kw = {"device_id": dev} if backend == "nccl" else {}
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, **kw)
    try:
        l_ref, sd_ref = _train(kind, False, dev, dtype)
        l_col, sd_col = _train(kind, True, dev, dtype)
    finally:
        dist.destroy_process_group()
    assert l_ref == l_col, (l_ref, l_col)
    assert sd_ref.keys() == sd_col.keys()
    for k in sd_ref:
        assert torch.equal(sd_ref[k], sd_col[k]), k


@pytest.mark.parametrize("kind", ["ddp", "fsdp"])
def test_force_collectives_cpu_gloo(kind, monkeypatch):
    _run(kind, "gloo", torch.device("cpu"), torch.float32, monkeypatch)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["ddp", "fsdp"])
def test_force_collectives_gpu_rccl(kind, monkeypatch):
    """The RCCL data plane on hardware: reduce-scatter / all-gather into flat-buffer views."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    _run(kind, "nccl", dev, torch.bfloat16, monkeypatch)
