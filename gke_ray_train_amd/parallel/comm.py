"""Communication planning for RCCL over xGMI (MI355X, single node, 8 GPUs fully connected).

Reference role: the NCCL data plane the reference gets implicitly from Ray Train's
``TorchConfig(backend="nccl")`` (ray-jobs/pytorch_llm_ray.py:362-364); SURVEY §2.5.

Topology facts used here (task statement / SURVEY §2.5): each MI355X has 7 point-to-point xGMI
links of ~153 GB/s, one to every peer. A single ring uses ONE outbound link per GPU, so a ring
all-reduce of B bytes costs ~2(p-1)/p * B / 153 GB/s; RCCL recovers the other links by running
several channels over different ring permutations, which needs messages large enough to give
every channel multi-MB chunks. Bucket sizing therefore trades:
  * per-collective fixed cost (launch + channel setup, tens of µs) -> wants FEW, LARGE buckets;
  * exposed tail: the last bucket's transfer cannot overlap backward -> wants a small last bucket.
``plan_bucket_bytes`` picks ~1/32 of the gradient bytes clamped to [32 MiB, 256 MiB] (a 7B bf16
model -> 256 MiB buckets, ~54 all-reduces/step; a 125M model -> 32 MiB), and ``RCCL_*`` knobs
are left to RCCL's own tuner unless the user sets them.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

XGMI_LINK_GBPS = 153.0
XGMI_LINKS = 7


def plan_bucket_bytes(total_grad_bytes: int, world_size: int) -> int:
    env = os.environ.get("GRT_BUCKET_MB")
    if env:
        return int(float(env) * 2 ** 20)
    if world_size <= 1:
        return max(total_grad_bytes, 1)
    lo, hi = 32 * 2 ** 20, 256 * 2 ** 20
    return int(min(hi, max(lo, total_grad_bytes // 32)))


def ring_allreduce_seconds(nbytes: float, world: int, links: int = 1, link_gbps: float = XGMI_LINK_GBPS) -> float:
    """Bandwidth-only model of a ring all-reduce over `links` concurrent xGMI links."""
    if world <= 1:
        return 0.0
    return 2.0 * (world - 1) / world * nbytes / (links * link_gbps * 1e9)


@dataclass
class Topology:
    world_size: int
    local_world_size: int
    rank: int
    local_rank: int
    backend: str

    @property
    def single_node(self) -> bool:
        return self.world_size == self.local_world_size


def topology() -> Topology:
    ws = dist.get_world_size() if dist.is_initialized() else 1
    rk = dist.get_rank() if dist.is_initialized() else 0
    lws = int(os.environ.get("LOCAL_WORLD_SIZE", ws))
    lr = int(os.environ.get("LOCAL_RANK", rk))
    be = dist.get_backend() if dist.is_initialized() else "none"
    return Topology(ws, lws, rk, lr, be)


def default_backend(use_gpu: bool) -> str:
    """torch's 'nccl' backend name IS RCCL on ROCm builds."""
    return "nccl" if use_gpu and torch.cuda.is_available() else "gloo"


def all_reduce_scalar(x: float, op=None, device=None) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device or ("cuda" if dist.get_backend() == "nccl" else "cpu"))
    dist.all_reduce(t, op=op or dist.ReduceOp.SUM)
    return float(t.item())


def small_all_reduce(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place SUM all-reduce of a small (latency-bound) tensor: over the xGMI IPC kernels
    (``parallel/ipc.py``) when the message routes there (``GRT_IPC_COLLECTIVES``: auto by size on a
    single-node RCCL group), else through the process group. Grad-norm scalars, logged losses,
    metrics and FSDP's replicated-parameter gradients go through here."""
    if t.is_cuda and t.dtype in (torch.float32, torch.bfloat16):
        from .ipc import communicator, ipc_mode, route_limit, routes
        comm = communicator(group, "default")
        if comm is not None and routes(t.numel() * t.element_size(), t.dtype, route_limit(ipc_mode(), comm.cap)):
            return comm.all_reduce(t)
    dist.all_reduce(t, group=group)
    return t
