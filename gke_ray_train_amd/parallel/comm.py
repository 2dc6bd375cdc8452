"""Communication planning for RCCL over xGMI (MI355X, single node, 8 GPUs fully connected).

Reference role: the NCCL data plane the reference gets implicitly from Ray Train's
``TorchConfig(backend="nccl")`` (ray-jobs/pytorch_llm_ray.py:362-364); SURVEY §2.5.

Topology facts used here (task statement / SURVEY §2.5): each MI355X has 7 point-to-point xGMI
links of ~153 GB/s, one to every peer. A single ring uses ONE outbound link per GPU, so a ring
all-reduce of B bytes costs ~2(p-1)/p * B / 153 GB/s; RCCL recovers the other links by running
several channels over different ring permutations, which needs messages large enough to give
every channel multi-MB chunks. Bucket sizing therefore trades:
  * per-collective fixed cost alpha (launch + channel setup, tens of µs) -> wants FEW, LARGE buckets;
  * exposed tail: the last bucket's transfer b / beta cannot overlap backward -> wants a SMALL last
    bucket.
``plan_bucket_bytes`` minimises (G / b) alpha + b / beta over the bucket size b for G gradient
bytes: b* = sqrt(G alpha beta), clamped to [16 MiB, 1 GiB]. alpha / beta per collective come from a
calibration file measured on the node (``tools/rccl_calibrate.py`` under torchrun writes it;
``GRT_COMM_CALIBRATION=<path>``), else from the xGMI prior below (not a measurement). ``RCCL_*``
knobs are left to RCCL's own tuner unless the user sets them.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

XGMI_LINK_GBPS = 153.0
XGMI_LINKS = 7


# Prior for 8 MI355X over xGMI when no calibration file is given: ~30 µs per collective, bus
# bandwidth ~ 7 links x ~50 GB/s of usable ring throughput. Algorithm bandwidth = bytes of the
# collective's input per second: all-reduce busbw * W / (2 (W - 1)), reduce-scatter / all-gather
# busbw * W / (W - 1).
PRIOR_ALPHA_US = 30.0
PRIOR_BUSBW_GBPS = 350.0


def _prior(op: str, world: int) -> dict:
    w = max(world, 2)
    scale = w / (2.0 * (w - 1)) if op == "all_reduce" else w / (w - 1.0)
    return {"alpha_us": PRIOR_ALPHA_US, "beta_GBps": PRIOR_BUSBW_GBPS * scale, "source": "prior"}


def comm_model(op: str, world: int) -> dict:
    """alpha (µs) / beta (GB/s of collective input) for ``op`` at ``world`` ranks from the
    calibration file — a single measurement (``{"world": W, op: {...}}``) or several
    (``{"by_world": {"2": {...}, "8": {...}}}``). An entry measured at another world size is used
    only after rescaling its algorithm bandwidth by the ring factor (bus bandwidth is what carries
    over between world sizes); with no usable entry, the prior."""
    path = os.environ.get("GRT_COMM_CALIBRATION")
    if path and os.path.exists(path):
        import json
        with open(path) as f:
            cal = json.load(f)
        tables = {int(k): v for k, v in cal.get("by_world", {}).items()}
        if not tables and cal.get("world") is not None:
            tables = {int(cal["world"]): cal}
        usable = {w: t[op] for w, t in tables.items() if t.get(op, {}).get("beta_GBps", 0) > 0}
        if usable:
            w_cal = min(usable, key=lambda w: (abs(w - world), -w))
            ent = usable[w_cal]
            beta = float(ent["beta_GBps"])
            if w_cal != world:  # algbw -> busbw at the measured size -> algbw at this size
                beta *= _prior(op, world)["beta_GBps"] / _prior(op, w_cal)["beta_GBps"]
            return {"alpha_us": float(ent["alpha_us"]), "beta_GBps": beta, "source": path, "world": w_cal}
    return _prior(op, world)


def plan_bucket_bytes(total_grad_bytes: int, world_size: int, op: str = "all_reduce") -> int:
    env = os.environ.get("GRT_BUCKET_MB")
    if env:
        return int(float(env) * 2 ** 20)
    if world_size <= 1:
        return max(total_grad_bytes, 1)
    m = comm_model(op, world_size)
    best = (float(total_grad_bytes) * m["alpha_us"] * 1e-6 * m["beta_GBps"] * 1e9) ** 0.5
    lo, hi = 16 * 2 ** 20, 2 ** 30
    b = min(hi, max(lo, best))
    return int(b // (8 * 2 ** 20) * (8 * 2 ** 20)) if b >= 8 * 2 ** 20 else int(b)


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
