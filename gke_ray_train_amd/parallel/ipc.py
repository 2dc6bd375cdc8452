"""xGMI peer-to-peer collectives: one-shot / two-shot all-reduce and a device barrier.

Reference role: the reference's small NCCL collectives — HF Trainer's loss all-gather every
``logging_steps``, eval-loss gathers (C06), barriers (C07) — and the grad-norm
reduction of ``clip_grad_norm_`` under DDP (ray-jobs/fine_tune_llama_ray.py:305,333). All are
latency-bound: bytes to a few MB, where RCCL's ring/channel setup costs more than the transfer.

MI355X design (SURVEY §2.5 plan item 2): every GPU of the node has a direct xGMI link to each
peer, so a one-shot all-reduce in which each GPU READS its peers' staging buffers (mapped into
its address space once through HIP IPC handles, exchanged over the process group at
construction) moves every byte in one hop over all 7 links at once. Medium messages use the
two-shot form (reduce 1/W of the message per rank, then gather), which reads each byte over the
fabric W times less. Kernels: ``csrc/kernels/ipc_comm.hip`` (system-scope release/acquire flags in
fine-grained memory, wall-clock-bounded waits that record an error instead of hanging).

Usage::

    comm = IpcCommunicator(group)          # collective: every rank of the group
    comm.all_reduce(t)                     # in place, SUM (or average=True), on the current stream
    comm.barrier()
    comm.check()                           # raises if a peer timed out in any earlier call

Constraints: ranks of one node only (IPC), world <= 8, calls issued in the same order on every
rank and ordered on the device (the current stream), message <= ``max_bytes`` and a multiple of
16 bytes (``all_reduce`` pads through a scratch tensor when it is not).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import _native

REALTIME_HZ = 100_000_000  # s_memrealtime tick rate


class IpcCommunicator:
    def __init__(self, group=None, max_bytes: int = 8 << 20, device: Optional[torch.device] = None,
                 timeout_s: float = 30.0, two_shot_bytes: Optional[int] = None):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("IpcCommunicator needs an initialised process group")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        C = _native.kernels()
        if self.world > C.IPC_MAX_RANKS:
            raise ValueError(f"IPC collectives cover one node (<= {C.IPC_MAX_RANKS} ranks), got {self.world}")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.cap = (int(max_bytes) + 15) // 16 * 16
        # two-shot pays once each GPU would otherwise read (W-1) x the message over the fabric
        self.two_shot_bytes = int(two_shot_bytes) if two_shot_bytes is not None else (
            512 << 10 if self.world > 2 else 1 << 62)
        self.timeout_ticks = int(timeout_s * REALTIME_HZ)
        self._C = C
        self.epoch = 0
        # own buffers: staging + result (2 parities each) in HBM, signals in fine-grained memory
        self._own = [C.ipc_alloc(2 * self.cap, False, self.dev_index),
                     C.ipc_alloc(2 * self.cap, False, self.dev_index),
                     C.ipc_alloc(C.IPC_SIGNAL_BYTES, True, self.dev_index)]
        self.err = torch.zeros(4, dtype=torch.int32, device=self.device)
        handles = [C.ipc_handle(p, self.dev_index) for p in self._own]
        gathered: List[Optional[list]] = [None] * self.world
        dist.all_gather_object(gathered, [os.getpid(), handles], group=group)
        self._opened = []
        ptrs = [[0] * self.world for _ in range(3)]
        for r, (_pid, hs) in enumerate(gathered):
            for k in range(3):
                if r == self.rank:
                    ptrs[k][r] = self._own[k]
                else:
                    p = C.ipc_open(hs[k], self.dev_index)
                    self._opened.append(p)
                    ptrs[k][r] = p
        self.staging, self.result, self.signal = ptrs
        dist.barrier(group=group)  # every peer has mapped every buffer before first use

    # ------------------------------------------------------------------ collectives
    def _next_epoch(self) -> int:
        self.epoch += 1
        return self.epoch & 0xFFFFFFFF

    def all_reduce(self, t: torch.Tensor, average: bool = False) -> torch.Tensor:
        """In-place SUM (or mean) of ``t`` over the group; fp32 / bf16 (fp32 accumulation)."""
        if t.dtype not in (torch.float32, torch.bfloat16):
            raise TypeError(f"ipc all_reduce supports fp32/bf16, got {t.dtype}")
        nbytes = t.numel() * t.element_size()
        if nbytes > self.cap:
            raise ValueError(f"message of {nbytes} bytes exceeds the IPC buffer ({self.cap}); use RCCL")
        scale = 1.0 / self.world if average else 1.0
        direct = t.is_contiguous() and nbytes % 16 == 0 and t.data_ptr() % 16 == 0
        if direct:
            buf = t
        else:
            per16 = 16 // t.element_size()
            buf = torch.zeros((t.numel() + per16 - 1) // per16 * per16, dtype=t.dtype, device=t.device)
            buf[:t.numel()].copy_(t.reshape(-1))
        two_shot = nbytes >= self.two_shot_bytes
        self._C.ipc_allreduce(self.staging, self.result, self.signal, self.err, self.cap, self.rank,
                              self._next_epoch(), self.timeout_ticks, buf, buf, two_shot, scale)
        if not direct:
            t.copy_(buf[:t.numel()].view_as(t))
        return t

    def barrier(self):
        """Device-side barrier on the current stream (no host synchronisation)."""
        self._C.ipc_barrier(self.staging, self.result, self.signal, self.err, self.cap, self.rank,
                            self._next_epoch(), self.timeout_ticks)

    def check(self):
        """Synchronise and raise if any earlier call timed out waiting for a peer."""
        e = int(self.err[0].item())
        if e:
            peers = [i for i in range(32) if e >> i & 1]
            raise RuntimeError(f"IPC collective timed out waiting for rank(s) {peers} (rank {self.rank})")

    def close(self):
        if self._C is None:
            return
        torch.cuda.synchronize(self.device)
        if dist.is_initialized():
            dist.barrier(group=self.group)  # no peer kernel still reads our buffers
        for p in self._opened:
            self._C.ipc_close(p, self.dev_index)
        self._opened = []
        for p in self._own:
            self._C.ipc_free(p, self.dev_index)
        self._own = []
        self._C = None


_default: Optional[IpcCommunicator] = None


def ipc_available(group=None) -> bool:
    """True when every rank of the group is a GPU process on this node and the kernels load."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_backend(group) != "nccl":
        return False
    if not torch.cuda.is_available() or not _native.kernels_available():
        return False
    world = dist.get_world_size(group)
    local = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    return 1 < world <= 8 and local == world


def default_communicator() -> Optional[IpcCommunicator]:
    """Process-wide communicator over the default group when ``GRT_IPC_COLLECTIVES=1`` and
    :func:`ipc_available`; otherwise None (callers fall back to RCCL)."""
    global _default
    if _default is None and os.environ.get("GRT_IPC_COLLECTIVES", "0") == "1" and ipc_available():
        _default = IpcCommunicator()
    return _default
