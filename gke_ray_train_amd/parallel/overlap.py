"""Optimizer step overlapped with the next forward pass (1 GPU / replicated data parallel).

Reference role: ``optimizer.step()`` after the gradient sync (reference
ray-jobs/pytorch_llm_ray.py:278; HF Trainer's step inside ``trainer.train()``,
ray-jobs/fine_tune_llama_ray.py:333), SURVEY §2.6 K-A13 / K-B12.

MI355X design: the fused AdamW pass is HBM-bound (≈22 bytes per parameter: a 7B model moves
≈150 GB, ≈26 ms at the achievable ≈6 TB/s) while the forward GEMMs are MFMA-bound and leave the
memory system mostly idle. So instead of running the update as one serial kernel at the end of
the step, ``OverlappedOptimizer.step`` splits it by the module that first uses each parameter in
the next forward (embedding, each decoder layer, final norm, LM head) and launches those updates,
in forward order, on a side HIP stream; a forward pre-hook on each module makes the compute
stream wait only for ITS chunk. Layer L+1's update then runs concurrently with layer L's forward
GEMMs. Semantics are unchanged: every parameter is updated with step t's gradients and clip
coefficient before step t+1 reads it, and ``synchronize()`` (or any device synchronisation)
completes all pending updates, so a timed region that ends with ``torch.cuda.synchronize()``
contains all of the optimizer work.

Ordering hazards and why they are safe:
* the clip coefficient and gradients of step t are produced on the compute stream before the
  side stream's start event; the next backward overwrites a chunk's gradients only after that
  chunk's module ran forward, i.e. after its update completed;
* hyper-parameter buffers and the clip state are rewritten in step t+1's ``step`` only after the
  compute stream has waited for every chunk of step t (``step`` waits all pending chunks first).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from .. import _native
from ..ops.optim import FusedAdamW, GradClipState
from .ddp import DistributedDataParallel, forward_wait_modules


class OverlappedOptimizer:
    def __init__(self, engine: DistributedDataParallel, optimizer: FusedAdamW, max_blocks: Optional[int] = None):
        if engine.zero:
            raise ValueError("ZeRO mode already overlaps its parameter all-gather with the forward; "
                             "the overlapped optimizer is for replicated parameters")
        self.engine = engine
        self.opt = optimizer
        # grid cap of the update kernels (0 = full grid): a few workgroups pull a bounded share
        # of HBM bandwidth beside the forward's GEMMs instead of flooding every CU
        self.max_blocks = int(os.environ.get("GRT_OVERLAP_OPT_BLOCKS", "0")) if max_blocks is None else int(max_blocks)
        flat_ids = {}
        for gi, g in enumerate(engine.groups):
            for p, off in zip(g.params, g.offsets):
                flat_ids[id(p)] = (gi, off, p.numel())
        waits = forward_wait_modules(engine.module, engine.UNIT_TYPES, set(flat_ids))
        # chunk = one module's parameters = one contiguous range per flat group (params of a module
        # are consecutive in registration order, hence in the reversed flat layout)
        self.chunks: List[Tuple[nn.Module, List[Tuple[int, int, int]]]] = []
        for m, ids in waits.items():
            rng: Dict[int, List[int]] = {}
            for i in ids:
                gi, off, n = flat_ids[i]
                lo, hi = rng.get(gi, [off, off + n])
                rng[gi] = [min(lo, off), max(hi, off + n)]
            self.chunks.append((m, [(gi, lo, hi) for gi, (lo, hi) in sorted(rng.items())]))
        self._check_disjoint()
        self._events: Dict[nn.Module, torch.cuda.Event] = {}
        self._stream: Optional[torch.cuda.Stream] = None
        self._hooks = [m.register_forward_pre_hook(self._make_hook(m)) for m, _ in self.chunks]

    def _check_disjoint(self):
        seen: Dict[int, List[Tuple[int, int]]] = {}
        for _, rs in self.chunks:
            for gi, lo, hi in rs:
                for a, b in seen.get(gi, []):
                    if lo < b and a < hi:
                        raise RuntimeError("overlapped optimizer: module parameter ranges interleave in the "
                                           "flat buffer; use the serial optimizer step")
                seen.setdefault(gi, []).append((lo, hi))

    def _make_hook(self, m):
        def hook(mod, args):
            ev = self._events.pop(m, None)
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)
        return hook

    @property
    def param_groups(self):
        return self.opt.param_groups

    def synchronize(self):
        """Make the current stream wait for every pending chunk update."""
        cur = torch.cuda.current_stream()
        for ev in self._events.values():
            cur.wait_event(ev)
        self._events.clear()

    @torch.no_grad()
    def step(self, grad_scale: Optional[GradClipState] = None):
        groups = self.engine.groups
        dev = groups[0].flat.device
        if dev.type != "cuda":
            return self.opt.step(grad_scale=grad_scale)
        self.synchronize()  # step t-1's chunks all done before we touch shared buffers
        work = self.opt.prepare_gpu_step()
        by_flat = {w[0].data_ptr(): w for w in work}
        per_group = []
        for g in groups:
            w = by_flat.get(g.flat.data_ptr())
            if w is None:
                raise RuntimeError("overlapped optimizer: optimizer param groups must be the engine's "
                                   "flat buffers (optimizer_param_groups())")
            per_group.append(w)
        cur = torch.cuda.current_stream(dev)
        if self._stream is None:
            self._stream = torch.cuda.Stream(dev)
        start = torch.cuda.Event()
        start.record(cur)
        C = _native.kernels()
        gs = None if grad_scale is None else grad_scale.buf
        with torch.cuda.stream(self._stream):
            self._stream.wait_event(start)
            for m, rs in self.chunks:
                for gi, lo, hi in rs:
                    p, g, ea, eas, master, hb = per_group[gi]
                    C.adamw(p.data[lo:hi], g[lo:hi], ea[lo:hi], eas[lo:hi],
                            None if master is None else master[lo:hi], hb, gs, self.max_blocks, lo)
                ev = torch.cuda.Event()
                ev.record(self._stream)
                self._events[m] = ev

    def state_dict(self):
        self.synchronize()
        return self.opt.state_dict()

    def load_state_dict(self, sd):
        self.synchronize()
        self.opt.load_state_dict(sd)

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
