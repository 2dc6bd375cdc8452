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

The update of each bf16 projection weight (``ops.Linear`` / LM head, dims multiples of 64) also
writes W^T (``adamw_t``: one extra 2-byte write per parameter inside the HBM-bound pass) and
registers it, so the next backward's input-gradient GEMM runs in the faster TN form on it
(``ops.linear.input_grad``); ``GRT_OPT_TRANSPOSE=0`` keeps the plain update.

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
from ..ops.optim import FusedAdamW, GradClipState, bump_param_generation
from .ddp import DistributedDataParallel, forward_wait_modules


def fine_forward_wait_modules(module: nn.Module, unit_types, param_ids: set) -> Dict[nn.Module, List[int]]:
    """``forward_wait_modules`` at projection granularity: inside a transformer layer each
    ``ops.linear.Linear`` projection waits only for its OWN weight's update (its forward pre-hook),
    and the layer's other parameters (norm weights, read directly by the layer's forward) are
    waited for at the layer's entry. The next step's first layer then starts once its norm and QKV
    weights are updated instead of its whole update (the step-boundary stall of
    profiles/r6_proxy8_steps.md: embedding + whole layer-0 update ahead of the first norm).
    Opt-in (GRT_OVERLAP_FINE=1): measured 287.8 vs 287.5 ms per headline step against the layer
    granularity (3 interleaved rounds, scripts/r6/fine_ab.sh) — the earlier start of layer 0 is
    cancelled by 4x the chunk launches / events. Returned in forward order."""
    coarse = forward_wait_modules(module, unit_types, param_ids)
    if os.environ.get("GRT_OVERLAP_FINE", "0") != "1":
        return coarse
    from ..ops.linear import Linear as _DirectLinear
    out: Dict[nn.Module, List[int]] = {}
    for m, ids in coarse.items():
        if type(m).__name__ not in unit_types:
            out[m] = ids
            continue
        mine = set(ids)
        lins = []
        for sm in m.modules():
            if isinstance(sm, _DirectLinear):
                own = [id(p) for p in sm.parameters(recurse=False) if id(p) in mine]
                if own:
                    lins.append((sm, own))
        taken = {i for _, own in lins for i in own}
        rest = [i for i in ids if i not in taken]
        if rest:
            out[m] = rest  # the layer's entry: its norm weights
        for sm, own in lins:  # registration order = the layer's forward order
            out[sm] = own
    return out


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
        waits = fine_forward_wait_modules(engine.module, engine.UNIT_TYPES, set(flat_ids))
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
        # per chunk: the parameters in it, so weights with a transposed copy get their own launch
        params_of = {id(p): p for g in engine.groups for p in g.params}
        self._chunk_params: Dict[nn.Module, List[Tuple[int, int, int, torch.Tensor]]] = {}
        for m, ids in waits.items():
            self._chunk_params[m] = sorted((flat_ids[i] + (params_of[i],) for i in ids), key=lambda t: (t[0], t[1]))
        self._wt: Dict[int, torch.Tensor] = {}
        if os.environ.get("GRT_OPT_TRANSPOSE", "1") != "0" and not optimizer.master_weights:
            from ..ops.linear import _TRANSPOSED_DGRAD, Linear as _DirectLinear
            proj = {id(mm.weight) for mm in engine.module.modules() if isinstance(mm, _DirectLinear)}
            head = getattr(engine.module, "lm_head", None)
            if isinstance(head, nn.Linear):
                proj.add(id(head.weight))
            for g in engine.groups:
                for p in g.params:
                    if (_TRANSPOSED_DGRAD and id(p) in proj and p.is_cuda and p.dtype == torch.bfloat16
                            and g.grad.dtype == torch.bfloat16 and p.dim() == 2 and p.shape[0] % 64 == 0
                            and p.shape[1] % 128 == 0 and getattr(p, "_grt_slot", None) is not None):
                        self._wt[id(p)] = torch.empty(p.shape[1], p.shape[0], device=p.device, dtype=p.dtype)
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

    @staticmethod
    def _make_stream(dev):
        """The update's side stream: confined to GRT_OPT_CUS CUs (``ops/streams.py``) so the
        forward GEMMs keep the rest of the chip; 0 = an ordinary stream on every CU."""
        if os.environ.get("GRT_OVERLAP_OPT_SERIAL", "0") == "1":
            # A/B switch: the same per-module (transposing) updates, run in order on the compute
            # stream at step() instead of beside the next forward
            return torch.cuda.current_stream(dev)
        n = int(os.environ.get("GRT_OPT_CUS", "0"))
        if n > 0:
            from ..ops.streams import cu_masked_stream
            return cu_masked_stream(n, dev, os.environ.get("GRT_OPT_CU_PATTERN", "spread"))
        return torch.cuda.Stream(dev)

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
        bump_param_generation()
        groups = self.engine.groups
        dev = groups[0].flat.device
        if dev.type != "cuda":
            return self.opt.step(grad_scale=grad_scale)
        self.synchronize()  # step t-1's chunks all done before we touch shared buffers
        work = self.opt.prepare_gpu_step()
        # the update runs here, not through self.opt.step(): tell an LR scheduler bound to the inner
        # optimizer that this step happened (torch's LRScheduler reads this flag; without it every
        # scheduler.step() warns "lr_scheduler.step() before optimizer.step()")
        self.opt._opt_called = True
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
            self._stream = self._make_stream(dev)
        start = torch.cuda.Event()
        start.record(cur)
        C = _native.kernels()
        gs = None if grad_scale is None else grad_scale.buf
        if gs is not None:  # read by the chunks on the side stream: not reusable before they ran
            gs.record_stream(self._stream)
        from ..ops.linear import register_transposed
        with torch.cuda.stream(self._stream):
            self._stream.wait_event(start)
            for m, rs in self.chunks:
                if self._wt:
                    self._launch_chunk_params(C, m, per_group, gs, register_transposed)
                else:
                    for gi, lo, hi in rs:
                        p, g, ea, eas, master, hb = per_group[gi]
                        C.adamw(p.data[lo:hi], g[lo:hi], ea[lo:hi], eas[lo:hi],
                                None if master is None else master[lo:hi], hb, gs, self.max_blocks, lo)
                ev = torch.cuda.Event()
                ev.record(self._stream)
                self._events[m] = ev

    def _launch_chunk_params(self, C, m, per_group, gs, register_transposed):
        """One launch per parameter of the chunk: projection weights through the transposing
        update (W^T registered for the next backward), runs of the others through the flat one."""
        run = None  # (gi, lo, hi) of consecutive plain parameters

        def flush():
            if run is not None:
                gi, lo, hi = run
                p, g, ea, eas, master, hb = per_group[gi]
                C.adamw(p.data[lo:hi], g[lo:hi], ea[lo:hi], eas[lo:hi],
                        None if master is None else master[lo:hi], hb, gs, self.max_blocks, lo)

        for gi, off, n, prm in self._chunk_params[m]:
            wt = self._wt.get(id(prm))
            if wt is None:
                if run is not None and run[0] == gi and run[2] <= off:
                    run = (gi, run[1], off + n)
                else:
                    flush()
                    run = (gi, off, off + n)
                continue
            flush()
            run = None
            p, g, ea, eas, master, hb = per_group[gi]
            shape = prm.shape
            C.adamw_t(p.data[off:off + n].view(shape), g[off:off + n].view(shape), ea[off:off + n].view(shape),
                      eas[off:off + n].view(shape), hb, gs, wt, off)
            register_transposed(prm, wt)
        flush()

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
