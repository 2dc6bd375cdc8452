"""Data-parallel engine: flat-buffer DDP with bucketed, backward-overlapped RCCL all-reduce.

Reference role: ``train.torch.prepare_model`` -> ``torch.nn.parallel.DistributedDataParallel``
over NCCL (reference ray-jobs/pytorch_llm_ray.py:230,362-364) and Accelerate's DDP wrap inside
``SFTTrainer.train()`` (ray-jobs/fine_tune_llama_ray.py:333); SURVEY §2.4 / §2.7 C02-C04.

MI355X design (not a translation of torch's C++ Reducer):
* every trainable parameter becomes a VIEW into one flat buffer per (dtype, decay-group), laid
  out in REVERSE registration order — the order gradients become ready in backward — so each
  bucket is a contiguous slice of the flat gradient buffer: the all-reduce runs on the gradient
  memory itself (no bucket pack/unpack copies, no gradient copies at all);
* gradient averaging is folded into the optimizer (SUM all-reduce, 1/world applied by the clip
  coefficient inside the fused AdamW pass) instead of a separate scaling kernel per bucket;
* buckets are sized by ``comm.plan_bucket_bytes`` for xGMI (fully connected, 7 links/GPU):
  large enough that RCCL runs at its multi-ring bandwidth, small enough that only the final
  bucket's transfer is exposed after the last backward kernel;
* buffers are not re-broadcast every step (the reference BasicLLM paid an 8 MiB PE-buffer
  broadcast per forward); parameters are broadcast once at construction;
* ``no_sync()`` for gradient accumulation (GRADIENT_ACCUMULATION_STEPS, fine_tune_config.json:14).
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops.linear import GradSlot, Linear as _DirectLinear
from .comm import plan_bucket_bytes


def _no_decay(name: str, p: torch.Tensor) -> bool:
    # HF Trainer's rule: biases and normalisation weights are excluded from weight decay
    n = name.lower()
    return p.dim() < 2 or n.endswith(".bias") or "norm" in n


@dataclass
class _Bucket:
    start: int
    end: int
    params: List[nn.Parameter] = field(default_factory=list)
    ready: int = 0
    work: Optional[object] = None


@dataclass
class _FlatGroup:
    dtype: torch.dtype
    decay: bool
    params: List[nn.Parameter]
    names: List[str]
    flat: torch.Tensor
    grad: torch.Tensor
    offsets: List[int]
    buckets: List[_Bucket]


class DistributedDataParallel(nn.Module):
    """nn.Module wrapper like torch DDP (``.module``, ``module.``-prefixed state_dict); the wrapped
    module's parameters become views into flat buffers and stay usable by any optimizer.

    The reference reads ``model.module.state_dict()`` (ray-jobs/pytorch_llm_ray.py:301), which
    breaks on one GPU because Ray's prepare_model does not wrap then; this wrapper is applied at
    every world size so that access always works.
    """

    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: Optional[float] = None,
                 broadcast_params: bool = True, grad_dtype: Optional[torch.dtype] = None,
                 split_decay: bool = True):
        super().__init__()
        self.module = module
        self.pg = process_group
        self.world_size = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if self.world_size > 1 else 0
        self._sync = True
        self._hooks = []
        self._grad_view = {}
        self._bucket_of = {}
        # weights whose backward GEMM writes straight into the flat gradient buffer
        self._direct = set()
        for m in module.modules():
            if isinstance(m, _DirectLinear) and m.weight.requires_grad:
                self._direct.add(id(m.weight))
        lm_head = getattr(module, "lm_head", None)
        if isinstance(lm_head, nn.Linear) and lm_head.weight.requires_grad:
            self._direct.add(id(lm_head.weight))
        named = []
        seen = set()
        for n, p in module.named_parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                named.append((n, p))
        total_bytes = sum(p.numel() * p.element_size() for _, p in named)
        self.bucket_bytes = int(bucket_cap_mb * 2 ** 20) if bucket_cap_mb else plan_bucket_bytes(total_bytes, self.world_size)
        # group by (dtype, decay), reverse registration order inside each group
        groups: Dict[tuple, List[tuple]] = {}
        for n, p in named:
            key = (p.dtype, (not _no_decay(n, p)) if split_decay else True)
            groups.setdefault(key, []).append((n, p))
        self.groups: List[_FlatGroup] = []
        for (dtype, decay), items in groups.items():
            items = list(reversed(items))
            self.groups.append(self._flatten(items, dtype, decay, grad_dtype or dtype))
        if broadcast_params and self.world_size > 1:
            with torch.no_grad():
                for g in self.groups:
                    dist.broadcast(g.flat, src=dist.get_global_rank(process_group, 0) if process_group else 0,
                                   group=process_group)
        # every parameter owns a GradSlot (its view into the flat gradient buffer + a "fresh"
        # flag); weights of ops.Linear / the LM head are additionally written in place by their
        # backward GEMM. zero_grad() only flips flags: no memset of the gradient buffer.
        self._slots = {}
        for g in self.groups:
            for b in g.buckets:
                for p in b.params:
                    self._bucket_of[p] = (g, b)
                    sl = GradSlot(self._grad_view[p], self._notify)
                    self._slots[p] = sl
                    if id(p) in self._direct:
                        p._grt_slot = sl
        self._register_hooks()

    # ------------------------------------------------------------------ layout
    def _flatten(self, items, dtype, decay, grad_dtype) -> _FlatGroup:
        align = 64  # elements: keeps every view 128-byte aligned for 16-byte vector kernels
        offsets, off = [], 0
        for _, p in items:
            offsets.append(off)
            off += (p.numel() + align - 1) // align * align
        dev = items[0][1].device
        flat = torch.zeros(off, dtype=dtype, device=dev)
        grad = torch.zeros(off, dtype=grad_dtype, device=dev)
        params = []
        with torch.no_grad():
            for (n, p), o in zip(items, offsets):
                flat[o:o + p.numel()].copy_(p.data.view(-1))
                p.data = flat[o:o + p.numel()].view_as(p)
                p.grad = grad[o:o + p.numel()].view_as(p)
                self._grad_view[p] = p.grad
                params.append(p)
        # buckets over the contiguous reverse-order layout
        buckets: List[_Bucket] = []
        elt = torch.tensor([], dtype=grad_dtype).element_size()
        cur = None
        for p, o in zip(params, offsets):
            n_el = (p.numel() + align - 1) // align * align
            if cur is None or (cur.end - cur.start) * elt >= self.bucket_bytes:
                cur = _Bucket(start=o, end=o)
                buckets.append(cur)
            cur.params.append(p)
            cur.end = o + n_el
        return _FlatGroup(dtype, decay, params, [n for n, _ in items], flat, grad, offsets, buckets)

    def _register_hooks(self):
        for g in self.groups:
            for b in g.buckets:
                for p in b.params:
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(g, b)))

    def _make_hook(self, g: _FlatGroup, b: _Bucket):
        def hook(p):
            # AccumulateGrad path (params not written by a direct-grad GEMM, or CPU fallbacks)
            sl = self._slots[p]
            if sl.consume_direct():  # the GEMM already wrote and announced this gradient
                return
            view = sl.view
            if p.grad is not view and p.grad.data_ptr() != view.data_ptr():
                with torch.no_grad():
                    if sl.fresh:
                        view.copy_(p.grad)
                    else:
                        view.add_(p.grad)
                p.grad = view
            sl.fresh = False
            self._mark_ready(g, b)
        return hook

    def _notify(self, p):
        p.grad = self._slots[p].view
        g, b = self._bucket_of[p]
        self._mark_ready(g, b)

    def _mark_ready(self, g, b):
        if not self._sync or self.world_size == 1:
            return
        b.ready += 1
        if b.ready > len(b.params):  # a parameter announced twice would launch a bucket early
            raise RuntimeError("DDP bucket readiness over-counted (gradient announced twice)")
        if b.ready == len(b.params):
            self._launch(g, b)

    def _launch(self, g: _FlatGroup, b: _Bucket):
        if b.work is None:
            b.work = dist.all_reduce(g.grad[b.start:b.end], op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    # ------------------------------------------------------------------ public API
    @contextlib.contextmanager
    def no_sync(self, enabled: bool = True):
        prev = self._sync
        self._sync = not enabled
        try:
            yield
        finally:
            self._sync = prev

    def finish_gradient_sync(self):
        """Wait for every bucket's all-reduce (launching any whose params got no gradient)."""
        stale = [p for p, sl in self._slots.items() if sl.fresh]
        if stale:  # parameters that got no gradient this step: their slots hold last step's data
            torch._foreach_zero_([self._slots[p].view for p in stale])
            for p in stale:
                self._slots[p].fresh = False
                p.grad = self._slots[p].view
        if self.world_size == 1:
            return
        for g in self.groups:
            for b in g.buckets:
                if b.work is None:
                    self._launch(g, b)
        for g in self.groups:
            for b in g.buckets:
                b.work.wait()
                b.work = None
                b.ready = 0

    def grad_buffers(self) -> List[torch.Tensor]:
        return [g.grad for g in self.groups]

    def zero_grad(self, set_to_none: bool = True):
        """Mark every gradient slot fresh: the next write overwrites (GEMM beta = 0 / copy)."""
        for p, sl in self._slots.items():
            sl.fresh = True
            p.grad = None

    def optimizer_param_groups(self, weight_decay: float = 0.0):
        """One flat Parameter per (dtype, decay) group; its .grad is the flat gradient buffer."""
        out = []
        for g in self.groups:
            fp = nn.Parameter(g.flat, requires_grad=False)
            fp.grad = g.grad
            out.append({"params": [fp], "weight_decay": weight_decay if g.decay else 0.0})
        return out

    def num_buckets(self) -> int:
        return sum(len(g.buckets) for g in self.groups)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            return getattr(self.module, name)

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
