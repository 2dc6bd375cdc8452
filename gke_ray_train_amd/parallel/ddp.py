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
* ``no_sync()`` for gradient accumulation (GRADIENT_ACCUMULATION_STEPS, fine_tune_config.json:14);
* ``shard_optimizer=True`` (ZeRO-1/2, world > 1): each bucket is REDUCE-SCATTERED during backward
  (half the bytes of an all-reduce on the critical path) into a contiguous per-rank gradient shard,
  the fused AdamW updates only this rank's 1/world of the parameters (optimizer state and its HBM
  traffic shrink by world), and the updated shards are ALL-GATHERED back into the flat parameter
  buffer asynchronously, bucket by bucket in forward order, each bucket waited for by a forward
  pre-hook of the first module that uses it — the gather overlaps the next step's forward.
* ZeRO: projection weights get W^T written on a side stream during the forward (after their
  bucket's all-gather) for the TN input-gradient GEMM (``GRT_ZERO_FWD_TRANSPOSE=0`` = NN form);
* ``GRT_FORCE_COLLECTIVES=1`` (or ``force_collectives=True``) with an initialised process group
  runs the multi-rank code path even at world size 1 — bucket all-reduce / reduce-scatter on the
  flat-buffer views, async ``Work.wait()`` from the hooks, ZeRO all-gathers waited by forward
  pre-hooks — so a one-GPU box executes the exact RCCL calls an 8-GPU node issues;
* one GPU: the gradient-norm reduction of each bucket (sum of squares, HBM-bound) runs on a side
  stream as soon as the bucket's last gradient is written, under the remaining backward GEMMs;
  ``clip_grad_norm_`` then only combines the per-bucket partial sums (``GRT_EARLY_GRAD_NORM=0``
  computes the norm after backward instead).
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops.linear import Embedding as _DirectEmbedding, GradSlot, Linear as _DirectLinear
from .comm import plan_bucket_bytes, small_all_reduce


class _DoneWork:
    """Stand-in for a collective's Work in proxy mode (the local copy already ran in stream order)."""

    def wait(self):
        return None


class _StreamWork:
    """Work of a collective issued on a side stream (IPC kernels): wait() orders the current
    stream after it, without a host synchronisation."""

    def __init__(self, event: torch.cuda.Event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)


def shared_param_ids(module: nn.Module) -> set:
    """ids of parameters owned by more than one module (tied embeddings): their gradient has two
    producers, so they must not use the single-writer direct gradient slots."""
    seen, shared = set(), set()
    for m in module.modules():
        for p in m.parameters(recurse=False):
            (shared if id(p) in seen else seen).add(id(p))
    return shared


def forward_wait_modules(module: nn.Module, unit_types, param_ids: set) -> Dict[nn.Module, List[int]]:
    """Which module's forward pre-hook must wait for each parameter (ids in ``param_ids``) to be
    ready: the enclosing transformer layer (``unit_types``) for parameters inside one — layers read
    their norm weights directly, not through submodule calls — else the parameter's own module
    (embedding, final norm, LM head). Returned in module registration order = forward order."""
    waits: Dict[nn.Module, List[int]] = {}
    claimed = set()
    for m in module.modules():
        if type(m).__name__ in unit_types:
            for p in m.parameters():
                if id(p) in param_ids and id(p) not in claimed:
                    claimed.add(id(p))
                    waits.setdefault(m, []).append(id(p))
    for m in module.modules():
        for p in m.parameters(recurse=False):
            if id(p) in param_ids and id(p) not in claimed:
                claimed.add(id(p))
                waits.setdefault(m, []).append(id(p))
    order = {m: i for i, m in enumerate(module.modules())}
    return dict(sorted(waits.items(), key=lambda kv: order[kv[0]]))


def _no_decay(name: str, p: torch.Tensor) -> bool:
    # HF Trainer's rule: biases and normalisation weights are excluded from weight decay
    n = name.lower()
    return p.dim() < 2 or n.endswith(".bias") or "norm" in n


@dataclass
class _Bucket:
    start: int
    end: int
    params: List[nn.Parameter] = field(default_factory=list)
    ready: set = field(default_factory=set)   # ids of the parameters announced this step
    work: Optional[object] = None
    shard_off: int = 0        # ZeRO: offset of this bucket's chunk in the rank's shard buffers
    ag_work: Optional[object] = None
    norm_slot: int = -1       # one GPU: this bucket's slot in the early grad-norm workspace
    normed: bool = False      # its sum of squares was launched for the current step


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
    shard_param: Optional[torch.Tensor] = None   # ZeRO: this rank's parameter shard (contiguous)
    shard_grad: Optional[torch.Tensor] = None


class DistributedDataParallel(nn.Module):

    """nn.Module wrapper like torch DDP (``.module``, ``module.``-prefixed state_dict); the wrapped
    module's parameters become views into flat buffers and stay usable by any optimizer.

    The reference reads ``model.module.state_dict()`` (ray-jobs/pytorch_llm_ray.py:301), which
    breaks on one GPU because Ray's prepare_model does not wrap then; this wrapper is applied at
    every world size so that access always works.
    """
    UNIT_TYPES = ("LlamaDecoderLayer", "EncoderLayer")
    _ipc_engines = 0  # engines that created a bucket communicator (collective order = creation order)

    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: Optional[float] = None,
                 broadcast_params: bool = True, grad_dtype: Optional[torch.dtype] = None,
                 split_decay: bool = True, shard_optimizer: bool = False, force_collectives: Optional[bool] = None,
                 proxy_world: int = 0):
        super().__init__()
        self.module = module
        self.pg = process_group
        self.world_size = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if self.world_size > 1 else 0
        # proxy_world = N on ONE process (no process group): lay out the buckets, ZeRO shards and the
        # optimizer state exactly as rank 0 of an N-rank job and run its per-rank compute; the
        # collectives become local copies of this rank's chunk (reduce-scatter output, all-gather
        # input), i.e. the step an N-GPU run executes minus the xGMI transfers (bench.py --proxy-world).
        # Only rank 0's shard is updated, so the loss is not meaningful in this mode.
        self.proxy = int(proxy_world) > 1 and self.world_size == 1
        if self.proxy:
            self.world_size, self.rank = int(proxy_world), 0
        if force_collectives is None:
            force_collectives = os.environ.get("GRT_FORCE_COLLECTIVES", "0") == "1"
        # comm: the collective code path runs (world > 1, or forced at world 1 for rehearsal)
        self.comm = self.proxy or self.world_size > 1 or (
            bool(force_collectives) and dist.is_available() and dist.is_initialized())
        self.zero = bool(shard_optimizer) and self.comm
        # gloo branch: list-based collectives. GRT_GLOO_TENSOR_COLLECTIVES=1 runs the RCCL code path
        # (reduce_scatter_tensor / all_gather_into_tensor) over gloo so CPU tests exercise it.
        self.gloo = (self.comm and not self.proxy and dist.get_backend(process_group) == "gloo"
                     and os.environ.get("GRT_GLOO_TENSOR_COLLECTIVES", "0") != "1")
        self._sync = True
        self._hooks = []
        self._grad_view = {}
        self._bucket_of = {}
        # weights whose backward GEMM writes straight into the flat gradient buffer
        self._direct = set()
        for m in module.modules():
            if isinstance(m, (_DirectLinear, _DirectEmbedding)) and m.weight.requires_grad:
                self._direct.add(id(m.weight))
            elif getattr(m, "_grt_direct_grad", False) and m.weight.requires_grad:
                self._direct.add(id(m.weight))  # e.g. RMSNorm: the HIP backward writes the slot
            if hasattr(m, "direct_grad_params"):  # e.g. LoRA adapters (peft/lora.py)
                self._direct.update(id(p) for p in m.direct_grad_params() if p.requires_grad)
        lm_head = getattr(module, "lm_head", None)
        if isinstance(lm_head, nn.Linear) and lm_head.weight.requires_grad:
            self._direct.add(id(lm_head.weight))
        self._direct -= shared_param_ids(module)  # tied weights: two writers -> AccumulateGrad path
        named = []
        seen = set()
        for n, p in module.named_parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                named.append((n, p))
        total_bytes = sum(p.numel() * p.element_size() for _, p in named)
        dev0 = named[0][1].device if named else torch.device("cpu")
        self._early_norm = (not self.comm and dev0.type == "cuda"
                            and os.environ.get("GRT_EARLY_GRAD_NORM", "1") != "0")
        if bucket_cap_mb:
            self.bucket_bytes = int(bucket_cap_mb * 2 ** 20)
        elif self._early_norm and not os.environ.get("GRT_BUCKET_MB"):
            self.bucket_bytes = 256 * 2 ** 20  # norm granularity only: no collectives on one GPU
        else:
            self.bucket_bytes = plan_bucket_bytes(total_bytes, max(self.world_size, 2 if self.comm else 1),
                                                  "reduce_scatter" if (shard_optimizer and self.comm) else "all_reduce")
        # group by (dtype, decay), reverse registration order inside each group
        groups: Dict[tuple, List[tuple]] = {}
        for n, p in named:
            key = (p.dtype, (not _no_decay(n, p)) if split_decay else True)
            groups.setdefault(key, []).append((n, p))
        self.groups: List[_FlatGroup] = []
        for (dtype, decay), items in groups.items():
            items = list(reversed(items))
            self.groups.append(self._flatten(items, dtype, decay, grad_dtype or dtype))
        if broadcast_params and self.world_size > 1 and not self.proxy:
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
        if self.zero:
            self._setup_shards()
            if os.environ.get("GRT_ZERO_FWD_TRANSPOSE", "1") != "0":
                # the sharded AdamW cannot write W^T (a rank owns a flat slice, not whole rows), so
                # each projection weight is transposed on a side stream in the forward, right after
                # its all-gather, for the backward's TN input-gradient GEMM (ops/linear.py)
                for m in module.modules():
                    if isinstance(m, _DirectLinear) and id(m.weight) in self._direct:
                        m.weight._grt_fwd_transpose = True
        # buckets small enough for the xGMI IPC kernels (parallel/ipc.py; e.g. the no-decay group of
        # norm weights) are all-reduced by them on a side stream instead of by RCCL. The decision
        # is a function of the bucket layout only, identical on every rank.
        self._ipc = None
        self._ipc_tag = None
        self._ipc_limit = 0
        self._ipc_stream = None
        self.ipc_bucket_launches = 0  # buckets all-reduced over IPC so far (tests / logs)
        if self.comm and not self.proxy and dev0.type == "cuda":
            from .ipc import communicator, ipc_mode, route_limit, routes
            if ipc_mode() != "0" and any(
                    routes((b.end - b.start) * g.grad.element_size(), g.grad.dtype, route_limit(ipc_mode(), 8 << 20))
                    for g in self.groups for b in g.buckets):
                # one communicator per engine: its epoch sequence is driven from this engine's
                # side stream only (two engines sharing one would interleave calls across streams)
                DistributedDataParallel._ipc_engines += 1
                self._ipc_tag = f"ddp-buckets-{DistributedDataParallel._ipc_engines}"
                self._ipc = communicator(process_group, self._ipc_tag)
                if self._ipc is not None:
                    self._ipc_limit = route_limit(ipc_mode(), self._ipc.cap)
                    self._ipc_stream = torch.cuda.Stream(dev0)
        self._norm_ws = None
        self._norm_stream = None
        self._norm_bad = False  # a step whose early norm cannot be trusted (fall back)
        if self._early_norm:
            from .. import _native
            C = _native.kernels()
            nslots = 0
            for g in self.groups:
                for b in g.buckets:
                    b.norm_slot = nslots
                    nslots += 1
            self._norm_ws = torch.zeros(nslots * C.sumsq_blocks(), device=dev0, dtype=torch.float32)
            self._norm_stream = torch.cuda.Stream(dev0)

    # ------------------------------------------------------------------ layout
    def _flatten(self, items, dtype, decay, grad_dtype) -> _FlatGroup:
        align = 64  # elements: keeps every view 128-byte aligned for 16-byte vector kernels
        # ZeRO: every bucket spans a multiple of align * world so it splits into equal aligned chunks
        bucket_align = align * (self.world_size if self.zero else 1)
        elt = torch.tensor([], dtype=grad_dtype).element_size()
        offsets, spans, off, cur_start = [], [], 0, 0
        for _, p in items:
            if off > cur_start and (off - cur_start) * elt >= self.bucket_bytes:
                off = (off + bucket_align - 1) // bucket_align * bucket_align
                spans.append((cur_start, off))
                cur_start = off
            offsets.append(off)
            off += (p.numel() + align - 1) // align * align
        off = (off + bucket_align - 1) // bucket_align * bucket_align
        spans.append((cur_start, off))
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
        buckets = [_Bucket(start=a, end=b) for a, b in spans]
        bi = 0
        for p, o in zip(params, offsets):
            while o >= buckets[bi].end:
                bi += 1
            buckets[bi].params.append(p)
        buckets = [b for b in buckets if b.params]
        return _FlatGroup(dtype, decay, params, [n for n, _ in items], flat, grad, offsets, buckets)

    def _setup_shards(self):
        """ZeRO: contiguous per-rank shard buffers (bucket chunks back to back) + forward pre-hooks."""
        W, r = self.world_size, self.rank
        for g in self.groups:
            tot = 0
            for b in g.buckets:
                b.shard_off = tot
                tot += (b.end - b.start) // W
            g.shard_param = torch.empty(tot, dtype=g.flat.dtype, device=g.flat.device)
            g.shard_grad = torch.zeros(tot, dtype=g.grad.dtype, device=g.grad.device)
            with torch.no_grad():
                for b in g.buckets:
                    c = (b.end - b.start) // W
                    g.shard_param[b.shard_off:b.shard_off + c].copy_(g.flat[b.start + r * c:b.start + (r + 1) * c])
        owner = {}
        for g in self.groups:
            for b in g.buckets:
                for p in b.params:
                    owner[id(p)] = b
        for m, ps in forward_wait_modules(self.module, self.UNIT_TYPES, set(owner)).items():
            bs = {id(owner[i]): owner[i] for i in ps}
            self._hooks.append(m.register_forward_pre_hook(self._make_gather_wait(list(bs.values()))))

    @staticmethod
    def _make_gather_wait(buckets):
        def hook(mod, args):
            for b in buckets:
                if b.ag_work is not None:
                    b.ag_work.wait()
                    b.ag_work = None
        return hook

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
            self._mark_ready(g, b, p)
        return hook

    def _notify(self, p):
        p.grad = self._slots[p].view
        g, b = self._bucket_of[p]
        self._mark_ready(g, b, p)

    def _mark_ready(self, g, b, p):
        if not self._sync:
            return
        if not self.comm:
            if self._early_norm:
                if id(p) in b.ready:  # announced twice: the early norm may have read a partial bucket
                    self._norm_bad = True
                    return
                b.ready.add(id(p))
                if len(b.ready) == len(b.params):
                    self._launch_norm(g, b)
            return
        if id(p) in b.ready:  # a parameter announced twice would launch a bucket early
            raise RuntimeError("DDP bucket readiness over-counted (gradient announced twice)")
        b.ready.add(id(p))
        if len(b.ready) == len(b.params):
            self._launch(g, b)

    def _launch_norm(self, g: _FlatGroup, b: _Bucket):
        """Sum of squares of a finished bucket's gradient on the side stream (ordered after the
        kernels that wrote it)."""
        from .. import _native
        cur = torch.cuda.current_stream(g.grad.device)
        self._norm_stream.wait_stream(cur)
        with torch.cuda.stream(self._norm_stream):
            _native.kernels().sumsq(g.grad[b.start:b.end], self._norm_ws, b.norm_slot)
        b.normed = True

    def _launch(self, g: _FlatGroup, b: _Bucket):
        if b.work is not None:
            return
        if self.proxy:  # this rank's reduce-scatter output: its chunk of the bucket
            c = (b.end - b.start) // self.world_size
            if self.zero:
                g.shard_grad[b.shard_off:b.shard_off + c].copy_(g.grad[b.start + self.rank * c:b.start + (self.rank + 1) * c])
            b.work = _DoneWork()
            return
        if self._ipc is not None:
            from .ipc import routes
            view = g.grad[b.start:b.end]
            if routes(view.numel() * view.element_size(), view.dtype, self._ipc_limit):
                cur = torch.cuda.current_stream(view.device)
                self._ipc_stream.wait_stream(cur)
                with torch.cuda.stream(self._ipc_stream):
                    self._ipc.all_reduce(view)
                    if self.zero:  # all-reduce + keep our chunk = the reduce-scatter's output
                        c = (b.end - b.start) // self.world_size
                        g.shard_grad[b.shard_off:b.shard_off + c].copy_(view[self.rank * c:(self.rank + 1) * c])
                    ev = torch.cuda.Event()
                    ev.record(self._ipc_stream)
                b.work = _StreamWork(ev)
                self.ipc_bucket_launches += 1
                return
        if not self.zero or self.gloo:  # gloo has no reduce-scatter: all-reduce, keep our chunk later
            b.work = dist.all_reduce(g.grad[b.start:b.end], op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
        else:
            c = (b.end - b.start) // self.world_size
            b.work = dist.reduce_scatter_tensor(g.shard_grad[b.shard_off:b.shard_off + c], g.grad[b.start:b.end],
                                                op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

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
        self.wait_params()  # ZeRO: a bucket no forward module waited for (unused parameters)
        stale = [p for p, sl in self._slots.items() if sl.fresh]
        if stale:  # parameters that got no gradient this step: their slots hold last step's data
            torch._foreach_zero_([self._slots[p].view for p in stale])
            for p in stale:
                self._slots[p].fresh = False
                p.grad = self._slots[p].view
        if not self.comm:
            if self._early_norm and self._sync:
                for g in self.groups:
                    for b in g.buckets:
                        if not b.normed:  # no gradient announced (unused params) or partial bucket
                            self._launch_norm(g, b)
                        b.ready.clear()
            return
        for g in self.groups:
            for b in g.buckets:
                if b.work is None:
                    self._launch(g, b)
        for g in self.groups:
            for b in g.buckets:
                b.work.wait()
                b.work = None
                b.ready.clear()
                if self.zero and self.gloo:
                    c = (b.end - b.start) // self.world_size
                    lo = b.start + self.rank * c
                    g.shard_grad[b.shard_off:b.shard_off + c].copy_(g.grad[lo:lo + c])

    def grad_buffers(self) -> List[torch.Tensor]:
        """Gradient buffers the optimizer consumes (ZeRO: this rank's reduced shards)."""
        if self.zero:
            return [g.shard_grad for g in self.groups]
        return [g.grad for g in self.groups]

    def clip_grad_norm_(self, max_norm: float):
        """Global grad norm of the AVERAGED gradient and the clip coefficient (device scalars, no
        host sync); the 1/world averaging is folded into the coefficient consumed by FusedAdamW."""
        from ..ops import clip_grad_norm_ as _clip
        W = self.world_size
        if self._early_norm:
            done = all(b.normed for g in self.groups for b in g.buckets)
            bad = self._norm_bad
            for g in self.groups:
                for b in g.buckets:
                    b.normed = False
            self._norm_bad = False
            if done and not bad:
                from .. import _native
                from ..ops import GradClipState
                cur = torch.cuda.current_stream(self._norm_ws.device)
                cur.wait_stream(self._norm_stream)
                st = GradClipState(self._norm_ws.device)
                _native.kernels().clip_finalize(self._norm_ws, self._norm_ws.numel(), float(max_norm), 1.0, st.buf)
                return st
        if not self.zero:
            return _clip(self.grad_buffers(), max_norm, prescale=1.0 / W)
        st = _clip(self.grad_buffers(), 0.0, prescale=1.0)
        ss = (st.buf[0] ** 2).reshape(1)
        if self.proxy:
            ss = ss * W  # the other ranks' shards, modelled as equal to this one
        else:
            small_all_reduce(ss, group=self.pg)
        total = ss[0].sqrt() / W
        coef = torch.clamp(max_norm / (total + 1e-6), max=1.0) if max_norm > 0 else torch.ones_like(total)
        st.buf[0] = total
        st.buf[1] = coef / W
        return st

    def after_optimizer_step(self):
        """ZeRO: start the all-gather of the updated shards, forward order; forward pre-hooks wait."""
        if not self.zero:
            return
        W = self.world_size
        for g in self.groups:
            for b in reversed(g.buckets):  # buckets are in backward order; forward needs the last first
                c = (b.end - b.start) // W
                src = g.shard_param[b.shard_off:b.shard_off + c]
                if self.proxy:  # the local part of the all-gather
                    g.flat[b.start + self.rank * c:b.start + (self.rank + 1) * c].copy_(src)
                    b.ag_work = _DoneWork()
                elif self.gloo:
                    b.ag_work = dist.all_gather(list(g.flat[b.start:b.end].chunk(W)), src, group=self.pg,
                                                async_op=True)
                else:
                    b.ag_work = dist.all_gather_into_tensor(g.flat[b.start:b.end], src, group=self.pg, async_op=True)

    def wait_params(self):
        for g in self.groups:
            for b in g.buckets:
                if b.ag_work is not None:
                    b.ag_work.wait()
                    b.ag_work = None

    def zero_grad(self, set_to_none: bool = True):
        """Mark every gradient slot fresh: the next write overwrites (GEMM beta = 0 / copy)."""
        for p, sl in self._slots.items():
            sl.fresh = True
            p.grad = None
        for g in self.groups:
            for b in g.buckets:
                b.normed = False
                if not self.comm:
                    b.ready.clear()
        self._norm_bad = False

    def optimizer_param_groups(self, weight_decay: float = 0.0):
        """One flat Parameter per (dtype, decay) group; its .grad is the flat gradient buffer
        (ZeRO: this rank's contiguous parameter / gradient shard)."""
        out = []
        for g in self.groups:
            fp = nn.Parameter(g.shard_param if self.zero else g.flat, requires_grad=False)
            fp.grad = g.shard_grad if self.zero else g.grad
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

    # ------------------------------------------------------------------ portable optimizer state
    # The flat layout (bucket padding, ZeRO's align x world bucket alignment, the bucket size the
    # planner picks for the world size) differs between world sizes, so the optimizer state of the
    # flat parameters cannot be resumed elsewhere. The portable form is HF's optimizer.pt layout: one
    # state entry per model parameter (index = position among the trainable named_parameters), in
    # the parameter's shape, plus one param group per engine group (reference checkpoint layout:
    # ray-jobs/fine_tune_llama_ray.py:313-319).
    _OPT_KEYS = ("exp_avg", "exp_avg_sq", "master")

    def _named_trainable(self):
        seen, out = set(), []
        for n, p in self.module.named_parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                out.append((n, p))
        return out

    def _inner_opt(self, optimizer):
        if hasattr(optimizer, "synchronize"):  # OverlappedOptimizer: pending chunk updates land first
            optimizer.synchronize()
        inner = getattr(optimizer, "opt", optimizer)
        if len(inner.param_groups) != len(self.groups) or any(len(pg["params"]) != 1 for pg in inner.param_groups):
            raise ValueError("portable optimizer state needs the optimizer built on optimizer_param_groups()")
        return inner, [pg["params"][0] for pg in inner.param_groups]

    def _gather_flat(self, g, t: torch.Tensor) -> Optional[torch.Tensor]:
        """Rank 0: the full flat-length state of a group (ZeRO: gathered to host); None elsewhere.
        ZeRO: every bucket's 1/world chunks are gathered to rank 0 (one collective per bucket)."""
        if not self.zero:  # replicated: rank 0's own state (device views; the caller snapshots them)
            return t.detach() if self.rank == 0 else None
        if self.proxy:
            raise NotImplementedError("proxy_world engines hold one rank's shard only")
        W = self.world_size
        full = torch.zeros(g.flat.numel(), dtype=t.dtype) if self.rank == 0 else None
        dst = dist.get_global_rank(self.pg, 0) if self.pg is not None else 0
        for b in g.buckets:
            c = (b.end - b.start) // W
            if c == 0:
                continue
            chunk = t[b.shard_off:b.shard_off + c].contiguous()
            parts = [torch.empty_like(chunk) for _ in range(W)] if self.rank == 0 else None
            dist.gather(chunk, parts, dst=dst, group=self.pg)
            if self.rank == 0:
                full[b.start:b.end].copy_(torch.cat(parts).to("cpu"))
        return full

    def portable_optimizer_state_dict(self, optimizer) -> Optional[dict]:
        """Collective. On rank 0: the optimizer state per model parameter (HF ``optimizer.pt``
        layout, host tensors in the parameters' shapes); None on the other ranks."""
        inner, fps = self._inner_opt(optimizer)
        named = self._named_trainable()
        index = {id(p): i for i, (_, p) in enumerate(named)}
        state: Dict[int, dict] = {}
        groups_out = []
        for gi, (g, fp) in enumerate(zip(self.groups, fps)):
            st = inner.state.get(fp, {})
            groups_out.append(dict({k: v for k, v in inner.param_groups[gi].items() if k != "params"},
                                   params=sorted(index[id(p)] for p in g.params)))
            for key in self._OPT_KEYS:
                v = st.get(key)
                if not isinstance(v, torch.Tensor):
                    continue
                full = self._gather_flat(g, v)
                if full is not None:
                    for p, o in zip(g.params, g.offsets):
                        v = full[o:o + p.numel()].view(p.shape)
                        # host views are cloned (torch.save would write the whole bucket storage per
                        # view); device views are copied out by the caller's host snapshot
                        state.setdefault(index[id(p)], {})[key] = v.clone() if v.device.type == "cpu" else v
            if self.rank == 0 and isinstance(st.get("step"), torch.Tensor):
                for p in g.params:
                    state.setdefault(index[id(p)], {})["step"] = st["step"].detach().to("cpu", torch.float32).clone()
        if self.rank != 0:
            return None
        return {"state": state, "param_groups": groups_out, "grt_param_names": [n for n, _ in named]}

    def load_portable_optimizer_state_dict(self, optimizer, sd: dict):
        """Every rank: rebuild this engine's flat (or ZeRO shard) optimizer state from a
        :meth:`portable_optimizer_state_dict` written at ANY world size / sharding."""
        inner, fps = self._inner_opt(optimizer)
        named = self._named_trainable()
        names = [n for n, _ in named]
        if list(sd.get("grt_param_names", [])) != names:
            raise ValueError("optimizer state was written for a different set of trainable parameters")
        index = {id(p): i for i, (_, p) in enumerate(named)}
        if len(sd["param_groups"]) != len(self.groups):
            raise ValueError(f"optimizer state has {len(sd['param_groups'])} param groups, the engine {len(self.groups)}")
        W, r = self.world_size, self.rank
        for gi, (g, fp) in enumerate(zip(self.groups, fps)):
            sg = sd["param_groups"][gi]
            if sorted(sg["params"]) != sorted(index[id(p)] for p in g.params):
                raise ValueError(f"param group {gi} holds different parameters than the engine's group {gi}")
            inner.param_groups[gi].update({k: v for k, v in sg.items() if k != "params"})
            first = sd["state"].get(index[id(g.params[0])], {})
            st = inner.state[fp]
            for key in self._OPT_KEYS:
                if not isinstance(first.get(key), torch.Tensor):
                    continue
                n_out = fp.numel()
                out = torch.zeros(n_out, dtype=torch.float32)
                for b in g.buckets:
                    if self.zero:
                        c = (b.end - b.start) // W
                        lo, hi, base = b.start + r * c, b.start + (r + 1) * c, b.shard_off
                    else:
                        lo, hi, base = b.start, b.end, b.start
                    for p in b.params:
                        o = self._flat_offset(g, p)
                        a_, e_ = max(o, lo), min(o + p.numel(), hi)
                        if a_ < e_:
                            src = sd["state"][index[id(p)]][key].reshape(-1)
                            out[base + a_ - lo:base + e_ - lo].copy_(src[a_ - o:e_ - o].float())
                st[key] = inner._state_tensor(out, fp)
            if "step" in first:
                st["step"] = torch.as_tensor(first["step"]).detach().to("cpu", torch.float32).clone().reshape(())

    @staticmethod
    def _flat_offset(g, p) -> int:
        off = getattr(g, "_offset_of", None)
        if off is None:
            off = g._offset_of = {id(q): o for q, o in zip(g.params, g.offsets)}
        return off[id(p)]

    def close(self):
        """Collective (every rank): release this engine's IPC bucket communicator — its staging
        buffers and peer mappings — once no further step will run on the engine."""
        if self._ipc is not None:
            from .ipc import release_communicator
            if self._ipc_stream is not None:
                torch.cuda.current_stream(self._ipc_stream.device).wait_stream(self._ipc_stream)
            release_communicator(self.pg, self._ipc_tag)
            self._ipc = None
            self._ipc_limit = 0
