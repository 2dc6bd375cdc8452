"""Fully-sharded data parallelism (ZeRO-3 style) over RCCL, with optional optimizer-state offload.

Not in the reference (its only strategy is DDP); required by BASELINE.json configs #3 (Llama-2-7B
FSDP full-shard bf16) and #5 (Llama-3-70B FSDP full-shard + CPU offload). SURVEY §2.4, §7.5.

Design for 8 x MI355X on xGMI:
* a *unit* = one transformer block (``LlamaDecoderLayer`` / ``EncoderLayer``) plus a root unit
  (embeddings, LM head). Each unit's weight MATRICES live as one padded flat bf16 buffer split
  into ``world`` contiguous shards; rank r keeps shard r in a single rank-local shard store, so
  the optimizer updates all of a rank's parameters with ONE fused AdamW launch;
* 1-D parameters (norm weights, biases: <0.01 % of a Llama) are replicated and all-reduced once
  per step (no per-layer latency-bound micro-collectives, no weight decay on them — HF rule);
* forward: a unit's all-gather (``all_gather_into_tensor`` = one RCCL collective per unit,
  ~400 MB for a 7B block at 8 ranks, well into the multi-ring bandwidth regime) is issued one
  unit AHEAD on RCCL's stream while the current unit computes; after the unit runs, its full
  buffer is released (``reshard_after_forward``);
* backward: an identity autograd node on each unit's output re-gathers the unit (prefetching the
  previous one) right before its backward kernels; weight gradients are written by the GEMMs
  straight into the unit's full gradient buffer (ops/linear.py slots), and when the last one
  lands the buffer is reduce-scattered (SUM; the 1/world average is folded into the optimizer)
  into this rank's gradient shard and freed;
* gathered-parameter and full-gradient buffers come from a per-size free list (every decoder
  block has the same size, so after the first step no unit gather or backward allocates: no
  caching-allocator churn with 1.7 GB 70B blocks); at most ``GRT_FSDP_RS_INFLIGHT`` (2)
  reduce-scatters are outstanding, so the full-gradient buffers in flight are bounded too;
* ``GRT_FORCE_COLLECTIVES=1`` runs the collective path (gather into separate buffers,
  reduce-scatter, replicated all-reduce) even at world size 1, for one-GPU RCCL rehearsal;
* ``cpu_offload=True``: fp32 Adam moments live in pinned host memory and are streamed through the
  GPU AdamW kernel in chunks on a side stream (H2D of chunk i+1 / D2H of chunk i-1 overlap the
  update of chunk i); parameters and gradients stay in HBM.
"""
from __future__ import annotations

import collections
import contextlib
import os
import math
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops.linear import GradSlot
from .comm import small_all_reduce

DEFAULT_UNITS = ("LlamaDecoderLayer", "EncoderLayer")
_ALIGN = 64


# GRT_FSDP_ZERO_FULL_GRAD=1: memset each unit's whole gradient buffer (A/B switch for the gap-only clear)
_ZERO_FULL_GRAD = os.environ.get("GRT_FSDP_ZERO_FULL_GRAD", "0") == "1"

class _BwdGather(torch.autograd.Function):
    """Identity on a unit's output; its backward fires right before the unit's backward kernels."""

    @staticmethod
    def forward(ctx, fsdp, unit, *xs):
        ctx.fsdp, ctx.unit = fsdp, unit
        return xs if len(xs) > 1 else xs[0]

    @staticmethod
    def backward(ctx, *gs):
        ctx.fsdp._pre_backward(ctx.unit)
        return (None, None) + gs


class _Unit:
    def __init__(self, idx, module, items, world):
        self.idx = idx
        self.module = module
        self.params = [p for _, p in items]
        self.names = [n for n, _ in items]
        self.shapes = [p.shape for p in self.params]
        self.numels = [p.numel() for p in self.params]
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += (n + _ALIGN - 1) // _ALIGN * _ALIGN
        per = (off + world - 1) // world
        per = (per + _ALIGN - 1) // _ALIGN * _ALIGN
        self.shard_numel = per
        self.total = per * world
        self.full: Optional[torch.Tensor] = None
        self.gather_work = None
        self.grad_full: Optional[torch.Tensor] = None
        self.ready = 0
        self.rs_work = None
        self.rs_out: Optional[torch.Tensor] = None
        self.in_backward = False
        self.slots: Dict[int, GradSlot] = {}


class _DoneWork:
    """Stand-in for a collective's Work in proxy mode (the local copy already ran in stream order)."""

    def wait(self):
        return None


class _StreamDoneWork:
    """Proxy-mode stand-in for a gather issued on the side stream: wait() orders the current stream
    after the copy (as a real collective's Work.wait() does)."""

    def __init__(self, event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)


def partition_units(module: nn.Module, world: int, unit_types=DEFAULT_UNITS):
    """The FSDP partition: one unit per transformer block plus a root unit (embeddings, LM head)
    holding every other matrix; 1-D parameters are replicated. Allocates nothing, so it also runs
    on a meta-device model (``parallel/planner.py`` sizes a 70B partition this way)."""
    unit_mods = [m for m in module.modules() if type(m).__name__ in unit_types]
    owner = {}
    for ui, m in enumerate(unit_mods):
        for n, p in m.named_parameters():
            owner.setdefault(id(p), ui)
    seen = set()
    per_unit: List[List[tuple]] = [[] for _ in range(len(unit_mods) + 1)]
    replicated: List[tuple] = []
    for n, p in module.named_parameters():
        if id(p) in seen or not p.requires_grad:
            continue
        seen.add(id(p))
        if p.dim() < 2:
            replicated.append((n, p))
        else:
            per_unit[owner.get(id(p), len(unit_mods))].append((n, p))
    mods = unit_mods + [module]
    units = [_Unit(i, mods[i], items, world) for i, items in enumerate(per_unit) if items]
    return units, replicated


class FullyShardedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, process_group=None, unit_types=DEFAULT_UNITS, reshard_after_forward=True,
                 cpu_offload: bool = False, sync_module_states: bool = True, param_init_fn=None, device=None,
                 offload_chunk_elems: int = 1 << 26, force_collectives: Optional[bool] = None,
                 proxy_world: int = 0):
        super().__init__()
        self.module = module
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if self.world > 1 else 0
        if force_collectives is None:
            force_collectives = os.environ.get("GRT_FORCE_COLLECTIVES", "0") == "1"
        # proxy_world = N on ONE process (no process group): rank 0 of an N-rank job — 1/N shards of
        # every unit, full-unit gather buffers allocated and released exactly as at world N, the
        # AdamW (or offload) state of 1/N — with each collective replaced by the local copy of this
        # rank's part (all-gather: own shard into its slot; reduce-scatter: own chunk of the full
        # gradient). The step an N-GPU run executes minus the xGMI transfers (bench.py
        # --parallel fsdp --proxy-world N; every slot of a gathered unit holds a copy of this rank's
        # shard, so the loss is not meaningful). Mirrors parallel/ddp.py's proxy mode.
        self.proxy = int(proxy_world) > 1 and self.world == 1
        if self.proxy:
            self.world, self.rank = int(proxy_world), 0
        self.comm = self.proxy or self.world > 1 or (bool(force_collectives) and dist.is_initialized())
        self._pool: Dict[int, List[torch.Tensor]] = {}
        self._rs_inflight = collections.deque()
        self._rs_cap = max(1, int(os.environ.get("GRT_FSDP_RS_INFLIGHT", "2")))
        self.reshard_after_forward = reshard_after_forward
        self.cpu_offload = cpu_offload
        self.offload_chunk = offload_chunk_elems
        self._sync = True
        # GRT_GLOO_TENSOR_COLLECTIVES=1: run the RCCL code path over gloo (CPU tests), see ddp.py
        self.gloo = (self.comm and not self.proxy and dist.get_backend(process_group) == "gloo"
                     and os.environ.get("GRT_GLOO_TENSOR_COLLECTIVES", "0") != "1")
        first = next(module.parameters())
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if first.device.type == "meta" else first.device)
        # ---------------------------------------------------------------- partition parameters
        self.units, self.replicated = partition_units(module, self.world, unit_types)
        self.dtype = next((p.dtype for u in self.units for p in u.params), torch.bfloat16)
        if self.dtype == torch.float32 and first.device.type != "meta":
            self.dtype = first.dtype
        # ---------------------------------------------------------------- shard stores
        self._replaced = {}      # id(original parameter) -> its materialised replacement
        self._replaced_keep = []  # the originals, alive until construction ends: no id() is reused
        tot = sum(u.shard_numel for u in self.units)
        self.shard_store = torch.zeros(tot, dtype=self.dtype, device=self.device)
        self.grad_store = torch.zeros(tot, dtype=self.dtype, device=self.device)
        off = 0
        for u in self.units:
            u.shard = self.shard_store[off:off + u.shard_numel]
            u.shard_grad = self.grad_store[off:off + u.shard_numel]
            off += u.shard_numel
            self._materialize_and_shard(u, param_init_fn, sync_module_states)
        # replicated (1-D) params: one flat buffer, all-reduced once per step
        self.replicated = [(n, self._replaced.get(id(p), p)) for n, p in self.replicated]
        for m in module.modules():
            own = [(n, p) for n, p in m.named_parameters(recurse=False) if p.device.type == "meta"]
            for n, p in own:
                newp = nn.Parameter(torch.empty(p.shape, dtype=self.dtype, device=self.device),
                                    requires_grad=p.requires_grad)
                setattr(m, n, newp)
                self._replaced[id(p)] = newp
                self._replaced_keep.append(p)
            if own and param_init_fn is not None:
                param_init_fn(m)
        self.replicated = [(n, self._replaced.get(id(p), p)) for n, p in self.replicated]
        self._replaced_keep = []
        rn = sum(p.numel() for _, p in self.replicated)
        self.rep_flat = torch.zeros(max(rn, 1), dtype=self.dtype, device=self.device)
        self.rep_grad = torch.zeros(max(rn, 1), dtype=self.dtype, device=self.device)
        o = 0
        with torch.no_grad():
            for _, p in self.replicated:
                self.rep_flat[o:o + p.numel()].copy_(p.data.view(-1))
                p.data = self.rep_flat[o:o + p.numel()].view_as(p)
                p.grad = self.rep_grad[o:o + p.numel()].view_as(p)
                o += p.numel()
        if sync_module_states and self.world > 1 and rn and not self.proxy:
            dist.broadcast(self.rep_flat, 0, group=process_group)
        self._rep_hooks = [p.register_post_accumulate_grad_hook(self._rep_hook) for _, p in self.replicated]
        self._rep_fresh = True
        # ---------------------------------------------------------------- hooks
        self._order: List[_Unit] = []
        for u in self.units:
            self._attach_slots(u)
        self._enable_forward_transposes()
        for u in self.units:
            if u.module is not module:
                u.module.register_forward_pre_hook(self._make_pre_fwd(u))
                u.module.register_forward_hook(self._make_post_fwd(u))
        self._root_unit = next((u for u in self.units if u.module is module), None)
        self._offload_state = None
        # overlapped offloaded optimizer (parallel/offload.py): per-unit "shard updated" events,
        # waited for before the unit's next all-gather / forward; it also zeroes the grad shards
        self._update_events: Dict[int, torch.cuda.Event] = {}
        self._forward_tail_hooks = []
        self._grad_zero_by_optimizer = False
        self._grads_consumed = False  # set by an optimizer that zeroed the gradients itself (offload.py)
        self._gstream = None

    def _enable_forward_transposes(self):
        """Projection weights get W^T written on a side stream at forward time (right after the unit's
        all-gather, ops/linear.transpose_for_backward), kept until the backward's input-gradient
        GEMM, which then runs in the TN form instead of the NN form (13-15 % faster on the Llama
        shapes; the NN kernels were 80 ms of the proxy-8 step, profiles/r6_proxy8_steps.md). The
        copies persist across steps (one buffer per weight), i.e. one full bf16 copy of the
        projection weights per rank, so only when that fits ``GRT_FSDP_FWD_TRANSPOSE_MAX_GIB``
        (default 24: Llama-2-7B / 3-8B yes, 70B no); ``GRT_FSDP_FWD_TRANSPOSE=0`` turns it off."""
        mode = os.environ.get("GRT_FSDP_FWD_TRANSPOSE", "auto")
        if mode == "0" or self.device.type != "cuda":
            return
        from ..ops.linear import Linear as _DirectLinear
        ws = [m.weight for u in self.units if u.module is not self.module for m in u.module.modules()
              if isinstance(m, _DirectLinear) and m.weight.requires_grad and m.weight.dtype == torch.bfloat16]
        # the units' recorded full sizes: after sharding a module's weight tensor no longer has them
        # (a 70B model measured as "fits" and kept 130 GiB of W^T copies, profiles/r6_offload_link.md)
        full = {id(p): n for u in self.units for p, n in zip(u.params, u.numels)}
        nbytes = sum(full.get(id(w), w.numel()) * w.element_size() for w in ws)
        self.fwd_transpose_bytes = nbytes
        if mode == "auto" and nbytes > float(os.environ.get("GRT_FSDP_FWD_TRANSPOSE_MAX_GIB", "24")) * (1 << 30):
            return
        for w in ws:
            w._grt_fsdp_fwd_transpose = True

    # ================================================================ optimizer hand-off
    def set_update_events(self, events):
        self._update_events = {id(u): ev for u, ev in events.items()}

    def _wait_update(self, u: _Unit, stream=None):
        ev = self._update_events.pop(id(u), None)
        if ev is not None:
            (stream or torch.cuda.current_stream(self.device)).wait_event(ev)

    def wait_updates(self):
        """The current stream waits for every pending unit update (checkpointing, eval, step)."""
        cur = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        for ev in self._update_events.values():
            cur.wait_event(ev)
        self._update_events.clear()

    # ================================================================ sharding helpers
    @torch.no_grad()
    def _materialize_and_shard(self, u: _Unit, init_fn, sync):
        if any(p.device.type == "meta" for p in u.params):
            ids = {id(p) for p in u.params}
            mods = list(u.module.modules()) if u.module is not self.module else list(self.module.modules())
            repl = {}
            for m in mods:
                own = [(n, p) for n, p in m.named_parameters(recurse=False) if id(p) in ids or
                       (u.module is not self.module and p.device.type == "meta")]
                if not own:
                    continue
                for n, p in own:
                    newp = nn.Parameter(torch.empty(p.shape, dtype=self.dtype, device=self.device),
                                        requires_grad=p.requires_grad)
                    setattr(m, n, newp)
                    repl[id(p)] = newp
                    self._replaced_keep.append(p)
                if init_fn is not None:
                    init_fn(m)
            u.params = [repl.get(id(p), p) for p in u.params]
            self._replaced.update(repl)
        full = torch.zeros(u.total, dtype=self.dtype, device=self.device)
        for p, o, n in zip(u.params, u.offsets, u.numels):
            full[o:o + n].copy_(p.data.reshape(-1))
        if sync and self.world > 1 and not self.proxy:
            dist.broadcast(full, 0, group=self.pg)
        u.shard.copy_(full[self.rank * u.shard_numel:(self.rank + 1) * u.shard_numel])
        if not self.comm:
            self._bind(u, u.shard)  # single rank: the shard IS the full buffer, never freed
        else:
            self._unbind(u)
        del full

    def _bind(self, u: _Unit, full: torch.Tensor):
        u.full = full
        for p, o, n, s in zip(u.params, u.offsets, u.numels, u.shapes):
            p.data = full[o:o + n].view(s)

    def _acquire(self, n: int, zero: bool = False) -> torch.Tensor:
        free = self._pool.get(n)
        buf = free.pop() if free else torch.empty(n, dtype=self.dtype, device=self.device)
        if zero:
            buf.zero_()
        return buf

    def _release(self, buf: Optional[torch.Tensor]):
        # Stream safety: the next user of a gather buffer is an all-gather, which RCCL orders after
        # the compute stream's queued kernels at issue; a gradient buffer comes back only after its
        # reduce-scatter was waited on (compute stream joined RCCL's), and is re-zeroed on it.
        if buf is not None and buf.numel() > 0:
            self._pool.setdefault(buf.numel(), []).append(buf)

    def _unbind(self, u: _Unit):
        if not self.comm:
            return
        if self.device.type == "cuda":  # side-stream W^T reads of this gather (ops/linear.py) finish
            cur = None  # before the buffer can be handed to the next all-gather
            for p in u.params:
                ev = getattr(p, "_grt_wt_pending", None)
                if ev is not None:
                    cur = cur or torch.cuda.current_stream(self.device)
                    cur.wait_event(ev)
                    p._grt_wt_pending = None
        if u.full is not None and u.full is not u.shard:
            self._release(u.full)
        u.full = None
        for p in u.params:
            p.data = torch.empty(0, dtype=self.dtype, device=self.device)

    # ================================================================ all-gather
    def _issue_gather(self, u: _Unit):
        if u.full is not None or u.gather_work is not None or not self.comm:
            return
        buf = self._acquire(u.total)
        if id(u) in self._update_events and self.device.type == "cuda":
            # the shard is still being updated on the optimizer's stream: issue the gather from a
            # side stream that waits for that update, so the compute stream (still running the
            # previous unit) never blocks on a later unit's optimizer work
            if self._gstream is None:
                self._gstream = torch.cuda.Stream(self.device)
            self._gstream.wait_stream(torch.cuda.current_stream(self.device))  # buffer reuse order
            self._wait_update(u, self._gstream)
            with torch.cuda.stream(self._gstream):
                self._gather_into(u, buf)
                if self.proxy:  # the local copy ran on the side stream: the consumer must wait for it
                    ev = torch.cuda.Event()
                    ev.record(self._gstream)
                    u.gather_work = _StreamDoneWork(ev)
        else:
            self._gather_into(u, buf)
        u._pending_buf = buf

    def _gather_into(self, u: _Unit, buf):
        if self.proxy:  # stand-in for the all-gather: this rank's shard into EVERY slot (one local
            # copy of the full unit; the other ranks' slots must hold real-magnitude weights, not
            # zeros: zero operands would let the GEMMs clock higher and flatter the proxy timing)
            buf.view(self.world, u.shard_numel).copy_(u.shard.unsqueeze(0).expand(self.world, -1))
            u.gather_work = _DoneWork()
        elif self.gloo:
            parts = list(buf.chunk(self.world))
            u.gather_work = dist.all_gather(parts, u.shard, group=self.pg, async_op=True)
        else:
            u.gather_work = dist.all_gather_into_tensor(buf, u.shard, group=self.pg, async_op=True)

    def _wait_gather(self, u: _Unit):
        if not self.comm:
            self._wait_update(u)  # world 1: the shard is the parameter; wait for its update
            return
        if u.full is None and u.gather_work is None:
            self._issue_gather(u)
        if u.gather_work is not None:
            u.gather_work.wait()
            u.gather_work = None
            self._bind(u, u._pending_buf)
            u._pending_buf = None

    def _next(self, u: _Unit, step: int) -> Optional[_Unit]:
        seq = [x for x in self.units if x.module is not self.module]
        if u.module is self.module or u not in seq:
            return None
        i = seq.index(u) + step
        return seq[i] if 0 <= i < len(seq) else None

    def add_forward_tail_hook(self, fn):
        """``fn()`` runs when the LAST decoder unit's training forward starts (the offloaded
        optimizer starts its moment uploads there, so they cross the host link during backward)."""
        self._forward_tail_hooks.append(fn)

    def _make_pre_fwd(self, u: _Unit):
        def hook(mod, args):
            self._wait_gather(u)
            nxt = self._next(u, +1)
            if nxt is not None and not u.in_backward:
                self._issue_gather(nxt)
            elif (nxt is None and not u.in_backward and self._forward_tail_hooks and u.module is not self.module
                  and torch.is_grad_enabled() and self.module.training):
                for fn in self._forward_tail_hooks:
                    fn()
        return hook

    def _make_post_fwd(self, u: _Unit):
        def hook(mod, args, out):
            if torch.is_grad_enabled() and self.module.training:
                if not u.in_backward:
                    if self.reshard_after_forward:
                        self._unbind(u)
                    tensors = out if isinstance(out, tuple) else (out,)
                    idx = [i for i, t in enumerate(tensors) if isinstance(t, torch.Tensor) and t.requires_grad]
                    if idx:
                        wrapped = _BwdGather.apply(self, u, *[tensors[i] for i in idx])
                        wrapped = wrapped if isinstance(wrapped, tuple) else (wrapped,)
                        lst = list(tensors)
                        for i, w in zip(idx, wrapped):
                            lst[i] = w
                        return tuple(lst) if isinstance(out, tuple) else lst[0]
            elif self.reshard_after_forward and not u.in_backward:
                self._unbind(u)
            return out
        return hook

    # ================================================================ backward
    def _pre_backward(self, u: _Unit):
        u.in_backward = True
        self._wait_gather(u)
        prev = self._next(u, -1)
        if prev is not None:
            self._issue_gather(prev)
        self._alloc_grads(u)

    def _alloc_grads(self, u: _Unit):
        if u.grad_full is not None:
            return
        # every parameter's slot is written whole by its first gradient of the step (GEMM beta = 0,
        # copy, or the zero fill of finish_gradient_sync for unused ones), so only the alignment gaps
        # between slots and the tail must be cleared (they must not inject garbage into the
        # reduction): a few small ranges instead of a memset of the whole unit (37 x 55 us per
        # Llama-2-7B step, profiles/r6_proxy8_steps.md)
        g = self._acquire(u.total, zero=_ZERO_FULL_GRAD)
        gaps = None if _ZERO_FULL_GRAD else getattr(u, "_grad_gaps", None)
        if gaps is None and not _ZERO_FULL_GRAD:
            gaps, end = [], 0
            for o, n in sorted(zip(u.offsets, u.numels)):
                if o > end:
                    gaps.append((end, o))
                end = max(end, o + n)
            if end < u.total:
                gaps.append((end, u.total))
            u._grad_gaps = gaps
        if gaps:
            torch._foreach_zero_([g[a:b] for a, b in gaps])
        u.grad_full = g
        u.ready = 0
        for p, o, n, s in zip(u.params, u.offsets, u.numels, u.shapes):
            sl = u.slots[id(p)]
            sl.view = g[o:o + n].view(s)
            sl.fresh = True
            p.grad = None

    def _attach_slots(self, u: _Unit):
        # Slots exist from construction on, so the forward takes the same (direct-grad) code path
        # in the original pass and in an activation-checkpoint recompute.
        shared = getattr(self, "_shared_ids", None)
        if shared is None:
            from .ddp import shared_param_ids
            shared = self._shared_ids = shared_param_ids(self.module)
        for p in u.params:
            sl = GradSlot(torch.empty(0, dtype=self.dtype, device=self.device), self._param_ready)
            if id(p) not in shared:  # tied weights keep the AccumulateGrad path (two producers)
                p._grt_slot = sl
            p._grt_unit = u
            u.slots[id(p)] = sl
            p._grt_fsdp_hook = p.register_post_accumulate_grad_hook(self._acc_hook)

    def _acc_hook(self, p):
        # AccumulateGrad path (params not written by a direct-grad GEMM): fold into the slot
        u = getattr(p, "_grt_unit", None)
        if u is None:
            return
        sl = u.slots[id(p)]
        if sl.consume_direct():  # the GEMM already wrote and announced this gradient
            return
        if p.grad is not None and p.grad.data_ptr() != sl.view.data_ptr():
            with torch.no_grad():
                sl.view.copy_(p.grad) if sl.fresh else sl.view.add_(p.grad)
        sl.fresh = False
        p.grad = None
        self._param_ready(p)

    def _param_ready(self, p):
        u = p._grt_unit
        sl = u.slots[id(p)]
        sl.fresh = False
        p.grad = None
        u.ready += 1
        if u.ready == len(u.params):
            self._reduce_scatter(u)

    def _reduce_scatter(self, u: _Unit):
        g = u.grad_full
        if not self.comm:
            if self._accumulating(u):
                u.shard_grad.add_(g)
            else:
                u.shard_grad.copy_(g)
            self._release(g)
        else:
            if self.gloo or self.proxy:
                if not self.proxy:
                    dist.all_reduce(g, group=self.pg)
                part = g[self.rank * u.shard_numel:(self.rank + 1) * u.shard_numel]
                if self._accumulating(u):
                    u.shard_grad.add_(part)
                else:
                    u.shard_grad.copy_(part)
                self._release(g)
            else:
                if u.rs_work is not None:  # previous micro-step's reduce-scatter of this unit
                    self._finish_rs(u)
                out = u.shard_grad if not self._accumulating(u) else torch.empty_like(u.shard_grad)
                u.rs_work = dist.reduce_scatter_tensor(out, g, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
                u.rs_out = out if out is not u.shard_grad else None
                u._rs_src = g
                self._rs_inflight.append(u)
                while len(self._rs_inflight) > self._rs_cap:  # bound the full-gradient buffers in flight
                    old = self._rs_inflight.popleft()
                    if old.rs_work is not None:
                        self._finish_rs(old)
        u.grad_full = None
        u.in_backward = False
        u.ready = 0
        u.acc_started = True
        if u.module is not self.module:
            self._unbind(u)

    def _finish_rs(self, u: _Unit):
        """Wait a unit's reduce-scatter (stream-ordered for RCCL) and fold an accumulation
        temporary into the shard; its source buffer may be released only after this."""
        u.rs_work.wait()
        u.rs_work = None
        if u.rs_out is not None:
            u.shard_grad.add_(u.rs_out)
            u.rs_out = None
        self._release(u._rs_src)
        u._rs_src = None

    def _accumulating(self, u):
        return getattr(u, "acc_started", False)

    # ================================================================ replicated params
    def _rep_hook(self, p):
        pass

    # ================================================================ public API
    @contextlib.contextmanager
    def no_sync(self, enabled: bool = True):
        prev = self._sync
        self._sync = not enabled
        try:
            yield
        finally:
            self._sync = prev

    def forward(self, *args, **kwargs):
        if self._root_unit is not None:
            self._wait_gather(self._root_unit)
            if self.module.training and torch.is_grad_enabled():
                self._alloc_grads(self._root_unit)
        first = next((x for x in self.units if x.module is not self.module), None)
        if first is not None:
            self._issue_gather(first)
        return self.module(*args, **kwargs)

    def finish_gradient_sync(self):
        """Complete reduce-scatters and the replicated-param all-reduce of this step."""
        for u in self.units:
            if u.grad_full is not None:  # unit whose grads never all arrived (unused params)
                for p in u.params:
                    sl = u.slots[id(p)]
                    if sl.fresh:
                        sl.view.zero_()
                        sl.fresh = False
                u.ready = len(u.params) - 1
                self._param_ready(u.params[-1]) if u.params else None
        for u in self.units:
            if u.rs_work is not None:
                self._finish_rs(u)
        self._rs_inflight.clear()
        if self.comm and self.replicated and self._sync and not self.proxy:
            small_all_reduce(self.rep_grad, group=self.pg)  # IPC kernels when small enough
        if self._root_unit is not None and self.comm:
            self._unbind(self._root_unit)

    def zero_grad(self, set_to_none: bool = True):
        for u in self.units:
            u.acc_started = False
        # the overlapped offload optimizer zeroes each unit's gradients on its update stream; a
        # zero_grad() that no step() consumed (skipped step, zero_grad at the top of a loop) must
        # still clear them, after the pending updates (replicated params accumulate into rep_grad)
        if not (self._grad_zero_by_optimizer and self._grads_consumed):
            if self._grad_zero_by_optimizer:
                self.wait_updates()
            self.grad_store.zero_()
            self.rep_grad.zero_()
        self._grads_consumed = False
        o = 0
        for _, p in self.replicated:  # a caller may have set .grad = None: re-attach the views
            p.grad = self.rep_grad[o:o + p.numel()].view_as(p)
            o += p.numel()

    def grad_buffers(self) -> List[torch.Tensor]:
        """Gradient shards (the global norm is completed by an all-reduce inside clip_grad_norm_)."""
        return [self.grad_store, self.rep_grad]

    @property
    def world_size(self) -> int:
        return self.world

    def build_optimizer(self, lr: float, weight_decay: float = 0.0, betas=(0.9, 0.999), eps=1e-8,
                        overlap: Optional[bool] = None, resident_fraction: Optional[float] = None,
                        prefetch_slots: int = 0):
        """Fused AdamW over this rank's shards. With ``cpu_offload`` the moments live in pinned host
        memory: by default the update is split by unit and overlapped with the next forward, with
        the first ``resident_fraction`` of the moments kept in HBM (parallel/offload.py);
        ``overlap=False`` / GRT_OFFLOAD_OVERLAP=0 is the serial after-backward stream
        (ops.optim.OffloadedAdamW)."""
        from ..ops.optim import FusedAdamW, OffloadedAdamW
        if self.cpu_offload and self.device.type == "cuda":
            if overlap is None:
                overlap = os.environ.get("GRT_OFFLOAD_OVERLAP", "1") != "0"
            if overlap:
                from .offload import OverlappedOffloadAdamW
                if resident_fraction is None:
                    resident_fraction = float(os.environ.get("GRT_OFFLOAD_RESIDENT", "0"))
                return OverlappedOffloadAdamW(self, chunk_elems=self.offload_chunk, resident_fraction=resident_fraction,
                                              prefetch_slots=prefetch_slots, lr=lr, betas=betas, eps=eps,
                                              weight_decay=weight_decay)
            return OffloadedAdamW(self.optimizer_param_groups(weight_decay), chunk_elems=self.offload_chunk, lr=lr,
                                  betas=betas, eps=eps)
        return FusedAdamW(self.optimizer_param_groups(weight_decay), lr=lr, betas=betas, eps=eps)

    def optimizer_param_groups(self, weight_decay: float = 0.0):
        sp = nn.Parameter(self.shard_store, requires_grad=False)
        sp.grad = self.grad_store
        rp = nn.Parameter(self.rep_flat, requires_grad=False)
        rp.grad = self.rep_grad
        return [{"params": [sp], "weight_decay": weight_decay}, {"params": [rp], "weight_decay": 0.0}]

    def clip_grad_norm_(self, max_norm: float):
        """Global grad norm over shards (sum of squares all-reduced), average folded in."""
        from ..ops import clip_grad_norm_ as _clip
        st = _clip([self.grad_store], 0.0, prescale=1.0)
        ss_shard = st.buf[0] ** 2
        st2 = _clip([self.rep_grad], 0.0, prescale=1.0)
        ss_rep = st2.buf[0] ** 2
        if self.comm and not self.proxy:
            small_all_reduce(ss_shard, group=self.pg)
        total = (ss_shard + ss_rep).sqrt() / self.world
        coef = torch.clamp(max_norm / (total + 1e-6), max=1.0) if max_norm > 0 else torch.ones_like(total)
        st.buf[0] = total
        st.buf[1] = coef / self.world
        return st

    @torch.no_grad()
    def full_state_dict(self) -> Dict[str, torch.Tensor]:
        """Gathered (unsharded) state dict on every rank, module parameter names."""
        self.wait_updates()
        out = {}
        for u in self.units:
            self._wait_gather(u)
            for n, p in zip(u.names, u.params):
                out[n] = p.detach().clone()
            if u.module is not self.module or self.comm:
                self._unbind(u)
        for n, p in self.replicated:
            out[n] = p.detach().clone()
        for n, b in self.module.named_buffers():
            out[n] = b.detach().clone()
        return out

    @torch.no_grad()
    def full_grad_dict(self) -> Dict[str, torch.Tensor]:
        """Unsharded gradients (sum over ranks), module parameter names — tests / debugging."""
        out = {}
        for u in self.units:
            if self.comm and not self.proxy:
                parts = [torch.empty_like(u.shard_grad) for _ in range(self.world)]
                dist.all_gather(parts, u.shard_grad.contiguous(), group=self.pg)
                full = torch.cat(parts)
            elif self.proxy:  # only rank 0's chunk exists
                full = torch.zeros(u.total, dtype=u.shard_grad.dtype, device=u.shard_grad.device)
                full[:u.shard_numel].copy_(u.shard_grad)
            else:
                full = u.shard_grad
            for n, o, k, s in zip(u.names, u.offsets, u.numels, u.shapes):
                out[n] = full[o:o + k].view(s).clone()
        o = 0
        for n, p in self.replicated:
            out[n] = self.rep_grad[o:o + p.numel()].view_as(p).clone()
            o += p.numel()
        return out

    @torch.no_grad()
    def load_full_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        """Load an unsharded state dict (module names): every rank keeps only its own shard."""
        missing = []
        for u in self.units:
            full = torch.zeros(u.total, dtype=self.dtype, device=self.device)
            for n, o, k in zip(u.names, u.offsets, u.numels):
                if n in sd:
                    full[o:o + k].copy_(sd[n].reshape(-1))
                else:
                    missing.append(n)
            u.shard.copy_(full[self.rank * u.shard_numel:(self.rank + 1) * u.shard_numel])
        for n, p in self.replicated:
            if n in sd:
                p.data.copy_(sd[n].view_as(p))
            else:
                missing.append(n)
        if strict and missing:
            raise KeyError(f"missing keys in state dict: {missing[:8]}")

    def sharded_state_dict(self) -> Dict[str, torch.Tensor]:
        self.wait_updates()
        return {"shard_store": self.shard_store.detach().clone(), "rep_flat": self.rep_flat.detach().clone(),
                "rank": torch.tensor(self.rank), "world": torch.tensor(self.world)}

    @torch.no_grad()
    def load_sharded_state_dict(self, sd):
        assert int(sd["world"]) == self.world and int(sd["rank"]) == self.rank, "resharding is not supported"
        self.shard_store.copy_(sd["shard_store"])
        self.rep_flat.copy_(sd["rep_flat"])
