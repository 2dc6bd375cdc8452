"""LoRA adapters (PEFT semantics) for the fused-projection Llama layout.

Reference: ``LoraConfig(lora_alpha=16, lora_dropout=0.1, r=64, bias="none", task_type="CAUSAL_LM",
target_modules=[q,k,v,o,gate,up,down]_proj)`` passed to SFTTrainer, then ``merge_and_unload()``
(ray-jobs/fine_tune_llama_ray.py:243-254,353; fine_tune_config.json:6-8,30-33).

The model keeps q/k/v and gate/up as ONE fused base GEMM each. A LoRA wrapper over a fused
projection holds one (A, B) pair per targeted HF sub-projection; the A matrices of all targeted
slices are concatenated so the down-projection is ONE GEMM ``x @ A_cat^T`` ([tokens, r * k]).
On MI355X the whole adapted projection is one autograd op (``_LoraFn``): each target's
up-projection ``h_i @ B_i^T`` is accumulated into its column block of the base output by the GEMM
epilogue (beta = 1, alpha = scaling), the input dropout is the counter-based kernel (no mask
stored, regenerated in the backward) and the adapter's input gradient is added into the base dX
by the dropout-backward kernel in place — no separate add kernels, no block-diagonal B, no
autograd gradient accumulation. Parameter names on disk follow HF PEFT
(``base_model.model.<module>.<proj>.lora_A.weight`` / ``lora_B.weight``).

K-concatenated form (MI355X default, ``GRT_LORA_KCAT=0`` = the epilogue form above): the adapter
rides INSIDE the base GEMM. The producer of the projection input (RMSNorm, attention, SwiGLU
kernel) writes it into a [tokens, in + R] row buffer (R = r * targets); ``lora_down`` writes
h' = s * dropout(x) A_cat^T into the R tail columns; the weight is kept as W' = [W | B_blockdiag]
([out, in + R]) with the B blocks refreshed from the trainable B each forward (``lora_refresh``
kernel). Then y = [x | h'] W'^T is ONE GEMM — base output plus every adapter's up-projection — so
the per-target read-modify-writes of y disappear, for R extra K columns (1-5 % of the base GEMM
at r = 64). The backward keeps the epilogue form (a single [dX | g] = dY W' GEMM was tried: its
N = in + R runs ~15 % below the tiled N = in on hipBLASLt/rocBLAS, more than the g GEMMs it saves).

Documented deviation: one dropout mask per fused input (HF draws separate masks for q, k, v).
"""
from __future__ import annotations

import json
import math
import os
import re
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native, ops
from ..ops.linear import input_grad
from ..ops.optim import param_generation
from .quant import NF4Linear


@dataclass
class LoraConfig:
    r: int = 8
    lora_alpha: int = 8
    lora_dropout: float = 0.0
    target_modules: Optional[List[str]] = None
    bias: str = "none"
    task_type: str = "CAUSAL_LM"
    modules_to_save: Optional[List[str]] = None
    init_lora_weights: bool = True
    use_rslora: bool = False

    @property
    def scaling(self) -> float:
        return self.lora_alpha / (math.sqrt(self.r) if self.use_rslora else self.r)

    def to_dict(self):
        d = asdict(self)
        d["peft_type"] = "LORA"
        return d


# LoRA adapter kernels (csrc/kernels/lora.hip): dropout + down-projection in one pass over x, and
# the adapter's dX contribution accumulated in one pass over dX. GRT_LORA_KERNELS=0 -> torch path
# (or a comma list of down, dx: only those kernels).
_LORA_KERNELS_ENV = os.environ.get("GRT_LORA_KERNELS", "1")
_LORA_KINDS = ({"down", "dx"} if _LORA_KERNELS_ENV == "1" else
               set() if _LORA_KERNELS_ENV == "0" else set(_LORA_KERNELS_ENV.split(",")))
_LORA_DOWN = "down" in _LORA_KINDS
_LORA_DX = "dx" in _LORA_KINDS


def _base_weight(base: nn.Module) -> torch.Tensor:
    return base.dequantize() if isinstance(base, NF4Linear) else base.weight


def _base_input_grad(base: nn.Module, dy2: torch.Tensor, acc: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dX of the frozen base projection: TN GEMM on a transposed weight (cached for a bf16 base;
    for NF4 the dequantising kernel writes W^T directly). With ``acc`` the GEMM adds onto it in its
    epilogue (beta = 1) and returns it."""
    if isinstance(base, NF4Linear):
        return base.input_grad(dy2, acc)
    if acc is not None:
        from ..ops.linear import transposed_weight
        wt = transposed_weight(base.weight) if dy2.is_cuda and dy2.dtype == torch.bfloat16 else None
        return acc.addmm_(dy2, wt.t()) if wt is not None else acc.addmm_(dy2, base.weight)
    return input_grad(dy2, base.weight)


# The adapter's dX term first, then the base dX GEMM accumulating onto it in its epilogue (beta = 1):
# the adapter kernel only WRITES its [M, K] term, and the GEMM's read of it overlaps its MFMA work,
# instead of a separate read-modify-write pass over dX after the GEMM. GRT_LORA_DX_EPI=0 -> RMW.
_LORA_DX_EPI = os.environ.get("GRT_LORA_DX_EPI", "1") != "0"


def _adapter_then_base_dx(ctx, C, base, dy2, g, acat):
    """dX = dY W + drop'(g A) as [adapter kernel writes T] + [base GEMM T += dY W]; None when the
    adapter kernel does not apply (the caller then runs the GEMM + read-modify-write path)."""
    if not (_LORA_DX_EPI and _LORA_DX and g.is_cuda and g.dtype == acat.dtype == dy2.dtype == torch.bfloat16):
        return None
    t = torch.empty(g.shape[0], acat.shape[1], device=dy2.device, dtype=dy2.dtype)
    if not C.lora_dx(g, acat.t().contiguous(), t, ctx.p, ctx.seed, ctx.offset, False):
        return None
    return _base_input_grad(base, dy2, t)


# LoRA gradients written by the adapter GEMMs straight into the data-parallel gradient slots
# (``p._grt_slot``, parallel/ddp.py / fsdp.py) instead of returned to autograd (AccumulateGrad copy
# + the engine's copy into the flat buffer, ~450 small kernels per Llama-2-7B step); the scaling is
# folded into the GEMMs' alpha. GRT_LORA_DIRECT_GRAD=0 -> autograd accumulation.
_LORA_DIRECT_GRAD = os.environ.get("GRT_LORA_DIRECT_GRAD", "1") != "0"
_LORA_KCAT = os.environ.get("GRT_LORA_KCAT", "1") != "0"
# NF4 base WITHOUT the resident dequant cache (QLoRA's 4-bit memory: 70B on one GPU, or
# GRT_NF4_CACHE=0): the K-concatenated forward still applies, on a transient W' that each forward
# dequantises straight into its head (nf4_dequantize_into) — one bf16 write per base weight and
# use, no resident bf16 copy. GRT_NF4_STREAM_KCAT=0: the unconcatenated per-use path.
_NF4_STREAM_KCAT = os.environ.get("GRT_NF4_STREAM_KCAT", "1") != "0"
# The adapter-gradient GEMMs g_i = s dY_i B_i, dB_i = dY_i^T h'_i and dA = g^T x_d on the
# framework's one-pass kernels (csrc/kernels/lora_grad.hip: each reads its [tokens, features]
# operand once) instead of hipBLASLt's skinny tiles (2-4 reads per product). GRT_LORA_GRAD_KERNELS=0:
# library GEMMs.
_LORA_GRAD_KERNELS = os.environ.get("GRT_LORA_GRAD_KERNELS", "1") != "0"


def _bf16_cuda(*ts):
    return all(t.is_cuda and t.dtype == torch.bfloat16 for t in ts)


def _tred_into(C, a, h, out, alpha, accumulate, transpose):
    """out (+)= alpha a^T h on the one-pass token-reduction kernel; False when it does not apply."""
    return _LORA_GRAD_KERNELS and _bf16_cuda(a, h, out) and C.lora_tred(a, h, out, alpha, accumulate, transpose)


def _packed(ts):
    """(order, view) when the 2-D tensors ``ts`` (same shape[1]) lie back to back in one buffer:
    ``view`` is their row concatenation in memory order ``order`` — no copy. Else None.
    The data-parallel engines flatten parameters (and their gradient slots) contiguously, so the
    A matrices of one adapted projection are normally adjacent (in reverse registration order)."""
    if len(ts) == 1:
        return [0], ts[0]
    t0 = ts[0]
    if any(t.dim() != 2 or t.shape[1] != t0.shape[1] or t.dtype != t0.dtype or not t.is_contiguous()
           or t.untyped_storage().data_ptr() != t0.untyped_storage().data_ptr() for t in ts):
        return None
    order = sorted(range(len(ts)), key=lambda i: ts[i].data_ptr())
    for i, j in zip(order, order[1:]):
        if ts[j].data_ptr() != ts[i].data_ptr() + ts[i].numel() * ts[i].element_size():
            return None
    first = ts[order[0]]
    rows = sum(t.shape[0] for t in ts)
    return order, first.as_strided((rows, first.shape[1]), (first.shape[1], 1))


def _slot_of(p):
    sl = getattr(p, "_grt_slot", None) if _LORA_DIRECT_GRAD and p.requires_grad else None
    if sl is not None and sl.view.dtype != p.dtype:  # e.g. fp32 gradient buffers under bf16 adapters
        return None
    return sl


class _LoraFn(torch.autograd.Function):
    """y = base(x) + scaling * sum_i  B_i A_i dropout(x)  (placed at target i's output columns).

    Targets are processed in the memory order of their A matrices (``_packed``): A_cat is then a
    view of the flat parameter buffer, h's column blocks follow that order, and dA_cat = g^T x_d is
    one GEMM written into the (equally adjacent) gradient slots."""

    @staticmethod
    def forward(ctx, x, base, spec, r, scaling, p, seed, offset, *ab):
        k = len(spec)
        As, Bs = ab[:k], ab[k:]
        x2 = x.reshape(-1, x.shape[-1])
        if x2.dtype != As[0].dtype:
            x2 = x2.to(As[0].dtype)
        x2 = x2.contiguous()
        C = _native.kernels()
        w = _base_weight(base)
        bias = getattr(base, "bias", None)
        y = F.linear(x2, w, bias)
        del w
        pk = _packed(As)
        if pk is None:
            order, acat = list(range(k)), torch.cat(As, 0)
        else:
            order, acat = pk
        # h = dropout(x) A^T in one pass over x (lora.hip; split over K when there are fewer than
        # ~3 32-token workgroups per CU); x_d is kept for the dA GEMM
        # the HIP adapter kernels are bf16-only (fp32 / fp16 adapters take the GEMM + dropout path)
        bf16 = x2.dtype == torch.bfloat16 and acat.dtype == torch.bfloat16 and x2.is_cuda
        res = C.lora_down(x2, acat, p, seed, offset, p > 0) if _LORA_DOWN and bf16 and x2.shape[0] >= 256 else []
        if res:
            h = res[0]
            xd = res[1] if p > 0 else x2
        else:
            xd = C.dropout_fwd_seeded(x2, p, seed, offset) if p > 0 else x2
            h = xd @ acat.t()                               # [M, r * k]
        for j, i in enumerate(order):                       # GEMM epilogue accumulates into y
            off, n = spec[i]
            y[:, off:off + n].addmm_(h[:, j * r:(j + 1) * r], Bs[i].t(), alpha=scaling)
        ctx.base, ctx.spec, ctx.r, ctx.scaling, ctx.p, ctx.seed, ctx.offset = base, spec, r, scaling, p, seed, offset
        ctx.order = order
        ctx.xshape = x.shape
        ctx.save_for_backward(xd, h, acat, *As, *Bs)
        return y.view(*x.shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        xd, h, acat, *ab = ctx.saved_tensors
        spec, r, s, order = ctx.spec, ctx.r, ctx.scaling, ctx.order
        k = len(spec)
        As, Bs = ab[:k], ab[k:]
        C = _native.kernels()
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.dtype != acat.dtype:
            dy2 = dy2.to(acat.dtype)
        dx = None
        # g = dL/dh = s * dY_i B_i per target, into its column block (alpha = s, no scaled copy of B)
        # every column block of g is written by its GEMM with beta = 0 (no zero fill, C not read)
        g = torch.empty(dy2.shape[0], r * k, device=dy2.device, dtype=dy2.dtype)
        dBs: List[Optional[torch.Tensor]] = [None] * k
        for j, i in enumerate(order):
            off, n = spec[i]
            dyi = dy2[:, off:off + n]
            hj = h[:, j * r:(j + 1) * r]
            g[:, j * r:(j + 1) * r].addmm_(dyi, Bs[i], beta=0.0, alpha=s)
            sl = _slot_of(Bs[i])
            if sl is not None:                               # dB_i = s dY_i^T h_i into the slot
                sl.write(lambda v: v.addmm_(dyi.t(), hj, beta=0.0, alpha=s), lambda v: v.addmm_(dyi.t(), hj, alpha=s))
                sl.notify(Bs[i])
            else:
                dBs[i] = torch.mm(dyi.t(), hj).mul_(s)
        dAs: List[Optional[torch.Tensor]] = [None] * k
        aslots = [_slot_of(As[i]) for i in order]
        pk = None
        if all(sl is not None for sl in aslots) and len({sl.fresh for sl in aslots}) == 1:
            pk = _packed([sl.view for sl in aslots])
        if pk is not None and pk[0] == list(range(k)):      # slots adjacent in the same order
            dst = pk[1]
            if aslots[0].fresh:
                dst.addmm_(g.t(), xd, beta=0.0)
            else:
                dst.addmm_(g.t(), xd)
            for sl, i in zip(aslots, order):
                sl.fresh, sl.direct = False, True
                sl.notify(As[i])
        else:
            dacat = g.t() @ xd                               # [r * k, in]
            for j, i in enumerate(order):
                rows = dacat[j * r:(j + 1) * r]
                sl = aslots[j]
                if sl is not None:
                    sl.write(lambda v: v.copy_(rows), lambda v: v.add_(rows))
                    sl.notify(As[i])
                else:
                    dAs[i] = rows
        if ctx.needs_input_grad[0]:
            dx = _adapter_then_base_dx(ctx, C, ctx.base, dy2, g, acat)
        if ctx.needs_input_grad[0] and dx is None:
            dx = _base_input_grad(ctx.base, dy2)           # base dX (frozen weight)
            # dx += drop'(g A): one read-modify-write of dx (lora.hip), else GEMM + dropout backward
            bf16 = g.dtype == acat.dtype == dx.dtype == torch.bfloat16 and g.is_cuda
            if not (_LORA_DX and bf16 and C.lora_dx(g, acat.t().contiguous(), dx, ctx.p, ctx.seed, ctx.offset, True)):
                if ctx.p > 0:
                    C.dropout_bwd_seeded(g @ acat, dx, ctx.p, ctx.seed, ctx.offset, True)
                else:
                    dx.addmm_(g, acat)
        if dx is not None:
            dx = dx.view(ctx.xshape)
        return (dx, None, None, None, None, None, None, None, *dAs, *dBs)


class _LoraKcatFn(torch.autograd.Function):
    """The K-concatenated adapted projection (module doc): x is the [M, in] head of a [M, in + R]
    row buffer whose tail this op fills with h' = s * dropout(x) A_cat^T; y = [x | h'] W'^T.
    The backward keeps the epilogue form's GEMMs (base dX on the cached W^T, per-target g = s dY_i B_i):
    one [dX | g] GEMM against W' was measured slower — its N = in + R is off the library's tiles."""

    @staticmethod
    def forward(ctx, x, mod, p, seed, offset, train, *ab):
        k = len(mod.targets)
        As, Bs = ab[:k], ab[k:]
        M, K = x.shape
        r, s = mod.r, mod.scaling
        R = r * k
        C = _native.kernels()
        xw = x.as_strided((M, K + R), (K + R, 1))   # [x | h'] rows (x's storage, see ops.fused._tail)
        pk = _packed(As)
        order, acat = (list(range(k)), torch.cat(As, 0)) if pk is None else pk
        res = C.lora_down(x, acat, p, seed, offset, p > 0, h_out=xw[:, K:], hscale=s) if _LORA_DOWN else []
        if res:
            xd = res[1] if p > 0 else x
        else:
            xd = C.dropout_fwd_seeded(x.contiguous(), p, seed, offset) if p > 0 else x
            xw[:, K:].copy_((xd @ acat.t()) * s)
        y = F.linear(xw, mod._kcat_weight(order, Bs, reuse=not train))
        if not train:  # no backward will run (evaluation / generation): nothing to keep
            return y
        # a contiguous copy of h' for the dB GEMMs (rank-r slices of a 4K-wide row stride halve their speed)
        hc = xw[:, K:].contiguous()
        ctx.mod, ctx.order, ctx.p, ctx.seed, ctx.offset = mod, order, p, seed, offset
        ctx.save_for_backward(hc, xd, acat, *As, *Bs)
        return y

    @staticmethod
    def backward(ctx, dy):
        hc, xd, acat, *ab = ctx.saved_tensors
        mod, order = ctx.mod, ctx.order
        k = len(mod.targets)
        As, Bs = ab[:k], ab[k:]
        r, s = mod.r, mod.scaling
        M = hc.shape[0]
        C = _native.kernels()
        dy2 = dy.reshape(M, -1)
        if dy2.dtype != hc.dtype:
            dy2 = dy2.to(hc.dtype)
        dx = None
        g = torch.empty(M, r * k, device=dy2.device, dtype=dy2.dtype)  # dL/dh (unscaled h) = s dY_i B_i
        dBs: List[Optional[torch.Tensor]] = [None] * k
        bt = getattr(mod, "_bt", None) if _LORA_GRAD_KERNELS and _bf16_cuda(dy2, hc) else None
        # g_i = s dY_i B_i of every target in one launch (B_i^T: rows j r .. of the B^T buffer
        # lora_refresh filled in this step's forward)
        g_done = bt is not None and C.lora_g_group(
            [dy2[:, mod._spec[i][0]:mod._spec[i][0] + mod._spec[i][1]] for i in order],
            [bt[j * r:(j + 1) * r, mod._spec[i][0]:mod._spec[i][0] + mod._spec[i][1]] for j, i in enumerate(order)],
            [g[:, j * r:(j + 1) * r] for j in range(len(order))], s, False)
        # dB_i = dY_i^T h'_i of every target in one launch, into the gradient slots (or new tensors)
        db_done = False
        if _LORA_GRAD_KERNELS and _bf16_cuda(dy2, hc) and len(order) > 1:
            slots = [_slot_of(Bs[i]) for i in order]
            outs = [sl.view if sl is not None else torch.empty(mod._spec[i][1], r, device=dy2.device, dtype=dy2.dtype)
                    for sl, i in zip(slots, order)]
            db_done = C.lora_tred_group(
                [dy2[:, mod._spec[i][0]:mod._spec[i][0] + mod._spec[i][1]] for i in order],
                [hc[:, j * r:(j + 1) * r] for j in range(len(order))], outs, 1.0,
                [sl is not None and not sl.fresh for sl in slots])
            if db_done:
                for sl, o, i in zip(slots, outs, order):
                    if sl is not None:
                        sl.fresh, sl.direct = False, True
                        sl.notify(Bs[i])
                    else:
                        dBs[i] = o
        for j, i in enumerate(order):
            off, n, _ = mod._spec[i]
            dyi = dy2[:, off:off + n]
            hj = hc[:, j * r:(j + 1) * r]                    # h' = s h: dB_i = dY_i^T h'_i
            gj = g[:, j * r:(j + 1) * r]
            if not (g_done or (bt is not None and C.lora_g(dyi, bt[j * r:(j + 1) * r, off:off + n], gj, s, False))):
                gj.addmm_(dyi, Bs[i], beta=0.0, alpha=s)
            if db_done:
                continue
            sl = _slot_of(Bs[i])
            if sl is not None:
                sl.write(lambda v: _tred_into(C, dyi, hj, v, 1.0, False, False) or v.addmm_(dyi.t(), hj, beta=0.0),
                         lambda v: _tred_into(C, dyi, hj, v, 1.0, True, False) or v.addmm_(dyi.t(), hj))
                sl.notify(Bs[i])
            else:
                dBs[i] = torch.empty(n, r, device=dy2.device, dtype=dy2.dtype)
                if not _tred_into(C, dyi, hj, dBs[i], 1.0, False, False):
                    dBs[i] = torch.mm(dyi.t(), hj)
        dAs = _lora_dA(g, xd, As, order, r, C)
        if ctx.needs_input_grad[0]:
            dx = _adapter_then_base_dx(ctx, C, mod.base, dy2, g, acat)
        if ctx.needs_input_grad[0] and dx is None:
            dx = _base_input_grad(mod.base, dy2)
            bf16 = g.dtype == acat.dtype == dx.dtype == torch.bfloat16
            if not (_LORA_DX and bf16 and C.lora_dx(g, acat.t().contiguous(), dx, ctx.p, ctx.seed, ctx.offset, True)):
                if ctx.p > 0:
                    C.dropout_bwd_seeded(g @ acat, dx, ctx.p, ctx.seed, ctx.offset, True)
                else:
                    dx.addmm_(g, acat)
        return (dx, None, None, None, None, None, *dAs, *dBs)


def _lora_dA(g, xd, As, order, r, C=None):
    """dA_cat = g^T x_d, written into the (adjacent) gradient slots when the engine provides them."""
    k = len(As)
    dAs: List[Optional[torch.Tensor]] = [None] * k
    aslots = [_slot_of(As[i]) for i in order]
    pk = None
    if all(sl is not None for sl in aslots) and len({sl.fresh for sl in aslots}) == 1:
        pk = _packed([sl.view for sl in aslots])
    if pk is not None and pk[0] == list(range(k)):
        dst = pk[1]
        fresh = aslots[0].fresh
        if not (C is not None and _tred_into(C, xd, g, dst, 1.0, not fresh, True)):  # dA^T = x_d^T g
            if fresh:
                dst.addmm_(g.t(), xd, beta=0.0)
            else:
                dst.addmm_(g.t(), xd)
        for sl, i in zip(aslots, order):
            sl.fresh, sl.direct = False, True
            sl.notify(As[i])
    else:
        dacat = torch.empty(g.shape[1], xd.shape[1], device=g.device, dtype=g.dtype)
        if not (C is not None and _tred_into(C, xd, g, dacat, 1.0, False, True)):
            dacat = g.t() @ xd
        for j, i in enumerate(order):
            rows = dacat[j * r:(j + 1) * r]
            sl = aslots[j]
            if sl is not None:
                sl.write(lambda v: v.copy_(rows), lambda v: v.add_(rows))
                sl.notify(As[i])
            else:
                dAs[i] = rows
    return dAs


class LoraLinear(nn.Module):
    """base(x) + scaling * B(dropout(A(x))) for every targeted (sub-)projection of ``base``."""

    def __init__(self, base: nn.Module, targets: List[tuple], cfg: LoraConfig):
        super().__init__()
        self.base = base
        self.r = cfg.r
        self.scaling = cfg.scaling
        self.dropout_p = cfg.lora_dropout
        dev = next((t.device for t in base.buffers()), None) or next(base.parameters()).device
        dt = getattr(base, "compute_dtype", None) or next(base.parameters()).dtype
        self.in_features = base.in_features
        self.out_features = base.out_features
        self.targets = [(name, off, n) for name, off, n in targets]
        self.lora_A = nn.ParameterDict()
        self.lora_B = nn.ParameterDict()
        for name, off, n in self.targets:
            a = torch.empty(cfg.r, self.in_features, device=dev, dtype=dt)
            nn.init.kaiming_uniform_(a, a=math.sqrt(5))  # PEFT default init (B = 0)
            self.lora_A[name] = nn.Parameter(a)
            self.lora_B[name] = nn.Parameter(torch.zeros(n, cfg.r, device=dev, dtype=dt))
        self.full_cover = (len(self.targets) == 1 and self.targets[0][1] == 0 and
                           self.targets[0][2] == self.out_features)
        self._spec = [(off, n, name) for name, off, n in self.targets]
        self._wk = None     # K-concatenated weight [out, in + R] (built lazily)
        self._wk_order = None
        self._wk_key = None  # (order, B versions, optimizer generation) the tail was last built from
        self._bt = None     # [R, out]: the B blocks transposed (adapter-gradient kernel), with W'

    @property
    def kcat_pad(self) -> int:
        """R when the K-concatenated form applies (the producer then leaves R tail columns), else 0."""
        R = self.r * len(self.targets)
        b = self.base
        if not (_LORA_KCAT and self.r % 64 == 0 and self.in_features % 128 == 0 and R <= 256
                and all(n % 64 == 0 and off % 8 == 0 for _, off, n in self.targets)):
            return 0
        if isinstance(b, NF4Linear):
            ok = (getattr(b, "_cache_on", False) or _NF4_STREAM_KCAT) and b.qweight.is_cuda \
                and b.compute_dtype == torch.bfloat16 and b.blocksize == 64
        else:
            w = getattr(b, "weight", None)
            ok = w is not None and w.is_cuda and w.dtype == torch.bfloat16 and not w.requires_grad \
                and getattr(b, "bias", None) is None
        a0 = next(iter(self.lora_A.values()))
        return R if ok and a0.dtype == torch.bfloat16 else 0

    @torch.no_grad()
    def _kcat_weight(self, order, Bs, reuse: bool = False):
        """W' = [W | B_blockdiag] with the base part built once (frozen) and the B blocks of the h'
        column order ``order`` refreshed (every forward: B changes with each optimizer step)."""
        K, r = self.in_features, self.r
        R = r * len(self.targets)
        if isinstance(self.base, NF4Linear) and not getattr(self.base, "_cache_on", False):
            return self._kcat_weight_streamed(order, Bs)
        if self._wk is None:
            w = self.base.dequantize() if isinstance(self.base, NF4Linear) else self.base.weight.detach()
            wk = torch.zeros(self.out_features, K + R, device=w.device, dtype=w.dtype)
            wk[:, :K].copy_(w)
            self._wk = wk
            if isinstance(self.base, NF4Linear):  # W' replaces the forward dequant cache (dX keeps W^T's)
                self.base._w_cache = None
            else:
                # the frozen bf16 weight becomes a view of W'[:, :K]: its own storage is released, so
                # the projection is held once (W') plus its W^T, not three times
                del w
                self.base.weight.data = wk[:, :K]
        if self._wk_order != list(order):  # block positions moved: clear the whole tail once
            self._wk[:, K:].zero_()
            self._wk_order = list(order)
            self._wk_key = None
        bl = [Bs[i].detach() for i in order]
        # Forwards without autograd (``reuse``: evaluation, generation) reuse the tail while B is
        # unchanged: same tensors, same version counters, no framework optimizer step since (the
        # fused kernels write through raw pointers: ops.optim.param_generation). A forward that
        # records a graph always refreshes and drops the key, so a training step never trusts it.
        key = (tuple(order), tuple((b.data_ptr(), b._version) for b in bl), param_generation())
        if reuse and self._wk_key == key:
            return self._wk
        self._wk_key = key if reuse else None
        offs = [self._spec[i][0] for i in order]
        if all(b.is_contiguous() for b in bl):
            # B^T [R, out] for the adapter-gradient kernel (lora_grad.hip lora_g): block j = B_{order[j]}^T
            if _LORA_GRAD_KERNELS and r == 64 and self._wk.is_cuda:
                if self._bt is None:
                    self._bt = torch.zeros(R, self.out_features, device=self._wk.device, dtype=self._wk.dtype)
                _native.kernels().lora_refresh(bl, offs, self._wk, self._bt, K, 0)
            else:
                _native.kernels().lora_refresh(bl, offs, self._wk, None, K)
        else:
            self._bt = None
            for j, (b, off) in enumerate(zip(bl, offs)):
                self._wk[off:off + b.shape[0], K + j * r:K + (j + 1) * r].copy_(b)
        return self._wk

    @torch.no_grad()
    def _kcat_weight_streamed(self, order, Bs):
        """W' for an NF4 base without the dequant cache: a fresh [out, in + R] buffer per forward, W
        dequantised into its head, the B blocks (and the B^T buffer of the adapter-gradient kernel)
        into the tail. Nothing bf16 of the base outlives the forward's GEMM."""
        K, r = self.in_features, self.r
        R = r * len(self.targets)
        q = self.base.qweight
        wk = torch.empty(self.out_features, K + R, device=q.device, dtype=torch.bfloat16)
        self.base.dequantize_into(wk[:, :K])
        wk[:, K:].zero_()
        bl = [Bs[i].detach() for i in order]
        offs = [self._spec[i][0] for i in order]
        if all(b.is_contiguous() for b in bl):
            if _LORA_GRAD_KERNELS and r == 64:
                if self._bt is None or self._wk_order != list(order):
                    self._bt = torch.zeros(R, self.out_features, device=q.device, dtype=torch.bfloat16)
                    self._wk_order = list(order)
                _native.kernels().lora_refresh(bl, offs, wk, self._bt, K, 0)
            else:
                _native.kernels().lora_refresh(bl, offs, wk, None, K)
        else:
            self._bt = None
            for j, (b, off) in enumerate(zip(bl, offs)):
                wk[off:off + b.shape[0], K + j * r:K + (j + 1) * r].copy_(b)
        return wk

    @torch.no_grad()
    def prepare_frozen_weights(self):
        """Materialise the frozen base's derived layouts now, while the model is prepared, instead of
        inside the first training step: the K-concatenated W' (or, without it, the NF4 dequant cache
        W) and the W^T of the TN dX GEMM. The base is frozen, so each is built exactly once either
        way; this only moves the one-time build (and its HBM allocations) out of ``train()``."""
        b = self.base
        w = getattr(b, "qweight", None) if isinstance(b, NF4Linear) else getattr(b, "weight", None)
        if w is None or not w.is_cuda:
            return
        names = [t[0] for t in self.targets]
        streamed = isinstance(b, NF4Linear) and not getattr(b, "_cache_on", False)
        if self.kcat_pad and not streamed:
            pk = _packed([self.lora_A[n] for n in names])
            self._kcat_weight(list(range(len(names))) if pk is None else pk[0], [self.lora_B[n] for n in names])
        elif isinstance(b, NF4Linear) and not streamed:
            b.dequantize()
        if isinstance(b, NF4Linear):
            b.prepare_input_grad()
        elif w.dtype == torch.bfloat16:
            from ..ops.linear import transposed_weight
            transposed_weight(w)

    def direct_grad_params(self) -> List[nn.Parameter]:
        """Parameters whose gradient the GPU backward writes into the engine's slot itself."""
        return list(self.lora_A.values()) + list(self.lora_B.values())

    def forward(self, x):
        if x.is_cuda:
            p = self.dropout_p if self.training else 0.0
            seed, offset = ops.fused.dropout_seed_offset(x) if p > 0 else (0, 0)
            names = [t[0] for t in self.targets]
            R = self.r * len(names)
            if (getattr(x, "_grt_tail", 0) == R and R and x.dim() == 2 and x.stride(1) == 1
                    and x.stride(0) == self.in_features + R and self.kcat_pad == R):
                ab = [self.lora_A[n] for n in names] + [self.lora_B[n] for n in names]
                train = torch.is_grad_enabled() and (x.requires_grad or any(t.requires_grad for t in ab))
                return _LoraKcatFn.apply(x, self, p, seed, offset, train, *ab)
            spec = [(off, n) for _, off, n in self.targets]
            return _LoraFn.apply(x, self.base, spec, self.r, self.scaling, p, seed, offset,
                                 *[self.lora_A[n] for n in names], *[self.lora_B[n] for n in names])
        y = self.base(x)
        xd = ops.dropout(x, self.dropout_p, self.training) if self.dropout_p > 0 else x
        names = [t[0] for t in self.targets]
        a = torch.cat([self.lora_A[n] for n in names], 0) if len(names) > 1 else self.lora_A[names[0]]
        h = F.linear(xd, a) * self.scaling                      # [T, r * k]
        if self.full_cover:
            return y + F.linear(h, self.lora_B[names[0]])
        # block-diagonal B placed at each target's output columns
        bfull = h.new_zeros(self.out_features, self.r * len(names))
        for i, (n, off, cnt) in enumerate(self.targets):
            bfull = bfull.index_copy(0, torch.arange(off, off + cnt, device=h.device),
                                     F.pad(self.lora_B[n], (i * self.r, (len(names) - 1 - i) * self.r)))
        return y + F.linear(h, bfull)

    @torch.no_grad()
    def merged_weight(self) -> torch.Tensor:
        w = self.base.dequantize() if isinstance(self.base, NF4Linear) else self.base.weight.detach().clone()
        w = w.clone()
        for n, off, cnt in self.targets:
            w[off:off + cnt] += (self.lora_B[n].float() @ self.lora_A[n].float() * self.scaling).to(w.dtype)
        return w


_ALL_PROJ = ["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"]


def _targets_for(module_name: str, mod: nn.Module, wanted: List[str]):
    slices = getattr(mod, "slices", None)
    if slices:
        out, off = [], 0
        for sub, n in slices:
            if sub in wanted:
                out.append((sub, off, n))
            off += n
        return out
    leaf = module_name.rsplit(".", 1)[-1]
    if leaf in wanted:
        return [(leaf, 0, mod.out_features)]
    return []


class PeftModel(nn.Module):
    def __init__(self, model: nn.Module, cfg: LoraConfig):
        super().__init__()
        self.base_model = model
        self.peft_config = {"default": cfg}
        wanted = cfg.target_modules or _ALL_PROJ
        if isinstance(wanted, str):
            wanted = [m for m in _ALL_PROJ if re.fullmatch(wanted, m)]
        for p in model.parameters():
            p.requires_grad_(False)
        self.lora_modules: Dict[str, LoraLinear] = {}
        for name, parent in list(model.named_modules()):
            for cname, child in list(parent.named_children()):
                full = f"{name}.{cname}" if name else cname
                if isinstance(child, (nn.Linear, NF4Linear)) and not full.endswith("lm_head"):
                    tg = _targets_for(full, child, wanted)
                    if tg:
                        lw = LoraLinear(child, tg, cfg)
                        setattr(parent, cname, lw)
                        self.lora_modules[full] = lw
        if cfg.modules_to_save:
            for n, p in model.named_parameters():
                if any(m in n for m in cfg.modules_to_save):
                    p.requires_grad_(True)
        if not self.lora_modules:
            raise ValueError(f"no module matched target_modules={wanted}")

    @property
    def config(self):
        return self.base_model.config

    def forward(self, *a, **k):
        return self.base_model(*a, **k)

    def generate(self, *a, **k):
        from ..models.generation import generate
        return generate(self.base_model, *a, **k)

    def trainable_parameters(self):
        return [p for p in self.parameters() if p.requires_grad]

    def prepare_frozen_weights(self):
        """See ``LoraLinear.prepare_frozen_weights`` (called by the trainers at construction)."""
        for m in self.lora_modules.values():
            m.prepare_frozen_weights()
        head = getattr(self.base_model, "lm_head", None)
        w = getattr(head, "weight", None)
        if w is not None and w.is_cuda and w.dtype == torch.bfloat16 and not w.requires_grad:
            from ..ops.linear import transposed_weight
            transposed_weight(w)  # the fused LM-head cross-entropy's dX GEMM

    def print_trainable_parameters(self):
        t = sum(p.numel() for p in self.parameters() if p.requires_grad)
        tot = sum(p.numel() for p in self.parameters()) + sum(
            m.base.in_features * m.base.out_features for m in self.lora_modules.values() if isinstance(m.base, NF4Linear))
        print(f"trainable params: {t:,} || all params: {tot:,} || trainable%: {100 * t / max(tot, 1):.4f}")
        return t, tot

    # ------------------------------------------------------------------ adapters on disk
    def adapter_state_dict(self) -> Dict[str, torch.Tensor]:
        out = {}
        for full, m in self.lora_modules.items():
            base = full.rsplit(".", 1)[0] if getattr(m.base, "slices", None) else full
            for sub, _, _ in m.targets:
                key = f"{base}.{sub}" if getattr(m.base, "slices", None) else full
                out[f"base_model.model.{key}.lora_A.weight"] = m.lora_A[sub].detach().contiguous()
                out[f"base_model.model.{key}.lora_B.weight"] = m.lora_B[sub].detach().contiguous()
        return out

    def load_adapter_state_dict(self, sd: Dict[str, torch.Tensor]):
        with torch.no_grad():
            for full, m in self.lora_modules.items():
                base = full.rsplit(".", 1)[0] if getattr(m.base, "slices", None) else full
                for sub, _, _ in m.targets:
                    key = f"{base}.{sub}" if getattr(m.base, "slices", None) else full
                    m.lora_A[sub].copy_(sd[f"base_model.model.{key}.lora_A.weight"])
                    m.lora_B[sub].copy_(sd[f"base_model.model.{key}.lora_B.weight"])

    def save_pretrained(self, path: str):
        from safetensors.torch import save_file
        os.makedirs(path, exist_ok=True)
        save_file({k: v.cpu() for k, v in self.adapter_state_dict().items()},
                  os.path.join(path, "adapter_model.safetensors"))
        self.save_adapter_config(path)

    def save_adapter_config(self, path: str):
        os.makedirs(path, exist_ok=True)
        cfg = self.peft_config["default"].to_dict()
        cfg["base_model_name_or_path"] = getattr(self.config, "name", "llama")
        with open(os.path.join(path, "adapter_config.json"), "w") as f:
            json.dump(cfg, f, indent=2)

    def load_adapter(self, path: str):
        from safetensors.torch import load_file
        self.load_adapter_state_dict(load_file(os.path.join(path, "adapter_model.safetensors")))

    # ------------------------------------------------------------------ merge
    @torch.no_grad()
    def merge_and_unload(self) -> nn.Module:
        """W <- W + scaling * B A for every adapter (NF4 bases are dequantised to bf16 first);
        returns the plain base model with ordinary (ops.Linear) projections."""
        from ..ops.linear import Linear
        model = self.base_model
        for full, m in list(self.lora_modules.items()):
            w = m.merged_weight()
            parent_name, cname = full.rsplit(".", 1) if "." in full else ("", full)
            parent = model.get_submodule(parent_name) if parent_name else model
            lin = Linear(m.in_features, m.out_features, bias=False, device=w.device, dtype=w.dtype)
            lin.weight.copy_(w)
            if getattr(m.base, "slices", None):
                from ..models.llama import FusedLinear
                fl = FusedLinear(m.in_features, m.base.slices, device=w.device, dtype=w.dtype)
                fl.weight.copy_(w)
                lin = fl
            setattr(parent, cname, lin)
        for name, parent in list(model.named_modules()):  # remaining (non-adapted) NF4 layers
            for cname, child in list(parent.named_children()):
                if isinstance(child, NF4Linear):
                    w = child.dequantize()
                    slices = getattr(child, "slices", None)
                    if slices:
                        from ..models.llama import FusedLinear
                        lin = FusedLinear(child.in_features, slices, device=w.device, dtype=w.dtype)
                    else:
                        lin = Linear(child.in_features, child.out_features, bias=False, device=w.device, dtype=w.dtype)
                    lin.weight.copy_(w)
                    setattr(parent, cname, lin)
        self.lora_modules = {}
        return model


def get_peft_model(model: nn.Module, cfg: LoraConfig) -> PeftModel:
    return PeftModel(model, cfg)


def prepare_model_for_kbit_training(model: nn.Module, use_gradient_checkpointing: bool = True):
    for p in model.parameters():
        p.requires_grad_(False)
    if use_gradient_checkpointing and hasattr(model, "gradient_checkpointing_enable"):
        model.gradient_checkpointing_enable()
    return model
