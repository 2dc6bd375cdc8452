"""Linear layer whose weight gradient is written by the GEMM straight into the DDP/FSDP bucket.

Torch's autograd produces a fresh dW tensor per backward and AccumulateGrad then adds it into
``param.grad`` — with gradient-as-bucket-view DDP that is an extra read+read+write of every
weight gradient per step plus a memset of the whole gradient buffer in ``zero_grad``
(profiles/r1_bench1gpu_kernel_stats.md: ~2.5 % of a Llama-2-7B step). Here the backward GEMM
writes dW into its slot of the flat gradient buffer directly: ``beta = 0`` on the first
contribution of a step (no zeroing pass needed) and ``beta = 1`` — hipBLASLt's in-epilogue
accumulation — on later gradient-accumulation micro-steps. The data-parallel engine is then
notified exactly like a post-accumulate-grad hook so bucketed all-reduce overlap is unchanged.

The engine attaches ``param._grt_slot = GradSlot(view, notify)``; without it this is F.linear.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F


class GradSlot:
    """A parameter's slot in a flat gradient buffer.

    ``direct`` marks that the backward GEMM wrote this step's contribution itself. Torch still
    fires the parameter's post-accumulate-grad hook for that input (with no gradient), so the
    engines' hooks consume the flag and skip that event instead of counting the parameter twice.
    """
    __slots__ = ("view", "fresh", "notify", "direct")

    def __init__(self, view: torch.Tensor, notify):
        self.view = view
        self.fresh = True
        self.notify = notify
        self.direct = False

    def write(self, fn_out, fn_acc):
        if self.fresh:
            fn_out(self.view)
            self.fresh = False
        else:
            fn_acc(self.view)
        self.direct = True

    def consume_direct(self) -> bool:
        if self.direct:
            self.direct = False
            return True
        return False


_WGRAD_NATIVE = os.environ.get("GRT_WGRAD_GEMM", "1") != "0"
# weight gradients as transposes + TN library GEMM (see wgrad); GRT_WGRAD_TN=0 -> MFMA kernel
_WGRAD_TN = os.environ.get("GRT_WGRAD_TN", "1") != "0"


# dX = dY W through the TN library kernel on a contiguous W^T (13-15 % faster than the NN form on
# the Llama projection shapes in isolation, profiles/r1_dgrad_layout_ab.jsonl). Frozen weights
# (LoRA / QLoRA base) get it for free: +2.3 % LoRA end to end (profiles/r1_transposed_dgrad_ab.txt).
# Trainable weights need a fresh W^T every step; the per-step transpose cancels the gain on the
# full fine-tune, so that path is opt-in (GRT_TRANSPOSED_DGRAD_TRAINABLE=1) — except for weights the
# engine marks ``_grt_fwd_transpose`` (ZeRO, whose sharded update cannot write W^T: there the
# forward-time transpose is +1.7 % over the NN dX GEMM, profiles/r2_zero_fwd_transpose_proxy.txt).
_TRANSPOSED_DGRAD = os.environ.get("GRT_TRANSPOSED_DGRAD", "1") != "0"
_TRANSPOSED_DGRAD_TRAINABLE = os.environ.get("GRT_TRANSPOSED_DGRAD_TRAINABLE", "0") == "1"


def transposed_weight(w: torch.Tensor):
    """Contiguous W^T, cached on the weight tensor while its contents are unchanged (keyed by
    storage pointer and version counter). Frozen weights (LoRA / QLoRA base, a PEFT LM head) are
    transposed once; trainable weights only use copies the data-parallel engine refreshes after
    each optimizer step (``register_transposed``), otherwise None."""
    ent = getattr(w, "_grt_wt", None)
    key = (w.data_ptr(), w._version)
    if ent is not None and ent[0] == key:
        return ent[1]
    if w.requires_grad:
        return None
    wt = w.detach().t().contiguous()
    w._grt_wt = (key, wt)
    return wt


def register_transposed(w: torch.Tensor, wt: torch.Tensor) -> None:
    """Record ``wt`` (already holding W^T) as the valid transposed copy of the current ``w``."""
    w._grt_wt = ((w.data_ptr(), w._version), wt)


_side_streams = {}


def _side_stream(dev) -> "torch.cuda.Stream":
    s = _side_streams.get(dev)
    if s is None:
        s = _side_streams[dev] = torch.cuda.Stream(dev)
    return s


def transpose_for_backward(w: torch.Tensor):
    """Trainable data-parallel weight at forward time: write W^T into a persistent buffer on a side
    stream (HIP transpose kernel, HBM-bound, overlapping the forward GEMMs) and return (W^T, event)
    for the backward's TN input-gradient GEMM; None where it does not apply (FSDP-managed or
    unaligned weights, non-bf16)."""
    fsdp_t = getattr(w, "_grt_fsdp_fwd_transpose", False)  # FSDP: W^T of the gathered weight
    if not (_TRANSPOSED_DGRAD and (_TRANSPOSED_DGRAD_TRAINABLE or getattr(w, "_grt_fwd_transpose", False) or fsdp_t)
            and w.is_cuda and w.dtype == torch.bfloat16
            and w.dim() == 2
            and w.shape[0] % 64 == 0 and w.shape[1] % 64 == 0 and getattr(w, "_grt_slot", None) is not None
            and (getattr(w, "_grt_unit", None) is None or fsdp_t) and w.is_contiguous()):
        return None
    from .. import _native
    buf = getattr(w, "_grt_wt_buf", None)
    if buf is None or buf.shape != (w.shape[1], w.shape[0]):
        buf = torch.empty(w.shape[1], w.shape[0], device=w.device, dtype=w.dtype)
        w._grt_wt_buf = buf
    side = _side_stream(w.device)
    side.wait_stream(torch.cuda.current_stream(w.device))
    with torch.cuda.stream(side):
        _native.kernels().transpose_into(w.detach(), buf)
        ev = torch.cuda.Event()
        ev.record(side)
    if fsdp_t:  # the gathered weight's buffer goes back to FSDP's pool after the unit's forward:
        w._grt_wt_pending = ev  # FSDP's _unbind orders that release after this read
    return buf, ev


def input_grad(dy2: torch.Tensor, w: torch.Tensor, wt_ev=None) -> torch.Tensor:
    """dX = dY W ([.., N] x [N, K]): F.linear(dY, W^T) when a transposed copy is available
    (``wt_ev`` from transpose_for_backward, or the cached copy of a frozen weight)."""
    if wt_ev is not None:
        wt, ev = wt_ev
        torch.cuda.current_stream(dy2.device).wait_event(ev)
        return F.linear(dy2, wt)
    if _TRANSPOSED_DGRAD and dy2.is_cuda and dy2.dtype == torch.bfloat16 and w.dim() == 2:
        wt = transposed_weight(w)
        if wt is not None:
            return F.linear(dy2, wt)
    return dy2 @ w
# Opt-in: the one-pass backward gives each vocabulary row to one wave, which serialises on the
# hottest tokens of a Zipf-distributed batch (measured +6.5 ms per Llama-2-7B step vs torch's
# partial-segment scheme, an A/B run, profiles/r1_embedding_ab.txt); the forward gather and the uniform-id case are fine.
_NATIVE_EMBEDDING = os.environ.get("GRT_NATIVE_EMBEDDING", "0") == "1"


# Where the two transposes of the TN weight gradient run (opt-in placements). GRT_WGRAD_XT_FWD=1:
# the inputs X of a projection are transposed in the FORWARD, right after the kernel that produced
# them (norm, SwiGLU, attention) while they may still sit in the 256 MB Infinity Cache, and X^T is
# saved for the backward instead of X; GRT_WGRAD_DYT_FIRST=1: dY^T at the top of the backward,
# right after its producer. Measured on the headline step (3 interleaved rounds, scripts/gpu_r4_xt.sh,
# profiles/r4_batch1.md): 298.4-298.7 / 298.3-298.9 ms vs 298.7-298.9 ms with the transposes inside
# ``wgrad`` — no cache benefit, +2 GiB peak (the attention output is saved twice), so both stay off.
_WGRAD_XT_FWD = os.environ.get("GRT_WGRAD_XT_FWD", "0") == "1"
_WGRAD_DYT_FIRST = os.environ.get("GRT_WGRAD_DYT_FIRST", "0") == "1"


def _tn_wgrad_ok(t2: torch.Tensor) -> bool:
    """``t2`` ([M, C] token-major) can be an operand of the transposed (TN) weight-gradient path."""
    return (_WGRAD_NATIVE and _WGRAD_TN and t2.is_cuda and t2.dtype == torch.bfloat16 and t2.dim() == 2
            and t2.shape[0] % 64 == 0 and t2.shape[1] % 64 == 0 and t2.is_contiguous())


def transposed(t2: torch.Tensor) -> torch.Tensor:
    """[M, C] -> contiguous [C, M] through the HIP transpose kernel (HBM / cache-bound)."""
    from .. import _native
    tt = torch.empty(t2.shape[1], t2.shape[0], device=t2.device, dtype=t2.dtype)
    _native.kernels().transpose_into(t2, tt)
    return tt


def provided_transposed(t2: torch.Tensor, t: torch.Tensor):
    """The contiguous [C, M] transpose of ``t2`` ([M, C], a 2-D view of ``t``) that the kernel which
    produced ``t`` wrote beside it (``t._grt_T``), or None. Taken once: the attribute is cleared, so
    the copy lives only as long as its consumer keeps it."""
    tt = getattr(t, "_grt_T", None)
    if tt is None:
        return None
    try:
        del t._grt_T
    except AttributeError:
        pass
    if (tt.dim() == 2 and tt.shape[0] == t2.shape[1] and tt.shape[1] == t2.shape[0] and tt.is_contiguous()
            and tt.dtype == t2.dtype == torch.bfloat16 and _WGRAD_NATIVE and _WGRAD_TN
            and t2.shape[0] % 64 == 0 and t2.shape[1] % 64 == 0):
        return tt
    return None


def wgrad_tn(dyt: torch.Tensor, xt: torch.Tensor, out: torch.Tensor, accumulate: bool) -> torch.Tensor:
    """dW = dY^T X from the already transposed operands ([N, M], [K, M]): the TN library GEMM."""
    if accumulate:
        out.addmm_(dyt, xt.t())
    else:
        torch.mm(dyt, xt.t(), out=out)
    return out


def wgrad(dy2: torch.Tensor, x2: torch.Tensor, out: torch.Tensor = None, accumulate: bool = False) -> torch.Tensor:
    """dW = dy2^T @ x2 ([M,N]^T [M,K] -> [N,K]), written into / accumulated onto ``out``.

    bf16 on MI355X runs the hand-written MFMA kernel (csrc/kernels/gemm.hip) when the shape tiles
    (N, K multiples of 256, M of 64); anything else goes to hipBLASLt through torch.
    """
    dy2 = dy2.reshape(-1, dy2.shape[-1])
    x2 = x2.reshape(-1, x2.shape[-1])
    if out is None:
        out = torch.empty(dy2.shape[1], x2.shape[1], device=dy2.device, dtype=dy2.dtype)
        accumulate = False
    if _WGRAD_NATIVE and dy2.is_cuda and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16 \
            and out.dtype == torch.bfloat16:
        from .. import _native
        C = _native.kernels()
        M, N, K = dy2.shape[0], dy2.shape[1], x2.shape[1]
        if (_WGRAD_TN and M % 64 == 0 and N % 64 == 0 and K % 64 == 0
                and dy2.is_contiguous() and x2.is_contiguous() and out.is_contiguous()):
            # token-major operands are the layout every GEMM handles worst (~1.1 PF): transpose
            # both (HIP, HBM-bound) and run the TN library GEMM on the reduction-contiguous copies
            # with its offline-tuned solutions (tools/tune_wgrad_tn.py; untuned microbench incl.
            # the transposes, tools/wgrad_transpose_ab.py: qkv 714 -> 617 us, o 242 -> 221, gate_up
            # 1362 -> 1287, LM head 1880 -> 1594; profiles/r2_perf_experiments.md)
            dyt = torch.empty(N, M, device=dy2.device, dtype=dy2.dtype)
            xt = torch.empty(K, M, device=x2.device, dtype=x2.dtype)
            C.transpose_into(dy2, dyt)
            C.transpose_into(x2, xt)
            if accumulate:
                out.addmm_(dyt, xt.t())
            else:
                torch.mm(dyt, xt.t(), out=out)
            return out
        if C.gemm_wgrad(dy2, x2, out, accumulate):
            return out
    if accumulate:
        out.addmm_(dy2.t(), x2)
    else:
        torch.mm(dy2.t(), x2, out=out)
    return out


class _DirectGradLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        # X^T written by the producing kernel (ops.fused.swiglu: the down projection's input)
        xt = provided_transposed(x2, x) if ctx.needs_input_grad[1] else None
        ctx.x_t = xt is not None and w.shape[0] % 64 == 0 and _tn_wgrad_ok(x2)
        if not ctx.x_t and _WGRAD_XT_FWD and ctx.needs_input_grad[1] and w.shape[0] % 64 == 0 and _tn_wgrad_ok(x2):
            ctx.x_t, xt = True, transposed(x2)
        ctx.save_for_backward(xt if ctx.x_t else x, w)
        ctx.has_b = b is not None
        ctx.wt_ev = transpose_for_backward(w) if ctx.needs_input_grad[0] else None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        # dY^T written by the producing kernel (ops.fused.swiglu backward: the gate / up gradient)
        dyt = provided_transposed(dy2, dy) if ctx.needs_input_grad[1] else None
        if dyt is not None and not ctx.x_t:  # X was saved untransposed: its transpose now
            x2 = x.reshape(-1, x.shape[-1])
            if _tn_wgrad_ok(x2) and w.shape[0] % 64 == 0:
                x = transposed(x2)
                ctx.x_t = True
            else:  # X cannot take the TN path (dtype / shape / layout): plain weight gradient
                dyt = None
        if ctx.x_t and dyt is None:  # X^T saved by the forward: dY^T now, while dY is fresh from its producer
            if not dy2.is_contiguous():
                dy2 = dy2.contiguous()
            dyt = transposed(dy2) if _WGRAD_DYT_FIRST else None
        dx = None
        if ctx.needs_input_grad[0]:
            dx = input_grad(dy, w, ctx.wt_ev)
            ctx.wt_ev = None
        dw = db = None
        if ctx.x_t:
            xt = x
            if dyt is None:
                dyt = transposed(dy2)
            fn = lambda v, acc: wgrad_tn(dyt, xt, v, acc)  # noqa: E731
        else:
            x2 = x.reshape(-1, x.shape[-1])
            fn = lambda v, acc: wgrad(dy2, x2, v, acc)  # noqa: E731
        if ctx.needs_input_grad[1]:
            slot = getattr(w, "_grt_slot", None)
            if slot is not None:
                slot.write(lambda v: fn(v, False), lambda v: fn(v, True))
                slot.notify(w)
            else:
                dw = torch.empty_like(w)
                fn(dw, False)
        if ctx.has_b:
            b_needs = ctx.needs_input_grad[2]
            if b_needs:
                db = dy2.sum(0)
        return dx, dw, db


_GEMV = os.environ.get("GRT_GEMV", "1") != "0"
# rows up to which the decode GEMV beats the library GEMM (Llama-3.1-8B decode, HIP graph: batch 1
# 285 vs 210 tok/s, batch 4 688 vs 793, batch 8 746 vs 1506 — profiles/r2_decode_batch_gemv.txt:
# the activations, re-read by every wave, and the per-row FMAs outgrow the weight stream)
GEMV_MAX_ROWS = int(os.environ.get("GRT_GEMV_MAX_ROWS", "2"))
# 3-8 rows with K % 256 == 0: the MFMA skinny kernel (gemv.hip gemv_mfma_kernel; the kernel takes up
# to 16). Llama-3.1-8B graph decode vs the library GEMM: batch 4 870 vs 795 tokens/s, batch 8 1564
# vs 1539, batch 16 2536 vs 2729 (profiles/r5_decode.md) — so the library keeps 9+ rows
GEMV_MFMA_MAX_ROWS = int(os.environ.get("GRT_GEMV_MFMA_MAX_ROWS", "8"))


def _gemv_rows_ok(rows: int, K: int) -> bool:
    return rows <= GEMV_MAX_ROWS or (rows <= GEMV_MFMA_MAX_ROWS and K % 256 == 0)


def linear(x, weight, bias=None):
    if weight.requires_grad and getattr(weight, "_grt_slot", None) is not None and torch.is_grad_enabled():
        return _DirectGradLinear.apply(x, weight, bias)
    K = weight.shape[-1]
    if (_GEMV and x.is_cuda and not torch.is_grad_enabled() and x.dtype == torch.bfloat16
            and weight.dtype == torch.bfloat16 and weight.dim() == 2 and weight.is_contiguous()
            and _gemv_rows_ok(x.numel() // K, K) and K % 8 == 0 and x.shape[-1] == K):
        # decode: 1-2 tokens per step are a weight stream -> HBM-bound GEMV kernel (gemv.hip)
        from .. import _native
        x2 = x.reshape(-1, K)
        if x2.stride(-1) == 1 and x2.stride(0) % 8 == 0 and x2.data_ptr() % 16 == 0 and weight.data_ptr() % 16 == 0:
            y = _native.kernels().gemv(x2, weight)
            if bias is not None:
                y = y + bias
            return y.view(*x.shape[:-1], weight.shape[0])
    return F.linear(x, weight, bias)


class Linear(nn.Linear):
    """nn.Linear (same parameters / state_dict) routed through ``ops.linear``.

    ``layer(x, labels=t)`` is the fused LM-head + cross-entropy (``ops.lm_head_cross_entropy``)
    instead of logits; going through ``__call__`` keeps module hooks (e.g. the ZeRO parameter
    gather wait of parallel/ddp.py) firing for the head's weight.
    """

    def forward(self, x, labels=None, ignore_index: int = -100, row_weights=None):
        if labels is not None:
            from .fused import lm_head_cross_entropy
            return lm_head_cross_entropy(x, self.weight, labels, bias=self.bias, ignore_index=ignore_index,
                                         row_weights=row_weights)
        return linear(x, self.weight, self.bias)


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w):
        from .. import _native
        ctx.save_for_backward(ids)
        ctx.wshape = w.shape
        ctx.w = w
        return _native.kernels().embedding_fwd(ids.reshape(-1).contiguous(), w).view(*ids.shape, w.shape[1])

    @staticmethod
    def backward(ctx, dy):
        from .. import _native
        (ids,) = ctx.saved_tensors
        C = _native.kernels()
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        w = ctx.w
        slot = getattr(w, "_grt_slot", None)
        if slot is not None:  # write dW straight into the data-parallel gradient buffer
            slot.write(lambda v: C.embedding_bwd(dy2, ids, v, False), lambda v: C.embedding_bwd(dy2, ids, v, True))
            slot.notify(w)
            return None, None
        dw = torch.empty(ctx.wshape, device=dy.device, dtype=dy.dtype)
        C.embedding_bwd(dy2, ids, dw, False)
        return None, dw


def embedding(ids, weight):
    """Token embedding: HIP gather forward + one-pass segmented backward on MI355X (bf16/fp32)."""
    if _NATIVE_EMBEDDING and weight.is_cuda and weight.dtype in (torch.bfloat16, torch.float32) \
            and weight.shape[1] % 8 == 0:
        if weight.requires_grad and torch.is_grad_enabled():
            return _Embedding.apply(ids, weight)
        from .. import _native
        return _native.kernels().embedding_fwd(ids.reshape(-1).contiguous(), weight).view(*ids.shape, weight.shape[1])
    return F.embedding(ids, weight)


class Embedding(nn.Embedding):
    """nn.Embedding (same parameter / state_dict) routed through ``ops.embedding``."""

    def forward(self, ids):
        if self.padding_idx is not None or self.max_norm is not None or self.sparse:
            return super().forward(ids)
        return embedding(ids, self.weight)
