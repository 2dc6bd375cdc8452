"""Autograd wrappers around the gfx950 HIP kernels.

Every op dispatches on the tensor's device: GPU tensors ALWAYS go to the native kernel (a
missing ``_C.so`` raises, see ``_native.py``); CPU tensors use ``_ref`` so the whole framework
(models, DDP over gloo, trainers) runs and is tested on CPU-only hosts.
"""
from __future__ import annotations

import math
import os

import torch

from .. import _native
from . import _ref
from .linear import input_grad, transpose_for_backward, wgrad


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ----------------------------------------------------------------------------- RMSNorm
def _tail(y, pad):
    """Mark a producer output written into a [rows, d + pad] row buffer: the consumer (a
    K-concatenated LoRA projection, peft/lora.py) may fill the ``pad`` tail columns."""
    if pad:
        y._grt_tail = pad
    return y


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps, pad=0):
        C = _native.kernels()
        xc = x.contiguous()
        y, _, rstd = C.rmsnorm_fwd(xc, None, w.contiguous(), eps, pad)
        ctx.save_for_backward(xc, w, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, rstd = ctx.saved_tensors
        if not ctx.needs_input_grad[1]:  # frozen weight (LoRA / QLoRA): dX only
            return _native.kernels().rmsnorm_bwd_dx(dy.contiguous(), x, w, rstd, None), None, None, None
        dx, dw = _norm_bwd_into_slot(w, lambda out, acc: _native.kernels().rmsnorm_bwd(
            dy.contiguous(), x, w, rstd, None, out, acc))
        return dx, dw, None, None


_NORM_DIRECT_GRAD = os.environ.get("GRT_NORM_DIRECT_GRAD", "1") != "0"


def _norm_bwd_into_slot(w, run):
    """RMSNorm backward whose weight gradient the kernel writes in the parameter dtype straight into
    the data-parallel gradient slot (``w._grt_slot``, parallel/ddp.py / fsdp.py) -> (dx, None);
    without a slot -> (dx, dw)."""
    slot = getattr(w, "_grt_slot", None) if _NORM_DIRECT_GRAD else None
    if slot is None or not w.requires_grad or slot.view.dtype != w.dtype:
        dx, dw = run(None, False)
        return dx, dw.to(w.dtype)
    res = []
    slot.write(lambda v: res.append(run(v, False)[0]), lambda v: res.append(run(v, True)[0]))
    slot.notify(w)
    return res[0], None


class _AddRMSNorm(torch.autograd.Function):
    """h = x + residual ; y = rmsnorm(h) * w  -> (y, h), residual add fused into the norm."""

    @staticmethod
    def forward(ctx, x, residual, w, eps, pad=0):
        C = _native.kernels()
        y, h, rstd = C.rmsnorm_fwd(x.contiguous(), residual.contiguous(), w.contiguous(), eps, pad)
        ctx.save_for_backward(h, w, rstd)
        return y, h

    @staticmethod
    def backward(ctx, dy, dh):
        h, w, rstd = ctx.saved_tensors
        dy = torch.zeros_like(h) if dy is None else dy.contiguous()
        dres = None if dh is None else dh.contiguous()
        if not ctx.needs_input_grad[2]:  # frozen weight (LoRA / QLoRA): dX only
            dx = _native.kernels().rmsnorm_bwd_dx(dy, h, w, rstd, dres)
            return dx, dx, None, None, None
        dx, dw = _norm_bwd_into_slot(w, lambda out, acc: _native.kernels().rmsnorm_bwd(dy, h, w, rstd, dres, out, acc))
        return dx, dx, dw, None, None


def rms_norm(x, w, eps=1e-5, pad: int = 0):
    """``pad`` > 0 (GPU, 2-D x): the output is the [rows, d] view of a [rows, d + pad] row buffer whose
    tail a K-concatenated LoRA consumer fills (``peft/lora.py``); numerically unchanged."""
    if _gpu(x):
        return _tail(_RMSNorm.apply(x, w, eps, pad if x.dim() == 2 else 0), pad if x.dim() == 2 else 0)
    return _ref.rmsnorm(x, w, eps)[0]


def add_rms_norm(x, residual, w, eps=1e-5, pad: int = 0):
    """Returns (rmsnorm(x + residual) * w, x + residual); ``pad`` as in ``rms_norm``."""
    if _gpu(x):
        pad = pad if x.dim() == 2 else 0
        y, h = _AddRMSNorm.apply(x, residual, w, eps, pad)
        return _tail(y, pad), h
    return _ref.rmsnorm(x, w, eps, residual=residual)


# ----------------------------------------------------------------------------- LayerNorm
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, w, b, eps):
        C = _native.kernels()
        y, h, mean, rstd = C.layernorm_fwd(x.contiguous(), None if residual is None else residual.contiguous(),
                                           w.contiguous(), None if b is None else b.contiguous(), eps)
        ctx.has_res = residual is not None
        ctx.has_b = b is not None
        ctx.save_for_backward(h, w, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        h, w, mean, rstd = ctx.saved_tensors
        dx, dw, db = _native.kernels().layernorm_bwd(dy.contiguous(), h, w, mean, rstd, None)
        return dx, (dx if ctx.has_res else None), dw.to(w.dtype), (db.to(w.dtype) if ctx.has_b else None), None


def layer_norm(x, w, b=None, eps=1e-5, residual=None):
    """LayerNorm(x [+ residual]) — the post-LN block of nn.TransformerEncoderLayer."""
    if _gpu(x):
        return _LayerNorm.apply(x, residual, w, b, eps)
    return _ref.layernorm(x, w, b, eps, residual=residual)[0]


# ----------------------------------------------------------------------------- activations
# SwiGLU kernels that also write the transposed result for the TN weight gradients of the
# neighbouring projections (h^T for down_proj, dgu^T for gate_up_proj; elementwise.hip
# swiglu_*_t_kernel): the consumer (ops/linear.py _DirectGradLinear) takes the copy from the
# tensor's ``_grt_T`` attribute instead of running its own transpose. GRT_SWIGLU_T=0: off.
_SWIGLU_T = os.environ.get("GRT_SWIGLU_T", "1") != "0"


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, pad=0, fwd_t=False, bwd_t=False):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        ctx.bwd_t = bwd_t
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the h^T output
        C = _native.kernels()
        if fwd_t:
            r = C.swiglu_fwd_t(gu, pad)
            if r:
                ctx.mark_non_differentiable(r[1])
                return r[0], r[1]
        return C.swiglu_fwd(gu, pad), None

    @staticmethod
    def backward(ctx, dout, _dt=None):
        (gu,) = ctx.saved_tensors
        C = _native.kernels()
        if ctx.bwd_t:
            r = C.swiglu_bwd_t(gu, dout.contiguous())
            if r:
                r[0]._grt_T = r[1]
                return r[0], None, None, None
        return C.swiglu_bwd(gu, dout.contiguous()), None, None, None


def swiglu(gu, pad: int = 0, fwd_t: bool = False, bwd_t: bool = False):
    """silu(gu[..., :F]) * gu[..., F:] for the fused [gate | up] projection output; ``pad`` as in
    ``rms_norm`` (the down projection's LoRA tail). ``fwd_t`` / ``bwd_t``: also produce h^T / dgu^T
    for a trainable down / gate_up projection's weight gradient (bf16, rows % 64, F % 128)."""
    if _gpu(gu):
        pad = pad if gu.dim() == 2 else 0
        fwd_t = fwd_t and _SWIGLU_T and gu.dtype == torch.bfloat16
        bwd_t = bwd_t and _SWIGLU_T and gu.dtype == torch.bfloat16
        y, yt = _SwiGLU.apply(gu, pad, fwd_t, bwd_t)
        if yt is not None:
            y._grt_T = yt
        return _tail(y, pad)
    return _ref.swiglu(gu)


class _GELU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        ctx.save_for_backward(x)
        return _native.kernels().gelu_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return _native.kernels().gelu_bwd(x, dy.contiguous())


def gelu(x):
    if _gpu(x) and x.numel() % (8 if x.dtype == torch.bfloat16 else 4) == 0:
        return _GELU.apply(x)
    return _ref.gelu(x)


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed, offset):
        y, mask = _native.kernels().dropout_fwd(x.contiguous(), p, seed, offset)
        ctx.p = p
        ctx.save_for_backward(mask)
        return y

    @staticmethod
    def backward(ctx, dy):
        (mask,) = ctx.saved_tensors
        return _native.kernels().dropout_bwd(dy.contiguous(), mask, ctx.p), None, None, None


def dropout_seed_offset(x):
    """(seed, offset) for a counter-based dropout over ``x``: a fresh 62-bit seed drawn from
    torch's CPU generator, offset 0. Drawing from the CPU generator (no device sync) makes the
    mask a function of the RNG state that ``torch.utils.checkpoint`` saves and restores — the
    recompute of a checkpointed segment draws the same seed, so the mask the backward
    regenerates is the forward's — and that trainers save in ``rng_state_<rank>.pth``, so a
    resumed run continues the mask sequence instead of replaying it from step 0."""
    seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
    return seed, 0


def dropout(x, p, training=True, seed=None):
    if not training or p == 0.0:
        return x
    if _gpu(x):
        s, off = dropout_seed_offset(x)
        return _Dropout.apply(x, p, s if seed is None else seed, off)
    return torch.nn.functional.dropout(x, p, training=True)


# ----------------------------------------------------------------------------- attention
class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale, seqlens_k, dropout_p, seed):
        C = _native.kernels()
        o, lse = C.attn_fwd(q, k, v, None, scale, causal, seqlens_k, dropout_p, seed)
        ctx.save_for_backward(q, k, v, o, lse, seqlens_k)
        ctx.causal, ctx.scale, ctx.dropout_p, ctx.seed = causal, scale, dropout_p, seed
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, seqlens_k = ctx.saved_tensors
        dq, dk, dv = _native.kernels().attn_bwd(do.contiguous(), q, k, v, o, lse, None, None, None,
                                                ctx.scale, ctx.causal, seqlens_k, ctx.dropout_p, ctx.seed)
        return dq, dk, dv, None, None, None, None, None


_DECODE_KERNEL = __import__("os").environ.get("GRT_DECODE_ATTN", "1") != "0"


def _dropout_seed() -> int:
    # drawn from torch's CPU generator (torch.manual_seed reproducible, no device sync)
    return int(torch.randint(0, 2 ** 31 - 1, (1,)).item())


def flash_attention(q, k, v, causal=True, scale=None, seqlens_k=None, dropout_p=0.0, seed=None):
    """q [B,Sq,Hq,D], k/v [B,Sk,Hkv,D] (any batch/seq/head strides) -> o [B,Sq,Hq,D].

    ``dropout_p`` > 0 drops attention probabilities (nn.MultiheadAttention / SDPA semantics:
    softmax normaliser over all keys, kept probabilities scaled by 1/(1-p)); the mask is a
    stateless counter hash of (seed, batch*head, query, key), regenerated in the backward.
    """
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if dropout_p > 0.0 and seed is None:
        seed = _dropout_seed()
    seed = 0 if seed is None else int(seed)
    if (_gpu(q) and q.shape[1] == 1 and q.dtype == torch.bfloat16 and q.shape[-1] == 128 and dropout_p == 0.0
            and not torch.is_grad_enabled() and (q.shape[2] // k.shape[2]) in (1, 2, 4, 8)
            and q.shape[2] % k.shape[2] == 0 and _DECODE_KERNEL):
        # one query token per sequence (decode): split-K kernel over the cached keys; every cached
        # key is at or before the query position, so the causal mask is the valid-length mask
        return _native.kernels().attn_decode(q, k, v, seqlens_k, scale)
    if _gpu(q) and ((q.dtype == torch.bfloat16 and q.shape[-1] == 128) or
                    (q.dtype == torch.float32 and q.shape[-1] in (64, 128))):
        return _FlashAttn.apply(q, k, v, causal, scale, seqlens_k, float(dropout_p), seed)
    if _gpu(q):
        _warn_once(f"flash_attention: no gfx950 kernel for dtype={q.dtype} head_dim={q.shape[-1]}; "
                   "using the fp32 math path")
    return _ref.attention(q, k, v, causal=causal, scale=scale, seqlens_k=seqlens_k, dropout_p=dropout_p, seed=seed)


_warned = set()


def _warn_once(msg):
    if msg not in _warned:
        _warned.add(msg)
        import warnings
        warnings.warn(msg)


# attention backward epilogues write dQ / dK un-rotated into dqkv (no rope_bwd pass);
# GRT_ROPE_BWD_FUSED=0 -> separate dq / dk tensors + the RoPE backward kernel
_ROPE_BWD_FUSED = os.environ.get("GRT_ROPE_BWD_FUSED", "1") != "0"


class Varlen:
    """Padding-free packing of variable-length sequences into one token axis (FlashAttention
    "varlen"): sequence i is token rows [cu[i], cu[i+1]); attention is causal inside each
    sequence and RoPE positions restart at 0 per sequence. ``cu`` (int32, device) and ``pos``
    (int32 [T], device) feed the kernels; ``cu_host`` / ``max_len`` are host ints (no sync)."""

    __slots__ = ("cu", "pos", "cu_host", "max_len")

    def __init__(self, lengths, device):
        lens = [int(n) for n in lengths]
        if not lens or min(lens) < 1:
            raise ValueError("Varlen: every packed sequence needs at least one token")
        cu = [0]
        for n in lens:
            cu.append(cu[-1] + n)
        self.cu_host = cu
        self.max_len = max(lens)
        self.cu = torch.tensor(cu, dtype=torch.int32).pin_memory().to(device, non_blocking=True) \
            if torch.device(device).type == "cuda" else torch.tensor(cu, dtype=torch.int32)
        pos = torch.cat([torch.arange(n, dtype=torch.int32) for n in lens])
        self.pos = pos.pin_memory().to(device, non_blocking=True) if torch.device(device).type == "cuda" else pos

    @property
    def total(self) -> int:
        return self.cu_host[-1]

    @property
    def lengths(self):
        return [b - a for a, b in zip(self.cu_host[:-1], self.cu_host[1:])]


_ATTN_DQKV_T = os.environ.get("GRT_ATTN_DQKV_T", "1") != "0"


class _RopeAttention(torch.autograd.Function):
    """qkv [B*S, (Hq + 2 Hkv) * D] -> o [B*S, Hq * D]: RoPE + causal flash attention fused.

    Backward writes dV straight into the V columns of dqkv (strided) and the un-rotated dQ/dK into
    its Q/K columns, so the fused-QKV gradient is produced with no split/cat copies.
    With ``varlen`` the B*S rows are the packed tokens of varlen.cu's sequences (B = 1, S = T).
    """

    @staticmethod
    def forward(ctx, qkv, cos, sin, B, S, hq, hkv, D, causal, scale, varlen=None, pad=0, bwd_t=False, fwd_t=False):
        C = _native.kernels()
        ctx.bwd_t = bwd_t
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the o^T output
        qkv = qkv.contiguous()
        cu, ml = (varlen.cu, varlen.max_len) if varlen is not None else (None, 0)
        q, k = C.rope_fwd(qkv, cos, sin, varlen.pos if varlen is not None else None, hq, hkv, D,
                          ml if varlen is not None else S)
        q4 = q.view(B, S, hq, D)
        k4 = k.view(B, S, hkv, D)
        v4 = qkv.view(B, S, hq + 2 * hkv, D)[:, :, hq + hkv:, :]
        # the output rows may be the head of [o | LoRA h] row buffers (the o_proj's K-concat tail)
        ld = hq * D + pad
        ow = torch.empty(B * S, ld, device=qkv.device, dtype=qkv.dtype)
        o = ow.as_strided((B, S, hq, D), (S * ld, ld, D, 1))
        ot = (torch.empty(hq * D, B * S, device=qkv.device, dtype=qkv.dtype)
              if fwd_t and (B * S) % 64 == 0 and (hq * D) % 64 == 0 else None)
        _, lse = C.attn_fwd(q4, k4, v4, o, scale, causal, None, cu_seqlens=cu, max_seqlen=ml, o_t=ot)
        ctx.save_for_backward(qkv, q, k, o, lse, cos, sin)
        ctx.dims = (B, S, hq, hkv, D, causal, scale)
        ctx.varlen = varlen
        if ot is not None:
            ctx.mark_non_differentiable(ot)
        return ow[:, :hq * D], ot

    @staticmethod
    def backward(ctx, do, _dot=None):
        qkv, q, k, o, lse, cos, sin = ctx.saved_tensors
        B, S, hq, hkv, D, causal, scale = ctx.dims
        vl = ctx.varlen
        cu, ml = (vl.cu, vl.max_len) if vl is not None else (None, 0)
        C = _native.kernels()
        dqkv = torch.empty_like(qkv)
        q4 = q.view(B, S, hq, D)
        k4 = k.view(B, S, hkv, D)
        v4 = qkv.view(B, S, hq + 2 * hkv, D)[:, :, hq + hkv:, :]
        d4 = dqkv.view(B, S, hq + 2 * hkv, D)
        dv4 = d4[:, :, hq + hkv:, :]
        if _ROPE_BWD_FUSED and cos.dim() == 2 and cos.shape[0] >= (ml if vl is not None else S):
            # the kernels' epilogues undo the RoPE and write dQ / dK straight into dqkv's columns
            # (packed: the key / query index inside its sequence IS its RoPE position); with bwd_t
            # they also write dqkv^T for the QKV projection's TN weight gradient (ops/linear.py
            # takes it from dqkv._grt_T instead of transposing dqkv)
            T, W = dqkv.shape[0], dqkv.shape[1]
            dqkv_t = (torch.empty(W, T, device=dqkv.device, dtype=dqkv.dtype)
                      if ctx.bwd_t and T % 64 == 0 and W % 64 == 0 else None)
            C.attn_bwd(do.contiguous().view(B, S, hq, D), q4, k4, v4, o, lse, d4[:, :, :hq], d4[:, :, hq:hq + hkv],
                       dv4, scale, causal, None, rope_cos=cos, rope_sin=sin, cu_seqlens=cu, max_seqlen=ml,
                       dqkv_t=dqkv_t)
            if dqkv_t is not None:
                dqkv._grt_T = dqkv_t
        else:
            dq, dk, _ = C.attn_bwd(do.contiguous().view(B, S, hq, D), q4, k4, v4, o, lse, None, None, dv4,
                                   scale, causal, None, cu_seqlens=cu, max_seqlen=ml)
            C.rope_bwd(dq, dk, dqkv, cos, sin, vl.pos if vl is not None else None, hq, hkv, D,
                       ml if vl is not None else S)
        return dqkv, None, None, None, None, None, None, None, None, None, None, None, None, None


def rope_attention(qkv, cos, sin, B, S, hq, hkv, D, causal=True, scale=None, varlen: "Varlen" = None,
                   pad: int = 0, bwd_t: bool = False, fwd_t: bool = False):
    """``varlen``: the B*S rows are padding-free packed sequences (B = 1; see ``Varlen``).
    ``pad`` as in ``rms_norm``: the o_proj's LoRA tail after each output row. ``bwd_t``: the
    backward also writes dqkv^T for a trainable QKV projection's weight gradient, ``fwd_t``: the
    forward also writes o^T for a trainable o projection's (GRT_ATTN_DQKV_T=0: neither)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if _gpu(qkv) and qkv.dtype == torch.bfloat16 and D == 128:
        bwd_t = bwd_t and _ATTN_DQKV_T
        fwd_t = fwd_t and _ATTN_DQKV_T and not pad
        o, ot = _RopeAttention.apply(qkv, cos, sin, B, S, hq, hkv, D, causal, scale, varlen, pad, bwd_t, fwd_t)
        if ot is not None:
            o._grt_T = ot
        return _tail(o, pad)
    x = qkv.view(B * S, hq + 2 * hkv, D)
    pos = varlen.pos if varlen is not None else None
    q = _ref.apply_rope(x[:, :hq], cos, sin, pos)
    k = _ref.apply_rope(x[:, hq:hq + hkv], cos, sin, pos)
    v = x[:, hq + hkv:]
    if varlen is not None:  # reference path: attention sequence by sequence
        outs = []
        for a, b in zip(varlen.cu_host[:-1], varlen.cu_host[1:]):
            outs.append(flash_attention(q[a:b].unsqueeze(0), k[a:b].unsqueeze(0), v[a:b].unsqueeze(0), causal,
                                        scale).squeeze(0))
        return torch.cat(outs).reshape(B * S, hq * D)
    o = flash_attention(q.view(B, S, hq, D), k.view(B, S, hkv, D), v.reshape(B, S, hkv, D), causal, scale)
    return o.reshape(B * S, hq * D)


# ----------------------------------------------------------------------------- cross entropy
class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index, inplace):
        C = _native.kernels()
        loss_rows, lse = C.ce_fwd(logits, labels, ignore_index)
        nvalid = (labels != ignore_index).sum().clamp_min(1).float()
        ctx.save_for_backward(logits, labels, lse, nvalid)
        ctx.ignore_index, ctx.inplace = ignore_index, inplace
        return loss_rows.sum() / nvalid

    @staticmethod
    def backward(ctx, g):
        logits, labels, lse, nvalid = ctx.saved_tensors
        gscale = (g.float() / nvalid).expand(logits.shape[0]).contiguous()
        d = _native.kernels().ce_bwd(logits, labels, lse, gscale, ctx.ignore_index, ctx.inplace)
        return d, None, None, None


def cross_entropy(logits, labels, ignore_index=-100, inplace_backward=False):
    """Mean CE over non-ignored rows. logits [N, V] (row-major), labels int64 [N]."""
    if _gpu(logits):
        return _CrossEntropy.apply(logits, labels.contiguous(), ignore_index, inplace_backward)
    return _ref.cross_entropy(logits, labels, ignore_index)


class _LMHeadCE(torch.autograd.Function):
    """loss = CE(hidden @ W^T [+ b], labels): the logits never escape, so the backward writes
    dlogits over the logits buffer in place (saves a [tokens, V] allocation per step).

    ``row_weights`` (fp32 [N], optional): loss = sum_i w_i * CE_i over non-ignored rows instead of
    the mean; the CE backward kernel already takes a per-row gradient scale, so weighting costs
    nothing (used to run several gradient-accumulation micro-batches as one batch, each keeping
    its own mean — trainer/sft.py)."""

    @staticmethod
    def forward(ctx, hidden, weight, bias, labels, ignore_index, row_weights):
        C = _native.kernels()
        logits = torch.nn.functional.linear(hidden, weight, bias)
        loss_rows, lse = C.ce_fwd(logits, labels, ignore_index)
        if row_weights is None:
            scale = (labels != ignore_index).sum().clamp_min(1).float().reciprocal()
            loss = loss_rows.sum() * scale
        else:
            scale = row_weights * (labels != ignore_index)
            loss = (loss_rows.float() * scale).sum()
        ctx.save_for_backward(hidden, weight, logits, labels, lse, scale)
        ctx.wt_ev = transpose_for_backward(weight) if ctx.needs_input_grad[0] else None
        ctx.ignore_index = ignore_index
        ctx.has_bias = bias is not None
        return loss

    @staticmethod
    def backward(ctx, g):
        hidden, weight, logits, labels, lse, scale = ctx.saved_tensors
        gscale = (g.float() * scale).expand(logits.shape[0]).contiguous()
        dlogits = _native.kernels().ce_bwd(logits, labels, lse, gscale, ctx.ignore_index, True)
        dh = dw = db = None
        if ctx.needs_input_grad[0]:
            dh = input_grad(dlogits, weight, ctx.wt_ev)
            ctx.wt_ev = None
        if ctx.needs_input_grad[1]:
            slot = getattr(weight, "_grt_slot", None)
            if slot is not None:   # GEMM writes dW straight into the DDP bucket (ops/linear.py)
                slot.write(lambda v: wgrad(dlogits, hidden, v, False), lambda v: wgrad(dlogits, hidden, v, True))
                slot.notify(weight)
            else:
                dw = wgrad(dlogits, hidden)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dlogits.sum(0)
        return dh, dw, db, None, None, None


def lm_head_cross_entropy(hidden, weight, labels, bias=None, ignore_index=-100, row_weights=None):
    """Mean CE of ``hidden @ weight^T`` over non-ignored rows, or the ``row_weights``-weighted sum."""
    if _gpu(hidden):
        rw = None if row_weights is None else row_weights.reshape(-1).float().contiguous()
        return _LMHeadCE.apply(hidden, weight, bias, labels.contiguous(), ignore_index, rw)
    logits = torch.nn.functional.linear(hidden, weight, bias)
    if row_weights is None:
        return _ref.cross_entropy(logits, labels, ignore_index)
    rows = torch.nn.functional.cross_entropy(logits.float(), labels, ignore_index=ignore_index, reduction="none")
    return (rows * row_weights.reshape(-1).float() * (labels != ignore_index)).sum()


# ----------------------------------------------------------------------------- NF4
def nf4_quantize(w, blocksize=64):
    if _gpu(w):
        return tuple(_native.kernels().nf4_quantize(w.contiguous().view(-1), blocksize))
    return _ref.nf4_quantize(w, blocksize)


def nf4_dequantize(packed, absmax, n, blocksize=64, dtype=torch.bfloat16, out=None):
    if _gpu(packed):
        return _native.kernels().nf4_dequantize(packed, absmax, n, blocksize, dtype, out)
    return _ref.nf4_dequantize(packed, absmax, n, blocksize, dtype)
