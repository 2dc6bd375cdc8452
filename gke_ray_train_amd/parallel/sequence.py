"""Sequence parallelism (DeepSpeed-Ulysses style) for long-context Llama training.

Reference role: none — the reference caps sequences at 1024 tokens (MAX_SEQ_LENGTH,
ray-jobs/fine_tune_config.json:27; BasicLLM windows of 256, ray-jobs/pytorch_llm_ray.py:332-333) and
has no context parallelism. This module is the §5.7 design, for sequences
whose activations do not fit one GPU even at 288 GB.

MI355X design: each rank of an SP group holds S/P consecutive tokens of the same sequences, so
everything outside attention (embedding, norms, projections, MLP, LM head + CE) is token-parallel
and needs no communication. Attention needs every key, so around the flash kernel two
all-to-alls re-partition Q/K/V from sequence-sharded [B, S/P, H, D] to head-sharded [B, S, H/P, D]
and the output back. On one MI355X node every GPU has a direct xGMI link to every peer: an
all-to-all moves 1/P of the tensor to each peer over all 7 links at once, which is why
Ulysses (all-to-all) rather than ring attention (neighbour send/recv, one link at a time) is the
MI355X-first choice. RoPE uses absolute positions (rank offset + local index) through the HIP
RoPE kernel's position array. GQA with fewer KV heads than ranks repeats KV heads before the
exchange (P % Hkv == 0).

Gradients: parameters are replicated across the SP group, so the data-parallel engine over the
WHOLE world (DP x SP ranks) averages them; ``shard_sequence`` returns a loss weight that turns each
rank's mean-over-local-tokens into the exact global-token mean under that averaging.

Usage::

    enable_sequence_parallel(model, group)           # group: the ranks sharing each sequence
    ids_loc, labels_loc, w = shard_sequence(ids, group)
    loss = model(ids_loc, shifted_labels=labels_loc)["loss"] * w
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist

from .. import _native, ops
from ..ops import _ref


def _world(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _rank(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


class _SeqToHead(torch.autograd.Function):
    """[B, S/P, H, D] (sequence shard) -> [B, S, H/P, D] (head shard); backward is the inverse."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _seq_to_head(x, group)

    @staticmethod
    def backward(ctx, g):
        return _head_to_seq(g.contiguous(), ctx.group), None


class _HeadToSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _head_to_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        return _seq_to_head(g.contiguous(), ctx.group), None


def _seq_to_head(x: torch.Tensor, group) -> torch.Tensor:
    P = _world(group)
    B, Sl, H, D = x.shape
    if P == 1:
        return x.contiguous()
    if H % P:
        raise ValueError(f"sequence parallel: {H} heads do not split over {P} ranks")
    # [B, Sl, P, H/P, D] -> [P, B, Sl, H/P, D]: chunk p goes to rank p (its head slice)
    send = x.reshape(B, Sl, P, H // P, D).permute(2, 0, 1, 3, 4).contiguous()
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    # recv[p] = rank p's tokens (sequence chunk p) of my heads -> [B, P*Sl, H/P, D]
    return recv.permute(1, 0, 2, 3, 4).reshape(B, P * Sl, H // P, D)


def _head_to_seq(x: torch.Tensor, group) -> torch.Tensor:
    P = _world(group)
    B, S, Hl, D = x.shape
    if P == 1:
        return x.contiguous()
    Sl = S // P
    # [B, P, Sl, Hl, D] -> [P, B, Sl, Hl, D]: chunk p (tokens of rank p) goes back to rank p
    send = x.reshape(B, P, Sl, Hl, D).permute(1, 0, 2, 3, 4).contiguous()
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    # recv[p] = my tokens of rank p's heads -> [B, Sl, P*Hl, D]
    return recv.permute(1, 2, 0, 3, 4).reshape(B, Sl, P * Hl, D)


class _RopePositions(torch.autograd.Function):
    """qkv [T, (hq + 2 hkv) D] -> rotated q [T, hq, D], k [T, hkv, D] at absolute positions."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, pos, hq, hkv, D):
        C = _native.kernels()
        qkv = qkv.contiguous()
        q, k = C.rope_fwd(qkv, cos, sin, pos, hq, hkv, D, cos.shape[0])
        ctx.save_for_backward(cos, sin, pos)
        ctx.dims = (qkv.shape, hq, hkv, D)
        return q, k

    @staticmethod
    def backward(ctx, dq, dk):
        cos, sin, pos = ctx.saved_tensors
        shape, hq, hkv, D = ctx.dims
        dqkv = torch.zeros(shape, device=dq.device, dtype=dq.dtype)  # V columns: through the view
        _native.kernels().rope_bwd(dq.contiguous(), dk.contiguous(), dqkv, cos, sin, pos, hq, hkv, D, cos.shape[0])
        return dqkv, None, None, None, None, None, None


def _rope(qkv, cos, sin, pos, hq, hkv, D):
    if qkv.is_cuda and qkv.dtype == torch.bfloat16 and D == 128:
        return _RopePositions.apply(qkv, cos, sin, pos, hq, hkv, D)
    x = qkv.view(-1, hq + 2 * hkv, D)
    return _ref.apply_rope(x[:, :hq], cos, sin, pos), _ref.apply_rope(x[:, hq:hq + hkv], cos, sin, pos)


def ulysses_attention(qkv: torch.Tensor, cos, sin, B: int, S_loc: int, hq: int, hkv: int, D: int, group,
                      causal: bool = True) -> torch.Tensor:
    """qkv [B*S_loc, (hq + 2 hkv) D] of this rank's tokens -> attention output [B*S_loc, hq D]."""
    P = _world(group)
    r = _rank(group)
    pos = (torch.arange(S_loc, device=qkv.device, dtype=torch.int32) + r * S_loc).repeat(B)
    q, k = _rope(qkv, cos, sin, pos, hq, hkv, D)
    v = qkv.view(B, S_loc, hq + 2 * hkv, D)[:, :, hq + hkv:]
    q = q.reshape(B, S_loc, hq, D)
    k = k.reshape(B, S_loc, hkv, D)
    if hkv % P:
        if P % hkv:
            raise ValueError(f"sequence parallel: {hkv} KV heads vs {P} ranks (need one to divide the other)")
        rep = P // hkv  # each rank gets one (repeated) KV head matching its query-head slice
        k = k.repeat_interleave(rep, dim=2)
        v = v.repeat_interleave(rep, dim=2)
    qh = _SeqToHead.apply(q, group)
    kh = _SeqToHead.apply(k, group)
    vh = _SeqToHead.apply(v.contiguous(), group)
    o = ops.flash_attention(qh, kh, vh, causal=causal)          # [B, S, hq/P, D]
    o = _HeadToSeq.apply(o, group)                                # [B, S_loc, hq, D]
    return o.reshape(B * S_loc, hq * D)


def enable_sequence_parallel(model, group=None):
    """Route every Llama attention layer through ``ulysses_attention`` over ``group``."""
    from ..models.llama import LlamaAttention
    if group is None:
        group = dist.group.WORLD
    model.sp_group = group
    model.sp_size = _world(group)
    for m in model.modules():
        if isinstance(m, LlamaAttention):
            m.sp_group = group
    return model


def shard_sequence(input_ids: torch.Tensor, group=None, attention_mask: Optional[torch.Tensor] = None,
                   ignore_index: int = -100) -> Tuple[torch.Tensor, torch.Tensor, float]:
    """Every rank of ``group`` holds the same [B, S] batch; returns this rank's [B, S/P] token
    chunk, its next-token labels (shifted over the FULL sequence, so the last token of chunk r is
    labelled with the first token of chunk r+1) and the loss weight P * n_local / n_global that
    makes the engine's average over ranks the exact mean over all valid label tokens."""
    P, r = _world(group), _rank(group)
    B, S = input_ids.shape
    if S % P:
        raise ValueError(f"sequence length {S} does not split over {P} ranks")
    lab = torch.full_like(input_ids, ignore_index)
    lab[:, :-1] = input_ids[:, 1:]
    if attention_mask is not None:
        lab[:, :-1].masked_fill_(attention_mask[:, 1:] == 0, ignore_index)
    Sl = S // P
    ids_loc = input_ids[:, r * Sl:(r + 1) * Sl].contiguous()
    lab_loc = lab[:, r * Sl:(r + 1) * Sl].contiguous()
    n_glob = int((lab != ignore_index).sum())
    n_loc = int((lab_loc != ignore_index).sum())
    w = P * n_loc / max(n_glob, 1) if n_loc else 0.0
    return ids_loc, lab_loc, w
