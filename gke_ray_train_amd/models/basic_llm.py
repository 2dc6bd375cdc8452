"""BasicLLM: the reference's char-level causal Transformer, rebuilt on the framework's ops.

Reference: ``BasicLLM`` / ``PositionalEncoding`` in ray-jobs/pytorch_llm_ray.py:57-105:
Embedding(V, d) * sqrt(d) + fixed sinusoidal PE -> dropout -> N x post-LN
``nn.TransformerEncoderLayer(d, nhead, dim_ff, dropout, batch_first=True, activation="gelu")``
under a causal mask -> Linear(d, V) with bias.

Same math and the SAME state_dict keys as the reference module (``token_embedding.weight``,
``positional_encoding.pe``, ``transformer_decoder.layers.{i}.self_attn.in_proj_weight`` …,
``fc_out.weight``), so ``model.pth`` files written by either load into the other. The compute
path differs: post-LN is one fused residual+LayerNorm kernel per sub-block, GELU/dropout/CE are
HIP kernels, attention is the flash kernel (fp32 or bf16, with in-kernel attention-probability dropout)
and the PE is a non-synced on-device constant (no per-step DDP buffer broadcast).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..ops.linear import Embedding, Linear


@dataclass
class BasicLLMConfig:
    vocab_size: int = 256
    embed_dim: int = 2048
    num_heads: int = 16
    num_layers: int = 24
    hidden_dim: int = 8192
    max_seq_len: int = 1024
    dropout: float = 0.1


BASIC_CONFIGS = {
    # reference config (ray-jobs/pytorch_llm_ray.py:324-344): ~1.21 B params
    "basic-1b": dict(embed_dim=2048, num_heads=16, num_layers=24, hidden_dim=8192, max_seq_len=1024),
    # GPT-2-small-shaped config named by BASELINE.json config #1
    "gpt2-small": dict(embed_dim=768, num_heads=12, num_layers=12, hidden_dim=3072, max_seq_len=1024),
    "basic-tiny": dict(embed_dim=256, num_heads=2, num_layers=2, hidden_dim=1024, max_seq_len=256),
}


def sinusoidal_pe(max_len: int, d: int) -> torch.Tensor:
    """[1, max_len, d] table identical to the reference PositionalEncoding (incl. odd d)."""
    position = torch.arange(max_len, dtype=torch.float).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d, 2).float() * (-math.log(10000.0) / d))
    pe = torch.zeros(max_len, d)
    pe[:, 0::2] = torch.sin(position * div_term)
    if d % 2 != 0:
        pe[:, 1::2] = torch.cos(position * (div_term[:-1] if div_term.size(0) > 1 else div_term))
    else:
        pe[:, 1::2] = torch.cos(position * div_term)
    return pe.unsqueeze(0)


class PositionalEncoding(nn.Module):
    def __init__(self, d_model: int, max_len: int = 5000):
        super().__init__()
        self.register_buffer("pe", sinusoidal_pe(max_len, d_model))


class _MHA(nn.Module):
    """Parameter container with nn.MultiheadAttention's names (in_proj_weight / out_proj)."""

    def __init__(self, d, nhead, dropout, device=None, dtype=None):
        super().__init__()
        self.embed_dim, self.num_heads, self.dropout = d, nhead, dropout
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d, device=device, dtype=dtype))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d, device=device, dtype=dtype))
        self.out_proj = Linear(d, d, device=device, dtype=dtype)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)

    def forward(self, x, B, S, training):
        d, H = self.embed_dim, self.num_heads
        Dh = d // H
        qkv = F.linear(x, self.in_proj_weight, self.in_proj_bias).view(B, S, 3, H, Dh)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        p = self.dropout if training else 0.0
        # on MI355X: the flash kernels with in-kernel probability dropout — exact fp32
        # (attention_f32.hip, the reference's fp32 training) or bf16 (attention.hip); CPU: the
        # explicit fp32 math path with the same dropout mask (reference semantics, :82-86)
        o = ops.flash_attention(q, k, v, causal=True, dropout_p=p)
        return self.out_proj(o.reshape(B * S, d))


class EncoderLayer(nn.Module):
    """Post-LN nn.TransformerEncoderLayer(activation='gelu', batch_first=True), fused."""

    def __init__(self, d, nhead, dim_ff, dropout, device=None, dtype=None):
        super().__init__()
        self.self_attn = _MHA(d, nhead, dropout, device, dtype)
        self.linear1 = Linear(d, dim_ff, device=device, dtype=dtype)
        self.linear2 = Linear(dim_ff, d, device=device, dtype=dtype)
        self.norm1 = nn.LayerNorm(d, eps=1e-5, device=device, dtype=dtype)
        self.norm2 = nn.LayerNorm(d, eps=1e-5, device=device, dtype=dtype)
        self.p = dropout

    def forward(self, x, B, S):
        tr = self.training
        sa = ops.dropout(self.self_attn(x, B, S, tr), self.p, tr)
        x = ops.layer_norm(sa, self.norm1.weight, self.norm1.bias, 1e-5, residual=x)
        ff = self.linear2(ops.dropout(ops.gelu(self.linear1(x)), self.p, tr))
        ff = ops.dropout(ff, self.p, tr)
        return ops.layer_norm(ff, self.norm2.weight, self.norm2.bias, 1e-5, residual=x)


class _Encoder(nn.Module):
    def __init__(self, layers):
        super().__init__()
        self.layers = nn.ModuleList(layers)


class BasicLLM(nn.Module):
    def __init__(self, vocab_size: int, embed_dim: int, num_heads: int, num_layers: int, hidden_dim: int,
                 max_seq_len: int = 1024, dropout: float = 0.1, device=None, dtype=None):
        super().__init__()
        self.config = BasicLLMConfig(vocab_size, embed_dim, num_heads, num_layers, hidden_dim, max_seq_len, dropout)
        self.embed_dim = embed_dim
        self.token_embedding = Embedding(vocab_size, embed_dim, device=device, dtype=dtype)
        self.positional_encoding = PositionalEncoding(embed_dim, max_seq_len)
        self.transformer_decoder = _Encoder(
            [EncoderLayer(embed_dim, num_heads, hidden_dim, dropout, device, dtype) for _ in range(num_layers)])
        self.fc_out = Linear(embed_dim, vocab_size, device=device, dtype=dtype)
        self.dropout_p = dropout
        self.max_seq_len = max_seq_len
        if device is not None:
            self.positional_encoding.to(device)

    def forward(self, src: torch.Tensor) -> torch.Tensor:
        B, S = src.shape
        d = self.embed_dim
        emb = self.token_embedding(src).view(B * S, d)
        pe = self.positional_encoding.pe[0, :S]
        x = (emb * math.sqrt(d) + pe.to(emb.dtype).repeat(B, 1)) if not emb.is_cuda else \
            _scale_add_pe(emb, pe, S, math.sqrt(d))
        x = ops.dropout(x, self.dropout_p, self.training)
        for layer in self.transformer_decoder.layers:
            x = layer(x, B, S)
        return self.fc_out(x).view(B, S, -1)

    def loss(self, src, targets):
        """Fused fc_out + CrossEntropyLoss (mean) — the reference's criterion (:237,:275)."""
        B, S = src.shape
        d = self.embed_dim
        emb = self.token_embedding(src).view(B * S, d)
        pe = self.positional_encoding.pe[0, :S]
        x = (emb * math.sqrt(d) + pe.to(emb.dtype).repeat(B, 1)) if not emb.is_cuda else \
            _scale_add_pe(emb, pe, S, math.sqrt(d))
        x = ops.dropout(x, self.dropout_p, self.training)
        for layer in self.transformer_decoder.layers:
            x = layer(x, B, S)
        return self.fc_out(x, labels=targets.reshape(-1))


class _ScaleAddPE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, emb, pe, S, scale):
        from .. import _native
        ctx.scale = scale
        return _native.kernels().scale_add_pe(emb.contiguous(), pe.float().contiguous(), S, scale)

    @staticmethod
    def backward(ctx, g):
        return g * ctx.scale, None, None, None


def _scale_add_pe(emb, pe, S, scale):
    return _ScaleAddPE.apply(emb, pe, S, scale)


def build_basic_llm(name="basic-1b", vocab_size=256, device=None, dtype=None, **overrides):
    cfg = dict(BASIC_CONFIGS[name])
    cfg.update(overrides)
    return BasicLLM(vocab_size=vocab_size, device=device, dtype=dtype, **cfg)
