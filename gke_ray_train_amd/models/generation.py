"""KV-cache generation for the Llama family (greedy / sampling).

Reference role: ``model.generate(**inputs, max_new_tokens=..., do_sample=False,
eos_token_id=[eos, <|eot_id|>])`` in the post-training comparison (ray-jobs/fine_tune_llama_ray.py:
138-146). The cache is one preallocated [B, S_max, Hkv, D] K and V tensor per
layer (sized for prompt + max_new_tokens up front, no re-allocation while decoding); prefill and
every decode step run the SAME flash-attention kernel over a strided view of the cache
(bottom-right-aligned causal mask, Sq = new tokens, Sk = tokens so far) with RoPE applied at the
absolute positions by the RoPE kernel's position array.
"""
from __future__ import annotations

from typing import List, Optional, Union

import torch

from .. import _native, ops
from ..ops import _ref


class KVCache:
    def __init__(self, cfg, B, max_len, device, dtype):
        hd, hkv = cfg.head_dim, cfg.num_key_value_heads
        self.k = [torch.zeros(B, max_len, hkv, hd, device=device, dtype=dtype) for _ in range(cfg.num_hidden_layers)]
        self.v = [torch.zeros(B, max_len, hkv, hd, device=device, dtype=dtype) for _ in range(cfg.num_hidden_layers)]
        self.len = 0
        self.max_len = max_len


def _layer_step(layer, h, residual, B, S, pos0, cos, sin, cache: KVCache, li: int):
    attn = layer.self_attn
    eps = layer.input_layernorm.eps
    if residual is None:
        residual = h
        x = ops.rms_norm(h, layer.input_layernorm.weight, eps)
    else:
        x, residual = ops.add_rms_norm(h, residual, layer.input_layernorm.weight, eps)
    qkv = attn.qkv_proj(x)
    hq, hkv, D = attn.hq, attn.hkv, attn.hd
    pos = torch.arange(pos0, pos0 + S, device=h.device, dtype=torch.int32).repeat(B)
    if qkv.is_cuda and qkv.dtype == torch.bfloat16 and D == 128:
        q, k = _native.kernels().rope_fwd(qkv.contiguous(), cos, sin, pos, hq, hkv, D, cos.shape[0])
    else:
        x3 = qkv.view(B * S, hq + 2 * hkv, D)
        q = _ref.apply_rope(x3[:, :hq], cos, sin, pos)
        k = _ref.apply_rope(x3[:, hq:hq + hkv], cos, sin, pos)
    v = qkv.view(B, S, hq + 2 * hkv, D)[:, :, hq + hkv:]
    cache.k[li][:, pos0:pos0 + S] = k.view(B, S, hkv, D)
    cache.v[li][:, pos0:pos0 + S] = v
    kk = cache.k[li][:, :pos0 + S]
    vv = cache.v[li][:, :pos0 + S]
    o = ops.flash_attention(q.view(B, S, hq, D), kk, vv, causal=True)
    h = attn.o_proj(o.reshape(B * S, hq * D))
    x, residual = ops.add_rms_norm(h, residual, layer.post_attention_layernorm.weight, eps)
    return layer.mlp(x), residual


@torch.no_grad()
def forward_cached(model, ids: torch.Tensor, cache: KVCache) -> torch.Tensor:
    """Run `ids` [B, S] at positions cache.len ... ; returns last-position logits [B, V]."""
    B, S = ids.shape
    pos0 = cache.len
    cos, sin = model.rope(cache.max_len, ids.device)
    h = model.model.embed_tokens(ids).view(B * S, -1)
    residual = None
    for li, layer in enumerate(model.model.layers):
        h, residual = _layer_step(layer, h, residual, B, S, pos0, cos, sin, cache, li)
    x, _ = ops.add_rms_norm(h, residual, model.model.norm.weight, model.model.norm.eps)
    last = x.view(B, S, -1)[:, -1]
    cache.len += S
    return model.lm_head(last).float()


@torch.no_grad()
def generate(model, input_ids: torch.Tensor, max_new_tokens: int = 32,
             eos_token_id: Optional[Union[int, List[int]]] = None, do_sample: bool = False, temperature: float = 1.0,
             top_p: Optional[float] = None, attention_mask=None, pad_token_id=None, generator=None, **_):
    """Returns [B, prompt + generated] token ids (HF ``generate`` output convention)."""
    was = model.training
    model.eval()
    B, S = input_ids.shape
    eos = set([eos_token_id] if isinstance(eos_token_id, int) else (eos_token_id or []))
    p = next(model.parameters())
    cache = KVCache(model.config, B, S + max_new_tokens, input_ids.device,
                    p.dtype if p.dtype in (torch.bfloat16, torch.float32) else torch.bfloat16)
    logits = forward_cached(model, input_ids, cache)
    out = [input_ids]
    finished = torch.zeros(B, dtype=torch.bool, device=input_ids.device)
    for _ in range(max_new_tokens):
        if do_sample:
            probs = torch.softmax(logits / max(temperature, 1e-5), -1)
            if top_p is not None and top_p < 1.0:
                sp, si = probs.sort(-1, descending=True)
                keep = sp.cumsum(-1) - sp <= top_p
                sp = sp * keep
                probs = torch.zeros_like(probs).scatter(-1, si, sp)
            nxt = torch.multinomial(probs / probs.sum(-1, keepdim=True), 1, generator=generator).squeeze(-1)
        else:
            nxt = logits.argmax(-1)
        if pad_token_id is not None:
            nxt = torch.where(finished, torch.full_like(nxt, pad_token_id), nxt)
        out.append(nxt[:, None])
        if eos:
            finished |= torch.isin(nxt, torch.tensor(sorted(eos), device=nxt.device))
            if bool(finished.all()):
                break
        logits = forward_cached(model, nxt[:, None], cache)
    if was:
        model.train()
    return torch.cat(out, 1)
