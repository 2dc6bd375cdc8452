"""KV-cache generation for the Llama family (greedy / sampling).

Reference role: ``model.generate(**inputs, max_new_tokens=..., do_sample=False,
eos_token_id=[eos, <|eot_id|>])`` in the post-training comparison (ray-jobs/fine_tune_llama_ray.py:
138-146). The cache is one preallocated [B, S_max, Hkv, D] K and V tensor per
layer (sized for prompt + max_new_tokens up front, no re-allocation while decoding); prefill and
every decode step run the SAME flash-attention kernel over a strided view of the cache
(bottom-right-aligned causal mask, Sq = new tokens, Sk = tokens so far) with RoPE applied at the
absolute positions by the RoPE kernel's position array.

On MI355X the one-token decode step is launch-bound (≈10 kernels per layer, a few µs of work
each), so ``GraphDecoder`` captures the WHOLE step — embedding, every layer, final norm, LM head
and the greedy argmax — into one HIP graph and replays it per token. Everything that changes
between tokens lives in device tensors the graph reads: the current position (RoPE position
array and the KV-cache write index) and the per-row valid key length, which the flash kernel
takes as its padding mask (``seqlens_k``) over the full-length cache, so the kernel's tile loop
still covers only the keys written so far. EOS checks touch the host every ``sync_every``
tokens instead of every token; the output is trimmed to HF's stopping point.
"""
from __future__ import annotations

import os
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
    if _fused_ok(qkv, cache, li):
        # RoPE of q / k and the cache append of k / v in one kernel (rope_append, elementwise.hip)
        q = _native.kernels().rope_append(qkv.contiguous(), cos, sin, pos, hq, hkv, D, cos.shape[0],
                                          cache.k[li], cache.v[li], S)
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
    return _mlp(layer.mlp, x), residual


def _fused_ok(qkv, cache: KVCache, li: int) -> bool:
    return (qkv.is_cuda and qkv.dtype == torch.bfloat16 and cache.k[li].dtype == torch.bfloat16
            and qkv.shape[-1] % 8 == 0 and _native.kernels_available())


def _mlp(mlp, x):
    """Decode MLP: for 1-2 tokens (``GEMV_MAX_ROWS``) the down projection is a GEMV whose input
    SwiGLU is computed on the fly from the fused gate/up output (gemv.hip, one launch instead of
    SwiGLU + GEMV)."""
    from ..ops import linear as _lin
    down = mlp.down_proj
    if (_lin._GEMV and x.is_cuda and x.dtype == torch.bfloat16 and x.shape[0] <= _lin.GEMV_MAX_ROWS
            and type(down) is _lin.Linear and down.bias is None and down.weight.dtype == torch.bfloat16
            and down.weight.is_contiguous() and down.in_features % 8 == 0 and not torch.is_grad_enabled()):
        gu = mlp.gate_up_proj(x)
        if gu.is_contiguous() and gu.data_ptr() % 16 == 0 and gu.shape[-1] == 2 * down.in_features:
            return _native.kernels().gemv(gu, down.weight, swiglu=True)
        return down(ops.swiglu(gu))
    return mlp(x)


@torch.no_grad()
def forward_cached(model, ids: torch.Tensor, cache: KVCache) -> torch.Tensor:
    """Run `ids` [B, S] at positions cache.len ... ; returns last-position logits [B, V]."""
    B, S = ids.shape
    pos0 = cache.len
    if pos0 + S > cache.max_len:  # rope_append writes no cache row past max_len: refuse, don't truncate
        raise ValueError(f"KV cache overflow: {pos0} cached + {S} new tokens > max_len {cache.max_len}")
    cos, sin = model.rope(cache.max_len, ids.device)
    h = model.model.embed_tokens(ids).view(B * S, -1)
    residual = None
    for li, layer in enumerate(model.model.layers):
        h, residual = _layer_step(layer, h, residual, B, S, pos0, cos, sin, cache, li)
    x, _ = ops.add_rms_norm(h, residual, model.model.norm.weight, model.model.norm.eps)
    last = x.view(B, S, -1)[:, -1]
    cache.len += S
    return model.lm_head(last).float()


def _graph_layer_step(layer, h, residual, B, cos, sin, cache: KVCache, li: int, pos_b, pos_l, lens):
    """One-token layer step with every position-dependent value read from device tensors."""
    attn = layer.self_attn
    eps = layer.input_layernorm.eps
    if residual is None:
        residual = h
        x = ops.rms_norm(h, layer.input_layernorm.weight, eps)
    else:
        x, residual = ops.add_rms_norm(h, residual, layer.input_layernorm.weight, eps)
    qkv = attn.qkv_proj(x)
    hq, hkv, D = attn.hq, attn.hkv, attn.hd
    # the new token's position is its cache slot (pos_b == pos_l for every row)
    q = _native.kernels().rope_append(qkv.contiguous(), cos, sin, pos_b, hq, hkv, D, cos.shape[0],
                                      cache.k[li], cache.v[li], 1)
    o = ops.flash_attention(q.view(B, 1, hq, D), cache.k[li], cache.v[li], causal=False, seqlens_k=lens)
    h = attn.o_proj(o.reshape(B, hq * D))
    x, residual = ops.add_rms_norm(h, residual, layer.post_attention_layernorm.weight, eps)
    return _mlp(layer.mlp, x), residual


_GEMV_NORM = os.environ.get("GRT_GEMV_NORM", "1") != "0"


def _plain_bf16_linear(lin) -> bool:
    from ..ops import linear as _lin
    w = getattr(lin, "weight", None)
    return (isinstance(lin, _lin.Linear) and type(lin).forward is _lin.Linear.forward and lin.bias is None
            and w.dtype == torch.bfloat16 and w.is_cuda and w.is_contiguous() and w.shape[1] % 8 == 0
            and w.data_ptr() % 16 == 0)


GEMV_FUSED_MAX_ROWS = 4  # gemv_fused's row limit (TORCH_CHECK in csrc/bindings/ops.cpp)


def _norm_fusable(model, B: int) -> bool:
    """Every projection a plain bf16 Linear (no LoRA / NF4 wrappers, no bias) and 1-2 rows: the
    decode step can run with its residual adds / RMSNorms inside the GEMVs (gemv.hip)."""
    from ..ops import linear as _lin
    if not (_GEMV_NORM and _lin._GEMV and B <= min(_lin.GEMV_MAX_ROWS, GEMV_FUSED_MAX_ROWS) and _native.kernels_available()):
        return False
    m = model.model
    norms = [m.norm] + [n for ly in m.layers for n in (ly.input_layernorm, ly.post_attention_layernorm)]
    lins = [model.lm_head] + [p for ly in m.layers for p in (ly.self_attn.qkv_proj, ly.self_attn.o_proj,
                                                               ly.mlp.gate_up_proj, ly.mlp.down_proj)]
    if model.config.head_dim != 128:  # the RoPE epilogue / decode attention kernels
        return False
    return (all(_plain_bf16_linear(p) for p in lins)
            and all(n.weight.dtype == torch.bfloat16 and n.weight.is_contiguous() and n.weight.data_ptr() % 16 == 0
                    for n in norms))


class _NormWorkspace:
    """Fixed-point sums of squares of the residual stream's rows (gemv.hip): two [B, 64] slots, the
    producer GEMVs (o_proj, down_proj) alternate between them and each zeroes the other for the
    next one. 2 producers per layer, so the slot sequence repeats every token (graph replay)."""

    def __init__(self, B: int, device):
        self.sumsq = torch.zeros(2, B, 64, dtype=torch.int64, device=device)


def _fused_norm_layer_step(layer, h, first: bool, ws: _NormWorkspace, B, cos, sin, cache: KVCache, li: int,
                           pos_b, lens):
    """One-token layer step with the residual adds, RMSNorms and RoPE inside the GEMVs: o_proj /
    down_proj write h = y + residual and add sum(h^2) to a fixed-point accumulator, qkv / gate_up
    normalise their input on the fly from (h, accumulator, norm weight), and the qkv epilogue
    rotates q / k and appends k / v to the cache. ``h`` IS the residual stream between
    layers; slot 0 carries the post-attention norm's statistics, slot 1 the next input norm's."""
    K = _native.kernels()
    attn, mlp = layer.self_attn, layer.mlp
    ln1, ln2 = layer.input_layernorm, layer.post_attention_layernorm
    hq, hkv, D = attn.hq, attn.hkv, attn.hd
    # the qkv GEMV's epilogue applies RoPE and appends k / v to the cache (no rope_append launch)
    rope = dict(cos=cos, sin=sin, pos=pos_b, kc=cache.k[li], vc=cache.v[li], hq=hq, hkv=hkv)
    if first:  # layer 0: h is the embedding (no residual add, no producer GEMV summed its squares)
        q = K.gemv_fused(ops.rms_norm(h, ln1.weight, ln1.eps), attn.qkv_proj.weight, ws.sumsq, 1, **rope)
    else:
        q = K.gemv_fused(h, attn.qkv_proj.weight, ws.sumsq, 1, g=ln1.weight, eps=ln1.eps, **rope)
    o = ops.flash_attention(q.view(B, 1, hq, D), cache.k[li], cache.v[li], causal=False, seqlens_k=lens)
    h = K.gemv_fused(o.reshape(B, hq * D), attn.o_proj.weight, ws.sumsq, 0, res=h)
    gu = K.gemv_fused(h, mlp.gate_up_proj.weight, ws.sumsq, 0, g=ln2.weight, eps=ln2.eps)
    return K.gemv_fused(gu, mlp.down_proj.weight, ws.sumsq, 1, swiglu=True, res=h)


class GraphDecoder:
    """Greedy / sampling decode with the per-token step captured in a HIP graph (see module doc).

    Usage: ``dec = GraphDecoder(model, B, max_len)``; ``logits = dec.prefill(ids)`` (eager, any
    prompt length); then ``logits = dec.step(next_ids)`` per token (graph replay). Needs a bf16
    Llama on the GPU with head_dim 128 (the HIP RoPE / flash kernels)."""

    def __init__(self, model, B: int, max_len: int):
        self.model = model
        p = next(model.parameters())
        self.device = p.device
        dt = p.dtype if p.dtype in (torch.bfloat16, torch.float32) else torch.bfloat16
        self.cache = KVCache(model.config, B, max_len, self.device, dt)
        self.B = B
        self.cos, self.sin = model.rope(max_len, self.device)
        self.ids = torch.zeros(B, 1, dtype=torch.long, device=self.device)
        self.pos_b = torch.zeros(B, dtype=torch.int32, device=self.device)   # RoPE positions
        self.pos_l = torch.zeros(1, dtype=torch.long, device=self.device)    # cache write index
        self.lens = torch.zeros(B, dtype=torch.int32, device=self.device)    # valid keys incl. new token
        self.graph = None
        self.logits = None
        # residual adds / norms inside the GEMVs when every projection is a plain bf16 Linear
        self.norm_ws = (_NormWorkspace(B, self.device)
                        if self.device.type == "cuda" and _norm_fusable(model, B) else None)

    @torch.no_grad()
    def prefill(self, input_ids: torch.Tensor) -> torch.Tensor:
        logits = forward_cached(self.model, input_ids, self.cache)
        n = self.cache.len
        self.pos_b.fill_(n)
        self.pos_l.fill_(n)
        self.lens.fill_(n + 1)
        return logits

    @torch.no_grad()
    def _step_body(self):
        m = self.model
        h = m.model.embed_tokens(self.ids).view(self.B, -1)
        if self.norm_ws is not None:
            for li, layer in enumerate(m.model.layers):
                h = _fused_norm_layer_step(layer, h, li == 0, self.norm_ws, self.B, self.cos, self.sin,
                                           self.cache, li, self.pos_b, self.lens)
            fn = m.model.norm
            logits = _native.kernels().gemv_fused(h, m.lm_head.weight, self.norm_ws.sumsq, 1, g=fn.weight,
                                                  eps=fn.eps).float()
            self.pos_b.add_(1)
            self.pos_l.add_(1)
            self.lens.add_(1)
            return logits
        residual = None
        for li, layer in enumerate(m.model.layers):
            h, residual = _graph_layer_step(layer, h, residual, self.B, self.cos, self.sin, self.cache, li,
                                            self.pos_b, self.pos_l, self.lens)
        x, _ = ops.add_rms_norm(h, residual, m.model.norm.weight, m.model.norm.eps)
        logits = m.lm_head(x).float()
        self.pos_b.add_(1)
        self.pos_l.add_(1)
        self.lens.add_(1)
        return logits

    def _capture(self):
        # warm up on a side stream (allocator pools, library handles), then capture one step;
        # the warm-up step's cache writes land at the current position and are rewritten by the
        # first replay, and the position tensors are restored afterwards
        saved = (self.pos_b.clone(), self.pos_l.clone(), self.lens.clone())
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self._step_body()
        torch.cuda.current_stream(self.device).wait_stream(s)
        for t, v in zip((self.pos_b, self.pos_l, self.lens), saved):
            t.copy_(v)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.logits = self._step_body()
        for t, v in zip((self.pos_b, self.pos_l, self.lens), saved):
            t.copy_(v)

    @torch.no_grad()
    def step(self, next_ids: torch.Tensor) -> torch.Tensor:
        if self.cache.len >= self.cache.max_len:
            raise RuntimeError("KV cache full")
        self.ids.copy_(next_ids.view(self.B, 1))
        if self.graph is None:
            self._capture()
        self.graph.replay()
        self.cache.len += 1
        return self.logits


def _graph_ok(model, input_ids) -> bool:
    p = next(model.parameters())
    cfg = model.config
    return (input_ids.is_cuda and p.dtype == torch.bfloat16 and cfg.head_dim == 128
            and _native.kernels_available())


@torch.no_grad()
def generate(model, input_ids: torch.Tensor, max_new_tokens: int = 32,
             eos_token_id: Optional[Union[int, List[int]]] = None, do_sample: bool = False, temperature: float = 1.0,
             top_p: Optional[float] = None, attention_mask=None, pad_token_id=None, generator=None,
             use_graph: Optional[bool] = None, sync_every: int = 16, **_):
    """Returns [B, prompt + generated] token ids (HF ``generate`` output convention)."""
    was = model.training
    model.eval()
    B, S = input_ids.shape
    eos = set([eos_token_id] if isinstance(eos_token_id, int) else (eos_token_id or []))
    eos_t = torch.tensor(sorted(eos), device=input_ids.device) if eos else None
    graph = use_graph if use_graph is not None else _graph_ok(model, input_ids)
    if graph:
        dec = GraphDecoder(model, B, S + max_new_tokens)
        logits = dec.prefill(input_ids)
        forward = dec.step
    else:
        p = next(model.parameters())
        cache = KVCache(model.config, B, S + max_new_tokens, input_ids.device,
                        p.dtype if p.dtype in (torch.bfloat16, torch.float32) else torch.bfloat16)
        logits = forward_cached(model, input_ids, cache)

        def forward(nxt):
            return forward_cached(model, nxt[:, None], cache)
    out = [input_ids]
    finished = torch.zeros(B, dtype=torch.bool, device=input_ids.device)
    all_done = []  # device flags: every row finished after token t
    for t in range(max_new_tokens):
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
        if eos_t is not None:
            finished |= torch.isin(nxt, eos_t)
            all_done.append(finished.all())
            if (t + 1) % sync_every == 0 and bool(finished.all()):
                break
        if t + 1 < max_new_tokens:
            logits = forward(nxt)
    if all_done:  # HF stops right after the token that finished the last row
        flags = torch.stack(all_done)
        if bool(flags.any()):
            first = int(flags.nonzero()[0, 0])
            out = out[:first + 2]
    if was:
        model.train()
    return torch.cat(out, 1)
