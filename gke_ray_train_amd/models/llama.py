"""Llama-2 / Llama-3 / Llama-3.1 causal LM, laid out for MI355X.

Reference role: ``AutoModelForCausalLM.from_pretrained("meta-llama/Meta-Llama-3.1-8B-Instruct")``
in the SFT job (reference ray-jobs/fine_tune_llama_ray.py:229-241, fine_tune_config.json:2);
``BASELINE.json`` adds Llama-2-7B (DDP / FSDP / LoRA) and Llama-3-70B (FSDP + offload).

MI355X-first layout decisions:
* Q/K/V are ONE fused projection (``qkv_proj``) and gate/up are ONE fused projection
  (``gate_up_proj``): one large hipBLASLt GEMM each instead of three / two, and the attention
  kernel reads Q/K/V straight out of the fused output (RoPE + flash attention are one autograd
  op, ``ops.rope_attention``) with no split/transposes in either direction.
* the residual stream is threaded through ``add_rms_norm`` so every residual add is fused into
  the following RMSNorm kernel;
* the LM head and the loss are one op (``ops.lm_head_cross_entropy``): the bf16 logits buffer is
  reused for dlogits, labels are shifted instead of the logits (no [tokens, V] slice copy).
* HF parameter names are preserved at the checkpoint boundary (``hf_state_dict`` /
  ``load_hf_state_dict``): the fused weights are split / concatenated there, so real HF
  checkpoints load and ``save_pretrained`` output is HF-layout.
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, field
from typing import Optional

import torch
import torch.nn as nn
import torch.utils.checkpoint as ckpt

from .. import ops
from ..ops.linear import Embedding, Linear
from ..ops import _ref


@dataclass
class LlamaConfig:
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 32
    max_position_embeddings: int = 4096
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    rope_scaling: Optional[dict] = None
    tie_word_embeddings: bool = False
    initializer_range: float = 0.02
    bos_token_id: int = 1
    eos_token_id: int = 2
    pad_token_id: Optional[int] = None
    model_type: str = "llama"
    name: str = "llama"

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads

    def num_params(self, include_embeddings=True) -> int:
        d, f, L, V = self.hidden_size, self.intermediate_size, self.num_hidden_layers, self.vocab_size
        hd = self.head_dim
        attn = d * (self.num_attention_heads * hd) + 2 * d * (self.num_key_value_heads * hd) + (self.num_attention_heads * hd) * d
        mlp = 3 * d * f
        per_layer = attn + mlp + 2 * d
        emb = V * d * (1 if self.tie_word_embeddings else 2)
        return L * per_layer + d + (emb if include_embeddings else 0)

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs/token: 6 * matmul params + causal attention (fwd+bwd = 3x fwd)."""
        n = self.num_params(include_embeddings=False) + self.vocab_size * self.hidden_size  # lm_head GEMM
        attn = 3 * 2 * 2 * self.num_hidden_layers * seq_len * self.hidden_size / 2  # QK^T + PV, causal half
        return 6.0 * n + attn

    def to_hf_dict(self) -> dict:
        d = asdict(self)
        d.pop("name")
        d["architectures"] = ["LlamaForCausalLM"]
        d["hidden_act"] = "silu"
        d["torch_dtype"] = "bfloat16"
        return d


CONFIGS = {
    "llama2-7b": dict(vocab_size=32000, hidden_size=4096, intermediate_size=11008, num_hidden_layers=32,
                      num_attention_heads=32, num_key_value_heads=32, max_position_embeddings=4096,
                      rope_theta=10000.0, rms_norm_eps=1e-5, name="llama2-7b"),
    "llama2-13b": dict(vocab_size=32000, hidden_size=5120, intermediate_size=13824, num_hidden_layers=40,
                       num_attention_heads=40, num_key_value_heads=40, max_position_embeddings=4096,
                       name="llama2-13b"),
    "llama3-8b": dict(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                      num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=8192,
                      rope_theta=500000.0, bos_token_id=128000, eos_token_id=128001, name="llama3-8b"),
    "llama3.1-8b": dict(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                        num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=131072,
                        rope_theta=500000.0, bos_token_id=128000, eos_token_id=128009,
                        rope_scaling=dict(type="llama3", factor=8.0, low_freq_factor=1.0, high_freq_factor=4.0,
                                          original_max_position_embeddings=8192), name="llama3.1-8b"),
    "llama3-70b": dict(vocab_size=128256, hidden_size=8192, intermediate_size=28672, num_hidden_layers=80,
                       num_attention_heads=64, num_key_value_heads=8, max_position_embeddings=8192,
                       rope_theta=500000.0, bos_token_id=128000, eos_token_id=128001, name="llama3-70b"),
    # small configs for tests / smoke (head_dim 128 so the HIP attention path is exercised)
    "llama-tiny": dict(vocab_size=512, hidden_size=256, intermediate_size=688, num_hidden_layers=2,
                       num_attention_heads=2, num_key_value_heads=2, max_position_embeddings=512, name="llama-tiny"),
    "llama-tiny-gqa": dict(vocab_size=512, hidden_size=512, intermediate_size=1376, num_hidden_layers=2,
                           num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512,
                           name="llama-tiny-gqa"),
    "llama-125m": dict(vocab_size=32000, hidden_size=768, intermediate_size=2048, num_hidden_layers=12,
                       num_attention_heads=6, num_key_value_heads=6, max_position_embeddings=2048, name="llama-125m"),
}
CONFIGS["meta-llama/Llama-2-7b-hf"] = CONFIGS["llama2-7b"]
CONFIGS["meta-llama/Meta-Llama-3.1-8B-Instruct"] = CONFIGS["llama3.1-8b"]
CONFIGS["meta-llama/Meta-Llama-3-8B"] = CONFIGS["llama3-8b"]
CONFIGS["meta-llama/Meta-Llama-3-70B"] = CONFIGS["llama3-70b"]


def get_config(name: str, **overrides) -> LlamaConfig:
    if name not in CONFIGS:
        raise KeyError(f"unknown Llama config {name!r}; known: {sorted(CONFIGS)}")
    d = dict(CONFIGS[name])
    d.update(overrides)
    return LlamaConfig(**d)


def _tail_pad(proj) -> int:
    """Columns a K-concatenated LoRA projection (peft/lora.py) wants after each row of its input, so
    the producer (norm / attention / SwiGLU kernel) writes that input into a [rows, in + pad] row
    buffer and the adapter's h lands beside it; 0 for a plain projection."""
    return getattr(proj, "kcat_pad", 0)


class FusedLinear(Linear):
    """nn.Linear whose output columns are the concatenation of named HF projections."""

    def __init__(self, in_features, slices, bias=False, device=None, dtype=None):
        super().__init__(in_features, sum(n for _, n in slices), bias=bias, device=device, dtype=dtype)
        self.slices = list(slices)


class LlamaAttention(nn.Module):
    def __init__(self, cfg: LlamaConfig, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        hd = cfg.head_dim
        self.hq, self.hkv, self.hd = cfg.num_attention_heads, cfg.num_key_value_heads, hd
        self.qkv_proj = FusedLinear(cfg.hidden_size, [("q_proj", self.hq * hd), ("k_proj", self.hkv * hd),
                                                      ("v_proj", self.hkv * hd)], device=device, dtype=dtype)
        self.o_proj = Linear(self.hq * hd, cfg.hidden_size, bias=False, device=device, dtype=dtype)

    def forward(self, x, B, S, cos, sin, varlen=None):
        qkv = self.qkv_proj(x)
        sp = getattr(self, "sp_group", None)
        if sp is not None:  # sequence parallel: S is this rank's token count (parallel/sequence.py)
            if varlen is not None:
                raise NotImplementedError("padding-free packing with sequence parallelism")
            from ..parallel.sequence import ulysses_attention
            o = ulysses_attention(qkv, cos, sin, B, S, self.hq, self.hkv, self.hd, sp, causal=True)
        else:
            o = ops.rope_attention(qkv, cos, sin, B, S, self.hq, self.hkv, self.hd, causal=True, varlen=varlen,
                                   pad=_tail_pad(self.o_proj), bwd_t=_direct_wgrad(self.qkv_proj),
                                   fwd_t=_direct_wgrad(self.o_proj))
        return self.o_proj(o)


def _direct_wgrad(lin) -> bool:
    """``lin``'s weight gradient runs on the direct TN path of ops/linear.py in this forward."""
    w = getattr(lin, "weight", None)
    return (isinstance(w, torch.Tensor) and w.requires_grad and w.is_cuda and torch.is_grad_enabled()
            and getattr(w, "_grt_slot", None) is not None)


class LlamaMLP(nn.Module):
    def __init__(self, cfg: LlamaConfig, device=None, dtype=None):
        super().__init__()
        f = cfg.intermediate_size
        self.gate_up_proj = FusedLinear(cfg.hidden_size, [("gate_proj", f), ("up_proj", f)], device=device, dtype=dtype)
        self.down_proj = Linear(f, cfg.hidden_size, bias=False, device=device, dtype=dtype)

    def forward(self, x):
        # trainable projections on the direct-gradient path take their weight-gradient operand
        # transposed from the SwiGLU kernels (h^T for down, dgu^T for gate / up)
        return self.down_proj(ops.swiglu(self.gate_up_proj(x), pad=_tail_pad(self.down_proj),
                                         fwd_t=_direct_wgrad(self.down_proj), bwd_t=_direct_wgrad(self.gate_up_proj)))


class RMSNorm(nn.Module):
    # the fused HIP backward (ops/fused.py) writes the weight gradient into the data-parallel slot
    _grt_direct_grad = True

    def __init__(self, d, eps, device=None, dtype=None):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d, device=device, dtype=dtype))
        self.eps = eps

    def forward(self, x, residual=None):
        """rms_norm(x) or, with ``residual``, the fused (norm(x + residual), x + residual)."""
        if residual is None:
            return ops.rms_norm(x, self.weight, self.eps)
        return ops.add_rms_norm(x, residual, self.weight, self.eps)


class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig, device=None, dtype=None):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, device, dtype)
        self.self_attn = LlamaAttention(cfg, device, dtype)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, device, dtype)
        self.mlp = LlamaMLP(cfg, device, dtype)

    def forward(self, h, residual, B, S, cos, sin, varlen=None):
        eps = self.input_layernorm.eps
        pad = _tail_pad(self.self_attn.qkv_proj)
        if residual is None:
            residual = h
            x = ops.rms_norm(h, self.input_layernorm.weight, eps, pad=pad)
        else:
            x, residual = ops.add_rms_norm(h, residual, self.input_layernorm.weight, eps, pad=pad)
        h = self.self_attn(x, B, S, cos, sin, varlen)
        x, residual = ops.add_rms_norm(h, residual, self.post_attention_layernorm.weight, eps,
                                       pad=_tail_pad(self.mlp.gate_up_proj))
        return self.mlp(x), residual


class LlamaModel(nn.Module):
    def __init__(self, cfg: LlamaConfig, device=None, dtype=None):
        super().__init__()
        self.embed_tokens = Embedding(cfg.vocab_size, cfg.hidden_size, device=device, dtype=dtype)
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg, device, dtype) for _ in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps, device, dtype)


class LlamaForCausalLM(nn.Module):
    """``forward(input_ids, labels=None) -> dict(loss=..., logits=...)`` (HF-style semantics:
    labels are the input ids, the model shifts them; ``-100`` is ignored)."""

    def __init__(self, cfg: LlamaConfig, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.config = cfg
        self.model = LlamaModel(cfg, device, dtype)
        self.lm_head = Linear(cfg.hidden_size, cfg.vocab_size, bias=False, device=device, dtype=dtype)
        if cfg.tie_word_embeddings:
            self.lm_head.weight = self.model.embed_tokens.weight
        self.gradient_checkpointing = False
        self._rope = {}

    # -------------------------------------------------------------- init
    @torch.no_grad()
    def init_weights(self, seed: Optional[int] = None):
        """HF LlamaPreTrainedModel._init_weights: N(0, 0.02) linears/embeddings, ones for norms."""
        g = None
        if seed is not None:
            dev = next(self.parameters()).device
            g = torch.Generator(device=dev)
            g.manual_seed(seed)
        std = self.config.initializer_range
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                m.weight.normal_(0.0, std, generator=g)
                if getattr(m, "bias", None) is not None:
                    m.bias.zero_()
            elif isinstance(m, RMSNorm):
                m.weight.fill_(1.0)
        return self

    def gradient_checkpointing_enable(self, enable: bool = True):
        self.gradient_checkpointing = enable

    def rope(self, S, device):
        key = (S, str(device))
        t = self._rope.get(key)
        if t is None:
            t = _ref.rope_tables(max(S, 1), self.config.head_dim, self.config.rope_theta, device=device,
                                 scaling=self.config.rope_scaling)
            self._rope[key] = t
        return t

    # -------------------------------------------------------------- forward
    def hidden_states(self, input_ids, varlen=None):
        B, S = input_ids.shape
        # sequence parallel: RoPE tables span the full sequence (this rank holds S of S * sp_size);
        # padding-free packing: positions restart per sequence, so the longest one bounds the table
        n = varlen.max_len if varlen is not None else S * getattr(self, "sp_size", 1)
        cos, sin = self.rope(n, input_ids.device)
        h = self.model.embed_tokens(input_ids).view(B * S, -1)
        residual = None
        for layer in self.model.layers:
            if self.gradient_checkpointing and self.training and torch.is_grad_enabled():
                if residual is None:
                    h, residual = ckpt.checkpoint(lambda a, L=layer: L(a, None, B, S, cos, sin, varlen), h,
                                                  use_reentrant=False)
                else:
                    h, residual = ckpt.checkpoint(layer, h, residual, B, S, cos, sin, varlen, use_reentrant=False)
            else:
                h, residual = layer(h, residual, B, S, cos, sin, varlen)
        x, _ = self.model.norm(h, residual)
        return x

    def forward(self, input_ids, labels=None, attention_mask=None, return_logits=None, shifted_labels=None,
                loss_weights=None, varlen=None):
        """``labels``: HF convention (shifted here). ``shifted_labels``: already next-token aligned
        (sequence-parallel shards, whose last token's label lives on the next rank).
        ``loss_weights`` ([B, S] fp32, optional): the loss is the weighted SUM of the per-position
        next-token CE (position t predicts t+1) instead of the mean over valid positions.
        ``varlen`` (``ops.Varlen``): ``input_ids`` [1, T] holds padding-free packed sequences —
        no padding tokens in any GEMM; attention stays inside each sequence, positions restart,
        and the last token of a sequence predicts nothing (its shifted label is -100)."""
        B, S = input_ids.shape
        if varlen is not None and (B != 1 or varlen.total != S):
            raise ValueError(f"varlen packing expects input_ids [1, {varlen.total}], got {tuple(input_ids.shape)}")
        x = self.hidden_states(input_ids, varlen)
        out = {}
        rw = None if loss_weights is None else loss_weights.reshape(-1)
        if shifted_labels is not None:
            out["loss"] = self.lm_head(x, labels=shifted_labels.reshape(-1), row_weights=rw)
        elif labels is not None:
            # shift labels (not logits): position t predicts token t+1
            shifted = torch.full_like(labels, -100)
            shifted[:, :-1] = labels[:, 1:]
            if attention_mask is not None:
                shifted[:, :-1].masked_fill_(attention_mask[:, 1:] == 0, -100)
            if varlen is not None:  # a sequence's last token does not predict the next sequence's first
                # index_fill_ with a device index: no host scalar upload (a blocking copy per step)
                shifted[0].index_fill_(0, varlen.cu[1:].long() - 1, -100)
            out["loss"] = self.lm_head(x, labels=shifted.view(-1), row_weights=rw)
        if (labels is None and shifted_labels is None) or return_logits:
            out["logits"] = self.lm_head(x).view(B, S, -1)
        return out

    # -------------------------------------------------------------- HF checkpoint boundary
    def hf_state_dict(self) -> dict:
        """State dict with HF LlamaForCausalLM parameter names (fused weights split)."""
        out = {}
        for name, t in self.state_dict().items():
            mod_name = name.rsplit(".", 1)[0]
            mod = self.get_submodule(mod_name) if mod_name else self
            if isinstance(mod, FusedLinear) and name.endswith(".weight"):
                base = mod_name.rsplit(".", 1)[0]
                start = 0
                for sub, n in mod.slices:
                    out[f"{base}.{sub}.weight"] = t[start:start + n]
                    start += n
            else:
                out[name] = t
        return out

    @torch.no_grad()
    def load_hf_state_dict(self, sd: dict, strict: bool = True):
        own = {}
        for name, mod in self.named_modules():
            if isinstance(mod, FusedLinear):
                base = name.rsplit(".", 1)[0]
                parts = [sd[f"{base}.{sub}.weight"] for sub, _ in mod.slices if f"{base}.{sub}.weight" in sd]
                if len(parts) == len(mod.slices):
                    own[f"{name}.weight"] = torch.cat(parts, 0)
        for k, v in sd.items():
            if any(k.endswith(f".{sub}.weight") for sub in ("q_proj", "k_proj", "v_proj", "gate_proj", "up_proj")):
                continue
            own[k] = v
        missing, unexpected = self.load_state_dict(own, strict=False)
        if strict and (missing or unexpected):
            raise RuntimeError(f"HF load mismatch: missing={missing} unexpected={unexpected}")
        return missing, unexpected


def _generate(self, input_ids, **kw):
    """KV-cache greedy / sampling decode (models/generation.py)."""
    from .generation import generate
    return generate(self, input_ids, **kw)


def _save_pretrained(self, path, **kw):
    from .hub import save_pretrained
    save_pretrained(self, path, **kw)


LlamaForCausalLM.generate = _generate
LlamaForCausalLM.save_pretrained = _save_pretrained


def build_llama(name_or_cfg="llama2-7b", device=None, dtype=torch.bfloat16, seed: Optional[int] = 0, **overrides):
    cfg = name_or_cfg if isinstance(name_or_cfg, LlamaConfig) else get_config(name_or_cfg, **overrides)
    model = LlamaForCausalLM(cfg, device=device, dtype=dtype)
    model.init_weights(seed)
    return model
