"""Pure-PyTorch reference implementations of every native op.

Used (a) on CPU hosts (gloo plumbing runs, unit tests) and (b) as the fp32 numerics oracle of
the HIP kernels in the GPU tests. Semantics mirror the HF / torch modules the reference scripts
run (Llama RMSNorm rounding, erf GELU, rotate-half RoPE, CE with ignore_index=-100).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def rmsnorm(x, w, eps, residual=None):
    h = x if residual is None else (x + residual)
    hf = h.float()
    rstd = torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps)
    y = (hf * rstd * w.float()).to(x.dtype)
    return y, h


def layernorm(x, w, b, eps, residual=None):
    h = x if residual is None else (x + residual)
    y = F.layer_norm(h.float(), (h.shape[-1],), w.float(), None if b is None else b.float(), eps).to(x.dtype)
    return y, h


def swiglu(gu):
    g, u = gu.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gu.dtype)


def gelu(x):
    return F.gelu(x.float(), approximate="none").to(x.dtype)


def rope_tables(seq_len, head_dim, theta=10000.0, device=None, scaling=None):
    """cos/sin tables [S, D/2] fp32 for the rotate-half convention.

    ``scaling`` = dict(type="llama3", factor, low_freq_factor, high_freq_factor,
    original_max_position_embeddings) reproduces Llama-3.1's frequency scaling.
    """
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("type", scaling.get("rope_type")) == "llama3":
        factor = scaling["factor"]
        lf, hf = scaling["low_freq_factor"], scaling["high_freq_factor"]
        old = scaling["original_max_position_embeddings"]
        low_wl, high_wl = old / lf, old / hf
        wl = 2 * math.pi / inv
        scaled = torch.where(wl > low_wl, inv / factor, inv)
        smooth = (old / wl - lf) / (hf - lf)
        mid = (1 - smooth) * scaled / factor + smooth * scaled
        is_mid = (wl >= high_wl) & (wl <= low_wl)
        inv = torch.where(is_mid, mid, scaled)
    t = torch.arange(seq_len, dtype=torch.float64)
    fr = torch.outer(t, inv)
    return fr.cos().float().to(device), fr.sin().float().to(device)


def apply_rope(x, cos, sin, pos=None):
    """x: [T, H, D]; cos/sin [S, D/2]; position of row t = pos[t] or t % S."""
    T = x.shape[0]
    S = cos.shape[0]
    idx = pos.long() if pos is not None else torch.arange(T, device=x.device) % S
    c = cos[idx].unsqueeze(1)
    s = sin[idx].unsqueeze(1)
    xf = x.float()
    x1, x2 = xf.chunk(2, dim=-1)
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(x.dtype)


_M32 = 0xFFFFFFFF


def _fmix32(h):
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & _M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & _M32
    return h ^ (h >> 16)


def attn_dropout_keep(seed: int, B: int, H: int, Sq: int, Sk: int, p: float, device=None) -> torch.Tensor:
    """[B, H, Sq, Sk] bool keep-mask of the attention-probability dropout, bit-identical to the
    counter hash of csrc/kernels/attention.hip (element (b*H + h, q, k))."""
    thresh = min(_M32, math.ceil(p * 2 ** 32))
    bh = torch.arange(B * H, device=device, dtype=torch.int64).view(B, H, 1, 1)
    q = torch.arange(Sq, device=device, dtype=torch.int64).view(1, 1, Sq, 1)
    k = torch.arange(Sk, device=device, dtype=torch.int64).view(1, 1, 1, Sk)
    h = (seed & _M32) ^ ((bh * 0x9E3779B1) & _M32)
    h = _fmix32(h ^ ((q * 0x85EBCA77) & _M32))
    h = _fmix32(h ^ ((k * 0xC2B2AE3D) & _M32))
    return h >= thresh


def _splitmix64(x):
    """numpy uint64 splitmix64 finaliser (wrapping arithmetic), as hash_u64 in elementwise.hip."""
    import numpy as np
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def dropout_keep_mask(seed: int, offset: int, n: int, p: float) -> torch.Tensor:
    """[n] bool keep-mask of the element dropout kernels (elementwise.hip ``drop_keep``),
    recomputed independently on the host: element i keeps iff 16 bits of
    splitmix64(splitmix64(seed) ^ ((offset + i) / 4)), selected by (offset + i) % 4, are
    >= round(p * 65536)."""
    import numpy as np
    key = _splitmix64(np.array([seed & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64))[0]
    idx = np.arange(offset, offset + n, dtype=np.uint64)
    h = _splitmix64(key ^ (idx >> np.uint64(2)))
    bits = (h >> (np.uint64(16) * (idx & np.uint64(3)))) & np.uint64(0xFFFF)
    thr = int(np.float32(p) * np.float32(65536.0) + np.float32(0.5))
    return torch.from_numpy(bits >= np.uint64(thr))


def attention(q, k, v, causal=True, scale=None, seqlens_k=None, dropout_p=0.0, seed=0):
    """q [B,Sq,Hq,D], k/v [B,Sk,Hkv,D] -> o [B,Sq,Hq,D]; math in fp32 (explicit matmul/softmax —
    no SDPA backend dispatch). ``dropout_p`` drops attention probabilities with the kernel's mask."""
    B, Sq, Hq, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    rep = Hq // Hkv
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    mask = torch.zeros(Sq, Sk, dtype=torch.bool, device=q.device)
    if causal:
        off = Sk - Sq
        mask = torch.arange(Sk, device=q.device)[None, :] > (torch.arange(Sq, device=q.device)[:, None] + off)
    mask = mask[None, None].expand(B, 1, Sq, Sk)
    if seqlens_k is not None:
        kv = torch.arange(Sk, device=q.device)[None, :] >= seqlens_k.to(q.device).long()[:, None]
        mask = mask | kv[:, None, None, :]
    s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    if dropout_p > 0.0:
        keep = attn_dropout_keep(seed, B, Hq, Sq, Sk, dropout_p, device=q.device)
        p = p * keep.to(p.dtype) / (1.0 - dropout_p)
    o = torch.matmul(p, vf).transpose(1, 2)
    return o.to(q.dtype)


def cross_entropy(logits, labels, ignore_index=-100):
    return F.cross_entropy(logits.float(), labels, ignore_index=ignore_index)


def adamw_(p, g, m, v, step, lr, beta1, beta2, eps, wd, grad_scale=1.0, master=None):
    """In-place torch.optim.AdamW semantics (decoupled decay) on fp32 state."""
    pf = master if master is not None else p.float()
    gf = g.float() * grad_scale
    m.mul_(beta1).add_(gf, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(gf, gf, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    pf.mul_(1 - lr * wd)
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    pf.addcdiv_(m, denom, value=-lr / bc1)
    if master is not None:
        p.copy_(pf)
    else:
        p.copy_(pf.to(p.dtype))


NF4_CODE = torch.tensor([
    -1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453,
    -0.28444138169288635, -0.18477343022823334, -0.09105003625154495, 0.0,
    0.07958029955625534, 0.16093020141124725, 0.24611230194568634, 0.33791524171829224,
    0.44070982933044434, 0.5626170039176941, 0.7229568362236023, 1.0])


def nf4_quantize(w, blocksize=64):
    flat = w.reshape(-1).float()
    blocks = flat.view(-1, blocksize)
    absmax = blocks.abs().amax(dim=1)
    normed = blocks / absmax.clamp_min(1e-30)[:, None]
    code = NF4_CODE.to(w.device)
    mids = (code[1:] + code[:-1]) / 2
    idx = (normed.unsqueeze(-1) > mids).sum(-1).to(torch.uint8).view(-1)
    packed = (idx[0::2] << 4) | idx[1::2]
    return packed, absmax


def nf4_dequantize(packed, absmax, n, blocksize=64, dtype=torch.bfloat16):
    code = NF4_CODE.to(packed.device)
    hi = (packed >> 4).long()
    lo = (packed & 15).long()
    idx = torch.stack([hi, lo], dim=1).view(-1)
    vals = code[idx].view(-1, blocksize) * absmax[:, None]
    return vals.view(-1)[:n].to(dtype)
