"""NF4 (4-bit NormalFloat) frozen linear layer for QLoRA.

Reference role: ``BitsAndBytesConfig(load_in_4bit=True, bnb_4bit_quant_type="nf4",
bnb_4bit_compute_dtype=bfloat16, bnb_4bit_use_double_quant=USE_NESTED_QUANT)``
(ray-jobs/fine_tune_llama_ray.py:215-227). Weights are quantised once on the GPU by the HIP
kernel (blocks of 64, fp32 absmax); forward and backward dequantise into a bf16 weight (never
stored for autograd, so the base model costs ~0.53 bytes/param resident) and run the hipBLASLt
GEMM — or, when ``set_dequant_cache`` finds room in HBM (auto for 8B on a 288 GB MI355X), reuse a
resident dequantised W / W^T (bit-identical; the base is frozen). ``double_quant`` additionally stores the absmax vector as 8-bit codes
with one fp32 scale per 256 blocks (bitsandbytes' nested quantisation) and expands it on device.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


@dataclass
class BitsAndBytesConfig:
    load_in_4bit: bool = True
    bnb_4bit_quant_type: str = "nf4"
    bnb_4bit_compute_dtype: torch.dtype = torch.bfloat16
    bnb_4bit_use_double_quant: bool = False
    blocksize: int = 64

    def __post_init__(self):
        if isinstance(self.bnb_4bit_compute_dtype, str):
            self.bnb_4bit_compute_dtype = getattr(torch, self.bnb_4bit_compute_dtype)
        if self.bnb_4bit_quant_type != "nf4":
            raise ValueError("only nf4 is implemented")


class _NF4Matmul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, layer):
        w = layer.dequantize()
        ctx.layer = layer
        return F.linear(x, w)

    @staticmethod
    def backward(ctx, dy):
        # recomputed (the bf16 weight is never kept alive for autograd), dequantised transposed
        return ctx.layer.input_grad(dy), None


class NF4Linear(nn.Module):
    def __init__(self, in_features: int, out_features: int, compute_dtype=torch.bfloat16, blocksize: int = 64,
                 double_quant: bool = False, device=None, slices=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.compute_dtype = compute_dtype
        self.blocksize = blocksize
        self.double_quant = double_quant
        n = in_features * out_features
        self.register_buffer("qweight", torch.zeros(n // 2, dtype=torch.uint8, device=device))
        nb = n // blocksize
        if double_quant:
            self.register_buffer("absmax_q", torch.zeros(nb, dtype=torch.uint8, device=device))
            self.register_buffer("absmax_scale", torch.zeros((nb + 255) // 256, dtype=torch.float32, device=device))
            self.register_buffer("absmax_offset", torch.zeros(1, dtype=torch.float32, device=device))
        else:
            self.register_buffer("absmax", torch.zeros(nb, dtype=torch.float32, device=device))
        if slices is not None:
            self.slices = list(slices)

    @classmethod
    @torch.no_grad()
    def from_linear(cls, lin: nn.Linear, cfg: BitsAndBytesConfig) -> "NF4Linear":
        w = lin.weight.detach()
        m = cls(lin.in_features, lin.out_features, cfg.bnb_4bit_compute_dtype, cfg.blocksize,
                cfg.bnb_4bit_use_double_quant, device=w.device, slices=getattr(lin, "slices", None))
        q, a = ops.nf4_quantize(w.contiguous().view(-1), cfg.blocksize)
        m.qweight.copy_(q)
        if cfg.bnb_4bit_use_double_quant:
            off = a.mean()
            c = a - off
            blocks = F.pad(c, (0, (-c.numel()) % 256)).view(-1, 256)
            sc = blocks.abs().amax(1).clamp_min(1e-12)
            codes = torch.round(blocks / sc[:, None] * 127).clamp(-127, 127).to(torch.int16) + 128
            m.absmax_q.copy_(codes.view(-1)[: a.numel()].to(torch.uint8))
            m.absmax_scale.copy_(sc)
            m.absmax_offset.fill_(float(off))
        else:
            m.absmax.copy_(a)
        return m

    def _absmax(self) -> torch.Tensor:
        if not self.double_quant:
            return self.absmax
        nb = self.absmax_q.numel()
        codes = self.absmax_q.to(torch.float32) - 128.0
        sc = self.absmax_scale.repeat_interleave(256)[:nb]
        return codes / 127.0 * sc + self.absmax_offset

    def _dequant(self) -> torch.Tensor:
        n = self.in_features * self.out_features
        w = ops.nf4_dequantize(self.qweight, self._absmax().contiguous(), n, self.blocksize, self.compute_dtype)
        return w.view(self.out_features, self.in_features)

    def _dequant_t(self) -> Optional[torch.Tensor]:
        if self.qweight.is_cuda and self.compute_dtype == torch.bfloat16 and self.blocksize == 64 \
                and self.in_features % 64 == 0 and self.out_features % 8 == 0:
            from .. import _native
            return _native.kernels().nf4_dequantize_t(self.qweight, self._absmax().contiguous(), self.out_features,
                                                      self.in_features, self.blocksize)
        return None

    def dequantize_into(self, out: torch.Tensor) -> torch.Tensor:
        """bf16 W written into ``out`` ([out_features, in_features] view with unit column stride, any
        row stride: the W head of the K-concatenated [W | B] buffer of peft/lora.py), returned."""
        if out.is_cuda and self.compute_dtype == torch.bfloat16 and out.dtype == torch.bfloat16:
            from .. import _native
            if _native.kernels().nf4_dequantize_into(self.qweight, self._absmax().contiguous(), out, self.blocksize):
                return out
        return out.copy_(self._dequant())

    def _cache_key(self):
        return (self.qweight.data_ptr(), self.qweight._version)

    def dequantize(self) -> torch.Tensor:
        """bf16 W [out, in]. With the dequant cache on (``set_dequant_cache``) the result of the
        first call is kept until the packed weights change (frozen base: never in training)."""
        if getattr(self, "_cache_on", False):
            c = getattr(self, "_w_cache", None)
            if c is None or c[0] != self._cache_key():
                self._w_cache = c = (self._cache_key(), self._dequant())
            return c[1]
        return self._dequant()

    def input_grad(self, dy: torch.Tensor, acc: Optional[torch.Tensor] = None) -> torch.Tensor:
        """dX = dY W: on MI355X the HIP kernel dequantises straight into W^T so the GEMM runs in the
        TN layout (ops.linear.input_grad); elsewhere dY @ W. With ``acc``: acc += dY W (the GEMM's
        beta = 1 epilogue), returned."""
        if getattr(self, "_cache_on", False):
            c = getattr(self, "_wt_cache", None)
            if c is None or c[0] != self._cache_key():
                self._wt_cache = c = (self._cache_key(), self._dequant_t())
            wt = c[1]
        else:
            wt = self._dequant_t() if dy.is_cuda else None
        if acc is not None:
            return acc.addmm_(dy, wt.t()) if wt is not None else acc.addmm_(dy, self.dequantize())
        if wt is not None:
            return F.linear(dy, wt)
        return dy @ self.dequantize()

    def prepare_input_grad(self):
        """Build the cached W^T of ``input_grad`` now (no-op without the dequant cache)."""
        if getattr(self, "_cache_on", False):
            c = getattr(self, "_wt_cache", None)
            if c is None or c[0] != self._cache_key():
                self._wt_cache = (self._cache_key(), self._dequant_t())

    def set_dequant_cache(self, on: bool):
        self._cache_on = bool(on)
        if not on:
            self._w_cache = self._wt_cache = None

    @property
    def weight(self):  # dequantised copy (merge_and_unload, inspection): never the cached tensor
        return self._dequant()

    def forward(self, x):
        if x.dtype != self.compute_dtype:
            x = x.to(self.compute_dtype)
        if torch.is_grad_enabled() and x.requires_grad:
            return _NF4Matmul.apply(x, self)
        return F.linear(x, self.dequantize())


def quantize_model_(model: nn.Module, cfg: BitsAndBytesConfig, skip=("lm_head",)) -> nn.Module:
    """Replace every nn.Linear (except ``skip``) by an NF4Linear, in place."""
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            full = f"{name}.{cname}" if name else cname
            if isinstance(child, nn.Linear) and not any(full.endswith(s) for s in skip):
                setattr(mod, cname, NF4Linear.from_linear(child, cfg))
                del child
    for p in model.parameters():
        p.requires_grad_(False)
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    set_dequant_cache(model)
    return model


def set_dequant_cache(model: nn.Module, mode: Optional[str] = None, budget_fraction: float = 0.15) -> bool:
    """Keep each NF4 layer's dequantised bf16 W and W^T resident instead of re-dequantising them in
    every forward and backward.

    The base weights are frozen, so the dequantised values never change: caching is bit-identical
    to dequantising per use. It trades HBM for time — 4 bytes per base parameter on top of the
    0.53 of the packed NF4 — which on a 288 GB MI355X is ~28 GB for Llama-3.1-8B (the SFT job's
    dequant kernels were 13.8 % of its step, profiles/r1_sft_job_kernel_breakdown.md) but does not
    fit for 70B. ``mode`` (default ``GRT_NF4_CACHE``, else "auto"): "1" on, "0" off, "auto" on
    when the cache fits in ``budget_fraction`` of the device's memory. Returns whether it is on."""
    layers = [m for m in model.modules() if isinstance(m, NF4Linear)]
    mode = mode or os.environ.get("GRT_NF4_CACHE", "auto")
    if not layers:
        return False
    dev = layers[0].qweight.device
    if mode == "auto":
        if dev.type != "cuda":
            on = False
        else:
            need = sum(4 * m.in_features * m.out_features for m in layers)
            on = need <= budget_fraction * torch.cuda.get_device_properties(dev).total_memory
    else:
        on = mode not in ("0", "off", "false")
    for m in layers:
        m.set_dequant_cache(on)
    return on
