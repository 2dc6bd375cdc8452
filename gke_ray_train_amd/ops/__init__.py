"""Hot-path ops: gfx950 HIP kernels on GPU tensors, PyTorch references on CPU tensors."""
from .fused import (add_rms_norm, cross_entropy, dropout, flash_attention, gelu, layer_norm,
                    lm_head_cross_entropy, nf4_dequantize, nf4_quantize, rms_norm, rope_attention, swiglu,
                    Varlen)
from .optim import FusedAdamW, GradClipState, clip_grad_norm_, make_optimizer
from ._ref import rope_tables

__all__ = [
    "add_rms_norm", "cross_entropy", "dropout", "flash_attention", "gelu", "layer_norm",
    "lm_head_cross_entropy", "nf4_dequantize", "nf4_quantize", "rms_norm", "rope_attention", "swiglu", "Varlen",
    "FusedAdamW", "GradClipState", "clip_grad_norm_", "make_optimizer", "rope_tables",
]
