#!/usr/bin/env python3
"""Every hand-written gfx950 kernel of the hot paths at its production shape, a few launches each,
for rocprofv3 PMC passes (scripts/gpu_pmc_zoo.sh). Shapes: the Llama-2-7B training step (8 x 1024
tokens) and the Llama-3.1-8B decode step."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native, ops  # noqa: E402
from gke_ray_train_amd.ops.linear import wgrad  # noqa: E402

REP = int(os.environ.get("ZOO_REP", "3"))
dev = "cuda"
bf = torch.bfloat16
C = _native.kernels()
T, d, f = 8192, 4096, 11008
torch.manual_seed(0)


def rep(fn):
    for _ in range(REP):
        fn()
    torch.cuda.synchronize()


# weight-gradient GEMM (qkv and down projections)
dy = torch.randn(T, 3 * d, device=dev, dtype=bf)
x = torch.randn(T, d, device=dev, dtype=bf)
rep(lambda: wgrad(dy, x))
dy2 = torch.randn(T, d, device=dev, dtype=bf)
x2 = torch.randn(T, f, device=dev, dtype=bf)
rep(lambda: wgrad(dy2, x2))
del dy, x, dy2, x2

# flash attention fwd + bwd (B 8, S 1024, 32 heads, D 128, causal)
q, k, v = (torch.randn(8, 1024, 32, 128, device=dev, dtype=bf, requires_grad=True) for _ in range(3))
do = torch.randn(8, 1024, 32, 128, device=dev, dtype=bf)


def attn():
    o = ops.flash_attention(q, k, v, causal=True)
    torch.autograd.backward(o, do)


rep(attn)
del q, k, v, do

# RMSNorm (+residual) fwd/bwd, SwiGLU fwd/bwd
h = torch.randn(T, d, device=dev, dtype=bf, requires_grad=True)
r = torch.randn(T, d, device=dev, dtype=bf, requires_grad=True)
w = torch.ones(d, device=dev, dtype=bf, requires_grad=True)


def norm():
    y, res = ops.add_rms_norm(h, r, w)
    torch.autograd.backward([y, res], [torch.ones_like(y), torch.ones_like(res)])


rep(norm)
gu = torch.randn(T, 2 * f, device=dev, dtype=bf, requires_grad=True)


def sw():
    y = ops.swiglu(gu)
    y.backward(torch.ones_like(y))


rep(sw)
del h, r, gu

# fused AdamW over 512 M parameters (bf16 params / grads, fp32 states)
n = 512 * 1024 * 1024
p = torch.randn(n, device=dev, dtype=bf)
g = torch.randn(n, device=dev, dtype=bf)
m = torch.zeros(n, device=dev)
vv = torch.zeros(n, device=dev)
hyper = torch.tensor([1e-4, 0.9, 0.999, 1e-8, 0.0, 0.1, 0.001, 1.0, 0.0, 1.0], device=dev)
rep(lambda: C.adamw(p, g, m, vv, None, hyper, None))
# gradient sum of squares (grad-norm partials) over the same 512 M bf16 elements
ws = torch.zeros(C.sumsq_blocks(), device=dev)
rep(lambda: C.sumsq(g, ws, 0))
del p, g, m, vv

# transposing AdamW on one down-projection weight [4096, 11008] (+ W^T side output)
pw = torch.randn(d, f, device=dev, dtype=bf)
gw = torch.randn(d, f, device=dev, dtype=bf)
mw, vw = torch.zeros(d, f, device=dev), torch.zeros(d, f, device=dev)
wt = torch.empty(f, d, device=dev, dtype=bf)
rep(lambda: C.adamw_t(pw, gw, mw, vw, hyper, None, wt, 0))
del pw, gw, mw, vw, wt

# weight-gradient operand transpose (down-projection input [8192, 11008])
xs = torch.randn(T, f, device=dev, dtype=bf)
xt = torch.empty(f, T, device=dev, dtype=bf)
rep(lambda: C.transpose_into(xs, xt))
del xs, xt

# LoRA adapter kernels at the Llama-2-7B fused-qkv shape (r 64 x 3 targets, dropout 0.1)
xl = torch.randn(T, d, device=dev, dtype=bf)
al = torch.randn(192, d, device=dev, dtype=bf) * 0.02
rep(lambda: C.lora_down(xl, al, 0.1, 1234, 0, True))
gl = torch.randn(T, 192, device=dev, dtype=bf)
dxl = torch.randn(T, d, device=dev, dtype=bf)
alt = al.t().contiguous()
rep(lambda: C.lora_dx(gl, alt, dxl, 0.1, 1234, 0, True))
# adapter-gradient kernels (lora_grad.hip): g = s dY B (q target: dY column block of the fused qkv
# gradient), dB = dY^T h', dA = g^T x_d (transposed out)
dyl = torch.randn(T, 3 * d, device=dev, dtype=bf)
btl = torch.randn(192, 3 * d, device=dev, dtype=bf) * 0.02
gq = gl[:, :64]
rep(lambda: C.lora_g(dyl[:, :d], btl[:64, :d], gq, 0.25, False))
dbl = torch.empty(d, 64, device=dev, dtype=bf)
rep(lambda: C.lora_tred(dyl[:, :d], gl[:, :64], dbl, 1.0, False, False))
dal = torch.empty(192, d, device=dev, dtype=bf)
rep(lambda: C.lora_tred(xl, gl, dal, 1.0, False, True))
del xl, al, gl, dxl, alt, dyl, btl, dbl, dal

# decode: GEMV (gate_up of Llama-3.1-8B, 1 token) and split-K decode attention (4K context)
xw = torch.randn(1, 4096, device=dev, dtype=bf)
W = torch.randn(2 * 14336, 4096, device=dev, dtype=bf)
rep(lambda: C.gemv(xw, W))
del W
qd = torch.randn(1, 1, 32, 128, device=dev, dtype=bf)
kc = torch.randn(1, 4096, 8, 128, device=dev, dtype=bf)
vc = torch.randn(1, 4096, 8, 128, device=dev, dtype=bf)
sl = torch.full((1,), 4096, device=dev, dtype=torch.int32)
rep(lambda: C.attn_decode(qd, kc, vc, sl, 128 ** -0.5))

# NF4 dequant (Llama-3.1-8B gate_up weight) and its transposed variant
wq = torch.randn(2 * 14336, 4096, device=dev, dtype=bf)
qw, am = ops.nf4_quantize(wq.view(-1))
rep(lambda: ops.nf4_dequantize(qw, am, wq.numel()))
rep(lambda: C.nf4_dequantize_t(qw, am, 2 * 14336, 4096, 64))
print("zoo done", flush=True)
