#!/usr/bin/env python3
"""Micro-benchmarks of the hot ops on one MI355X: GEMM shapes of a Llama-2-7B step (hipBLASLt),
flash attention fwd/bwd (HIP), RMSNorm/SwiGLU/CE/AdamW (HIP). Prints one JSON line per op.

Timing: CUDA events around N back-to-back launches after warmup, random data (guide rule 25).
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def gemms(T=8192, d=4096, f=11008, V=32000):
    out = []
    dev = "cuda"
    try:
        from gke_ray_train_amd import _native
        C = _native.kernels()
    except Exception:
        C = None
    shapes = {
        "qkv_fwd": (T, d, 3 * d), "o_fwd": (T, d, d), "gate_up_fwd": (T, d, 2 * f), "down_fwd": (T, f, d),
        "lm_head_fwd": (T, d, V),
    }
    for name, (M, K, N) in shapes.items():
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        dw = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        t = timeit(lambda: torch.nn.functional.linear(x, w))
        out.append(dict(op=f"gemm_{name}", ms=t * 1e3, tflops=fl / t / 1e12))
        t = timeit(lambda: dy @ w)
        out.append(dict(op=f"gemm_{name.replace('fwd', 'dgrad')}", ms=t * 1e3, tflops=fl / t / 1e12))
        t = timeit(lambda: torch.mm(dy.t(), x, out=dw))
        out.append(dict(op=f"gemm_{name.replace('fwd', 'wgrad')}", ms=t * 1e3, tflops=fl / t / 1e12))
        if C is not None and C.gemm_wgrad(dy, x, dw, False):
            ref = dw.float()
            torch.mm(dy.t(), x, out=dw)
            err = (ref - dw.float()).abs().max().item() / dw.float().abs().max().item()
            t = timeit(lambda: C.gemm_wgrad(dy, x, dw, False))
            out.append(dict(op=f"gemm_{name.replace('fwd', 'wgrad')}_grt", ms=t * 1e3, tflops=fl / t / 1e12,
                            rel_err=err))
            if os.environ.get("GRT_GEMM_DIAG"):
                for mode in (1, 2, 3, 4, 5, 6):
                    t = timeit(lambda: C.gemm_wgrad(dy, x, dw, False, mode))
                    out.append(dict(op=f"gemm_{name.replace('fwd', 'wgrad')}_grt_mode{mode}", ms=t * 1e3,
                                    tflops=fl / t / 1e12))
    return out


def attention(B=8, S=1024, H=32, Hkv=32, D=128):
    from gke_ray_train_amd import _native
    C = _native.kernels()
    dev = "cuda"
    q = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16)
    k = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16)
    sc = 1 / math.sqrt(D)
    o, lse = C.attn_fwd(q, k, v, None, sc, True, None)
    do = torch.randn_like(o)
    fl = 4.0 * B * H * S * S * D / 2
    t = timeit(lambda: C.attn_fwd(q, k, v, o, sc, True, None))
    t2 = timeit(lambda: C.attn_bwd(do, q, k, v, o, lse, None, None, None, sc, True, None))
    return [dict(op="attn_fwd", ms=t * 1e3, tflops=fl / t / 1e12, shape=[B, S, H, Hkv, D]),
            dict(op="attn_bwd", ms=t2 * 1e3, tflops=2.5 * fl / t2 / 1e12, shape=[B, S, H, Hkv, D])]


def memops(T=8192, d=4096, f=11008):
    from gke_ray_train_amd import _native
    C = _native.kernels()
    dev = "cuda"
    out = []
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    r = torch.randn_like(x)
    w = torch.ones(d, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: C.rmsnorm_fwd(x, r, w, 1e-5))
    out.append(dict(op="add_rmsnorm_fwd", ms=t * 1e3, gbs=4 * x.numel() * 2 / t / 1e9))
    y, h, rstd = C.rmsnorm_fwd(x, r, w, 1e-5)
    t = timeit(lambda: C.rmsnorm_bwd(y, h, w, rstd, r))
    out.append(dict(op="rmsnorm_bwd", ms=t * 1e3, gbs=4 * x.numel() * 2 / t / 1e9))
    gu = torch.randn(T, 2 * f, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: C.swiglu_fwd(gu))
    out.append(dict(op="swiglu_fwd", ms=t * 1e3, gbs=3 * T * f * 2 / t / 1e9))
    do = torch.randn(T, f, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: C.swiglu_bwd(gu, do))
    out.append(dict(op="swiglu_bwd", ms=t * 1e3, gbs=5 * T * f * 2 / t / 1e9))
    n = 1 << 28
    p = torch.randn(n, device=dev, dtype=torch.bfloat16)
    g = torch.randn(n, device=dev, dtype=torch.bfloat16)
    m = torch.zeros(n, device=dev)
    vv = torch.zeros(n, device=dev)
    hyper = torch.tensor([1e-4, 0.9, 0.999, 1e-8, 0.0, 0.1, 0.001, 1.0, 0.0, 1.0], device=dev)
    t = timeit(lambda: C.adamw(p, g, m, vv, None, hyper, None), iters=10)
    out.append(dict(op="adamw_bf16", ms=t * 1e3, gbs=n * 22 / t / 1e9))
    logits = torch.randn(T, 32000, device=dev, dtype=torch.bfloat16)
    lab = torch.randint(0, 32000, (T,), device=dev)
    t = timeit(lambda: C.ce_fwd(logits, lab, -100))
    out.append(dict(op="ce_fwd", ms=t * 1e3, gbs=logits.numel() * 2 / t / 1e9))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="all")
    a = ap.parse_args()
    res = []
    if a.what in ("all", "gemm"):
        res += gemms()
    if a.what in ("all", "attn"):
        res += attention()
        res += attention(B=2, S=4096)
        res += attention(B=8, S=1024, H=32, Hkv=8)
    if a.what in ("all", "mem"):
        res += memops()
    if a.what == "normbwd":  # A/B of the rmsnorm backward grid (env is read once per process)
        res += [r for r in memops() if r["op"] == "rmsnorm_bwd"]
    for r in res:
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}))
