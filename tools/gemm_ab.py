#!/usr/bin/env python3
"""Interleaved A/B timing of the wgrad GEMM variants vs hipBLASLt (cdna_hip_programming.md rule 24:
N variants x M rounds in ONE process, median reported; random operands)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402

C = _native.kernels()
T, d, f, V = 8192, 4096, 11008, 32000
SHAPES = {"qkv": (3 * d, d), "o": (d, d), "gate_up": (2 * f, d), "down": (d, f), "lm_head": (V, d)}
modes = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3").split(",")]
rounds, iters = 7, 8


def time_it(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


for name, (N, K) in SHAPES.items():
    dy = torch.randn(T, N, device="cuda").bfloat16()
    x = torch.randn(T, K, device="cuda").bfloat16()
    dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * T * N * K
    variants = {"hipblaslt": lambda: torch.mm(dy.t(), x, out=dw)}
    for m in modes:
        variants[f"grt{m}"] = (lambda m=m: C.gemm_wgrad(dy, x, dw, False, m))
    for fn in variants.values():
        for _ in range(3):
            fn()
    res = {k: [] for k in variants}
    for _ in range(rounds):
        for k, fn in variants.items():
            res[k].append(time_it(fn))
    out = {"shape": name}
    for k, v in res.items():
        out[k] = round(fl / (statistics.median(v) * 1e-3) / 1e12, 1)
    print(json.dumps(out), flush=True)
