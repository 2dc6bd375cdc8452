#!/usr/bin/env python3
"""Memory-bound kernels of the Llama-2-7B training step at their production shapes (8 x 1024 tokens,
d 4096, F 11008): median time of --reps launches (CUDA events) and the HBM bandwidth each reaches,
counted as the bytes the kernel MUST move (every input read once, every output written once).
One JSON line per kernel; `--md` prints a markdown table as well (profiles/r5_membw.md).

    python tools/membw_bench.py [--reps 30] [--md]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402

T, D, F = 8192, 4096, 11008
BF = torch.bfloat16


def med(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--md", action="store_true")
    a = ap.parse_args()
    C = _native.kernels()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    rows = []

    def run(name, fn, nbytes, calls_per_step):
        us = med(fn, a.reps)
        r = {"kernel": name, "us": round(us, 1), "MB": round(nbytes / 1e6, 1),
             "TBps": round(nbytes / us / 1e6, 2), "calls_per_step": calls_per_step,
             "ms_per_step": round(us * calls_per_step / 1e3, 2)}
        print(json.dumps(r), flush=True)
        rows.append(r)

    e = 2  # bf16 bytes
    x = torch.randn(T, D, device=dev, dtype=BF)
    res = torch.randn(T, D, device=dev, dtype=BF)
    w = torch.ones(D, device=dev, dtype=BF)
    run("rmsnorm_fwd (+residual)", lambda: C.rmsnorm_fwd(x, res, w, 1e-5, 0), 4 * T * D * e + 4 * T, 64)
    y, h, rstd = C.rmsnorm_fwd(x, res, w, 1e-5, 0)
    dy = torch.randn(T, D, device=dev, dtype=BF)
    dres = torch.randn(T, D, device=dev, dtype=BF)
    dw = torch.zeros(D, device=dev, dtype=BF)
    run("rmsnorm_bwd (+dres, dw slot)", lambda: C.rmsnorm_bwd(dy, h, w, rstd, dres, dw, True),
        4 * T * D * e + 4 * T, 64)
    run("rmsnorm_bwd_dx (frozen w)", lambda: C.rmsnorm_bwd_dx(dy, h, w, rstd, dres), 4 * T * D * e + 4 * T, 0)
    del y, h, dy, dres
    gu = torch.randn(T, 2 * F, device=dev, dtype=BF)
    dout = torch.randn(T, F, device=dev, dtype=BF)
    run("swiglu_fwd_t (h, h^T)", lambda: C.swiglu_fwd_t(gu, 0), T * 2 * F * e + 2 * T * F * e, 32)
    run("swiglu_bwd_t (dgu, dgu^T)", lambda: C.swiglu_bwd_t(gu, dout), T * 2 * F * e + T * F * e + 2 * T * 2 * F * e, 32)
    del gu, dout
    for name, (r, c) in {"[T, d]": (T, D), "[T, 3d]": (T, 3 * D), "[T, F]": (T, F)}.items():
        src = torch.randn(r, c, device=dev, dtype=BF)
        dst = torch.empty(c, r, device=dev, dtype=BF)
        run(f"transpose {name}", lambda: C.transpose_into(src, dst), 2 * r * c * e, 0)
        del src, dst
    nb = C.sumsq_blocks()
    ws = torch.zeros(nb, device=dev)
    g = torch.randn(128 << 20, device=dev, dtype=BF)  # one 256 MiB gradient bucket
    run("sumsq (256 MiB bucket)", lambda: C.sumsq(g, ws, 0), g.numel() * e, 35)
    del g
    if a.md:
        print("\n| kernel | us | MB moved | TB/s | calls/step | ms/step |\n|---|---|---|---|---|---|")
        for r in rows:
            print(f"| {r['kernel']} | {r['us']} | {r['MB']} | {r['TBps']} | {r['calls_per_step']} | {r['ms_per_step']} |")


if __name__ == "__main__":
    main()
