#!/usr/bin/env python3
"""Isolated AdamW kernels at the Llama-2-7B projection shapes: the transposing update (adamw_t:
param, moments, W^T) and the flat update (adamw), stochastic rounding on / off. Median of --reps
launches; GB/s counts the bytes each kernel must move (adamw_t: 24 B / param, adamw: 22 B).
usage: python tools/adamw_bench.py [--reps 20]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008)}


def med(fn, reps):
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
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    C = _native.kernels()
    dev = torch.device("cuda")
    for name, (r, c) in SHAPES.items():
        p = torch.randn(r, c, device=dev).bfloat16()
        g = torch.randn(r, c, device=dev).bfloat16() * 1e-3
        m = torch.zeros(r, c, device=dev)
        v = torch.zeros(r, c, device=dev)
        pt = torch.empty(c, r, device=dev, dtype=torch.bfloat16)
        row = {"param": name, "shape": [r, c]}
        for sr in (0.0, 1.0):
            hyper = torch.tensor([1e-5, 0.9, 0.999, 1e-8, 0.0, 0.1, 0.001, 1.0, sr, 3.0], device=dev)
            us = med(lambda: C.adamw_t(p, g, m, v, hyper, None, pt, 0), a.reps)
            row[f"adamw_t_sr{int(sr)}_us"] = round(us, 1)
            row[f"adamw_t_sr{int(sr)}_TBps"] = round(24 * p.numel() / us / 1e6, 2)
            us = med(lambda: C.adamw(p.view(-1), g.view(-1), m.view(-1), v.view(-1), None, hyper, None, 0, 0), a.reps)
            row[f"adamw_sr{int(sr)}_us"] = round(us, 1)
            row[f"adamw_sr{int(sr)}_TBps"] = round(22 * p.numel() / us / 1e6, 2)
            # flat update + a separate transpose pass for W^T (26 B / param in two streaming passes)
            def flat_t():
                C.adamw(p.view(-1), g.view(-1), m.view(-1), v.view(-1), None, hyper, None, 0, 0)
                C.transpose_into(p, pt)
            us = med(flat_t, a.reps)
            row[f"flat+transpose_sr{int(sr)}_us"] = round(us, 1)
            us = med(lambda: C.transpose_into(p, pt), a.reps)
            row["transpose_us"] = round(us, 1)
            row["transpose_TBps"] = round(4 * p.numel() / us / 1e6, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
