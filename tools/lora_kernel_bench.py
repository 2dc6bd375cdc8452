#!/usr/bin/env python3
"""LoRA adapter kernels at the reference SFT job's shapes (Llama-3.1-8B, r = 64 on q/k/v/o/gate/up/down,
one packed step of T tokens): per module the grouped g = s dY B products (lora_g_group), the grouped
dB = dY^T h' token reductions (lora_tred_group), dA^T = x_d^T g (lora_tred, transposed) and the
dropout + down-projection h' = s drop(x) A^T (lora_down). Median of --reps launches per shape, with
the bytes of the big operand over time. Launch-time switches (GRT_LORA_G_NS, GRT_LORA_TRED_WPC, ...)
are read once per process: A/B them with separate runs.

    python tools/lora_kernel_bench.py [--tokens 6144] [--reps 20] [--tag name]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402

H, I, KV, R = 4096, 14336, 1024, 64
# module -> (input width, [target widths])
MODULES = {"qkv": (H, [H, KV, KV]), "o": (H, [H]), "gate_up": (H, [I, I]), "down": (I, [H])}


def timeit(fn, reps):
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
    ap.add_argument("--tokens", type=int, default=6144)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    C = _native.kernels()
    T = a.tokens
    dev = torch.device("cuda")
    torch.manual_seed(0)
    total = {}
    for name, (kin, ns) in MODULES.items():
        N = sum(ns)
        k = len(ns)
        dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        bt = torch.randn(R * k, N, device=dev, dtype=torch.bfloat16) * 0.05
        g = torch.empty(T, R * k, device=dev, dtype=torch.bfloat16)
        hc = torch.randn(T, R * k, device=dev, dtype=torch.bfloat16)
        x = torch.randn(T, kin, device=dev, dtype=torch.bfloat16)
        acat = torch.randn(R * k, kin, device=dev, dtype=torch.bfloat16) * 0.05
        offs = [sum(ns[:j]) for j in range(k)]
        dys = [dy[:, o:o + n] for o, n in zip(offs, ns)]
        bts = [bt[j * R:(j + 1) * R, o:o + n] for j, (o, n) in enumerate(zip(offs, ns))]
        gs = [g[:, j * R:(j + 1) * R] for j in range(k)]
        hs = [hc[:, j * R:(j + 1) * R] for j in range(k)]
        dbs = [torch.empty(n, R, device=dev, dtype=torch.bfloat16) for n in ns]
        dat = torch.empty(R * k, kin, device=dev, dtype=torch.bfloat16)
        xw = torch.empty(T, kin + R * k, device=dev, dtype=torch.bfloat16)
        xw[:, :kin] = x
        arms = {
            "lora_g": (lambda: C.lora_g_group(dys, bts, gs, 0.25, False), dy.numel() * 2),
            "tred_dB": (lambda: C.lora_tred_group(dys, hs, dbs, 1.0, [False] * k) if k > 1
                        else C.lora_tred(dys[0], hs[0], dbs[0], 1.0, False, False), dy.numel() * 2),
            "tred_dA": (lambda: C.lora_tred(x, g, dat, 1.0, False, True), x.numel() * 2),
            "lora_down": (lambda: C.lora_down(xw[:, :kin], acat, 0.1, 7, 0, True, h_out=xw[:, kin:], hscale=0.25),
                          x.numel() * 2 * 2),
        }
        for an, (fn, nbytes) in arms.items():
            fn()
            torch.cuda.synchronize()
            us = timeit(fn, a.reps)
            total[an] = total.get(an, 0.0) + us
            print(json.dumps({"tag": a.tag, "module": name, "kernel": an, "T": T, "us": round(us, 1),
                              "GBps": round(nbytes / us / 1e3, 1)}), flush=True)
    print(json.dumps({"tag": a.tag, "per_layer_us": {k: round(v, 1) for k, v in total.items()},
                      "per_layer_total_us": round(sum(total.values()), 1)}), flush=True)


if __name__ == "__main__":
    main()
