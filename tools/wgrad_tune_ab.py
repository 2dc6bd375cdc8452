#!/usr/bin/env python3
"""Weight-gradient GEMM dW = dY^T X (Llama-2-7B shapes, 8192 tokens): TunableOp-tuned hipBLASLt
(the NT layout torch.mm(dy.t(), x) issues) vs the hand-written kernel (csrc/kernels/gemm.hip),
interleaved rounds in one process, median TFLOP/s. Tuning results go to --out (not the shipped
table) so the A/B decides what, if anything, is adopted."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="gpurun_out/wgrad_tunableop.csv")
ap.add_argument("--rounds", type=int, default=7)
a = ap.parse_args()

C = _native.kernels()
T, d, f, V = 8192, 4096, 11008, 32000
SHAPES = {"qkv": (3 * d, d), "o": (d, d), "gate_up": (2 * f, d), "down": (d, f), "lm_head": (V, d)}
ops = {}
for name, (N, K) in SHAPES.items():
    dy = torch.randn(T, N, device="cuda").bfloat16()
    x = torch.randn(T, K, device="cuda").bfloat16()
    ops[name] = (dy, x, torch.empty(N, K, device="cuda", dtype=torch.bfloat16), 2.0 * T * N * K)

# default heuristic timing first (tuning off), then tune
def time_it(fn, iters=8):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters

tun = torch.cuda.tunable
tun.enable(True)
tun.tuning_enable(True)
tun.set_max_tuning_duration(30)
tun.set_max_tuning_iterations(40)
os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
tun.set_filename(a.out)
for name, (dy, x, dw, _) in ops.items():
    torch.mm(dy.t(), x, out=dw)
    torch.cuda.synchronize()
    print(f"tuned {name}", flush=True)
tun.tuning_enable(False)
with open(a.out, "w") as fh:
    for k, v in tun.get_validators():
        fh.write(f"Validator,{k},{v}\n")
    for op_sig, param_sig, kernel, ms in tun.get_results():
        fh.write(f"{op_sig},{param_sig},{kernel},{ms}\n")

for name, (dy, x, dw, fl) in ops.items():
    variants = {"hipblaslt_tuned": lambda: torch.mm(dy.t(), x, out=dw),
                "grt": lambda: C.gemm_wgrad(dy, x, dw, False, 0)}
    for fn in variants.values():
        for _ in range(3):
            fn()
    res = {k: [] for k in variants}
    for _ in range(a.rounds):
        for k, fn in variants.items():
            res[k].append(time_it(fn))
    out = {"shape": name}
    for k, v in res.items():
        out[k] = round(fl / (statistics.median(v) * 1e-3) / 1e12, 1)
    print(json.dumps(out), flush=True)
