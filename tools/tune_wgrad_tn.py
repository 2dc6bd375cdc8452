#!/usr/bin/env python3
"""TunableOp-tune the TN weight-gradient GEMMs (dW = dY^T X as torch.mm(dY^T, (X^T)^T), ops/linear.py
wgrad) of the Llama-2-7B step on top of the shipped table and write the merged table to --out.
Run on an MI355X, then gate it (tools/gemm_overread_probe.py --table OUT --prune OUT) and A/B it
(GRT_TUNED_GEMM_FILE=OUT) before adopting."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.ops.gemm_tuning import RESULTS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="gpurun_out/tunableop_tn.csv")
ap.add_argument("--tokens", type=int, default=8192)
ap.add_argument("--duration", type=int, default=40, help="max tuning ms per shape")
a = ap.parse_args()

tun = torch.cuda.tunable
tun.enable(True)
tun.read_file(str(RESULTS))
tun.tuning_enable(True)
tun.set_max_tuning_duration(a.duration)
tun.set_max_tuning_iterations(40)
os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
tun.set_filename(a.out)
T, d, f, V = a.tokens, 4096, 11008, 32000
for name, (N, K) in {"qkv": (3 * d, d), "o": (d, d), "gate_up": (2 * f, d), "down": (d, f), "lm_head": (V, d)}.items():
    dyt = torch.randn(N, T, device="cuda", dtype=torch.bfloat16)
    xt = torch.randn(K, T, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    torch.mm(dyt, xt.t(), out=out)
    out.addmm_(dyt, xt.t())  # the accumulating form (gradient accumulation) too
    torch.cuda.synchronize()
    print(f"tuned wgrad TN {name}: N={N} K={K}", flush=True)
tun.tuning_enable(False)
with open(a.out, "w") as fh:
    for k, v in tun.get_validators():
        fh.write(f"Validator,{k},{v}\n")
    for op_sig, param_sig, kernel, ms in tun.get_results():
        fh.write(f"{op_sig},{param_sig},{kernel},{ms}\n")
print("results:", a.out, sum(1 for _ in open(a.out)), "lines", flush=True)
