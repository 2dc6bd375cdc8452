#!/usr/bin/env python3
"""Weight gradient with ONE transposed operand: tune (TunableOp, on top of the shipped table) and
time the two single-transpose layouts against the shipped path (both operands transposed + TN):
  xt   torch.mm(dY^T view, (X^T)^T)   - only X is transposed (pays off when dY is the big operand)
  dyt  torch.mm(dY^T, X)              - only dY is transposed (pays off when X is the big operand)
Writes the merged table to --out; prints per-shape medians (us) including the transposes paid."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402
from gke_ray_train_amd.ops.gemm_tuning import RESULTS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="gpurun_out/tunableop_single.csv")
ap.add_argument("--duration", type=int, default=40)
a = ap.parse_args()
C = _native.kernels()
tun = torch.cuda.tunable
tun.enable(True)
tun.read_file(str(RESULTS))
tun.set_max_tuning_duration(a.duration)
tun.set_max_tuning_iterations(40)
os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
tun.set_filename(a.out)
T, d, f, V = 8192, 4096, 11008, 32000
SHAPES = {"qkv": (3 * d, d), "o": (d, d), "gate_up": (2 * f, d), "down": (d, f), "lm_head": (V, d)}
cases = {}
for name, (N, K) in SHAPES.items():
    c = dict(dy=torch.randn(T, N, device="cuda").bfloat16(), x=torch.randn(T, K, device="cuda").bfloat16(),
             out=torch.empty(N, K, device="cuda", dtype=torch.bfloat16),
             dyt=torch.empty(N, T, device="cuda", dtype=torch.bfloat16),
             xt=torch.empty(K, T, device="cuda", dtype=torch.bfloat16))
    C.transpose_into(c["dy"], c["dyt"])
    C.transpose_into(c["x"], c["xt"])
    cases[name] = c
tun.tuning_enable(True)
for name, c in cases.items():
    torch.mm(c["dy"].t(), c["xt"].t(), out=c["out"])
    torch.mm(c["dyt"], c["x"], out=c["out"])
    c["out"].addmm_(c["dy"].t(), c["xt"].t())
    c["out"].addmm_(c["dyt"], c["x"])
    torch.cuda.synchronize()
    print("tuned", name, flush=True)
tun.tuning_enable(False)
with open(a.out, "w") as fh:
    for k, v in tun.get_validators():
        fh.write(f"Validator,{k},{v}\n")
    for op_sig, param_sig, kernel, ms in tun.get_results():
        fh.write(f"{op_sig},{param_sig},{kernel},{ms}\n")


def time_it(fn, iters=6):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1000


res = {n: {"tn2": [], "xt": [], "dyt": []} for n in cases}
for _ in range(5):
    for n, c in cases.items():
        res[n]["tn2"].append(time_it(lambda: (C.transpose_into(c["dy"], c["dyt"]), C.transpose_into(c["x"], c["xt"]),
                                              torch.mm(c["dyt"], c["xt"].t(), out=c["out"]))))
        res[n]["xt"].append(time_it(lambda: (C.transpose_into(c["x"], c["xt"]),
                                             torch.mm(c["dy"].t(), c["xt"].t(), out=c["out"]))))
        res[n]["dyt"].append(time_it(lambda: (C.transpose_into(c["dy"], c["dyt"]), torch.mm(c["dyt"], c["x"], out=c["out"]))))
for n in cases:
    print(json.dumps({"shape": n, **{k + "_us": round(statistics.median(v), 1) for k, v in res[n].items()}}), flush=True)
