#!/usr/bin/env python3
"""Tune the forward / dX GEMMs of a Llama training step with torch TunableOp and store the winners
in gke_ray_train_amd/tuning/tunableop_mi355x.csv (run once on an MI355X; see ops/gemm_tuning.py)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.ops.gemm_tuning import RESULTS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tokens", type=int, default=8192)
ap.add_argument("--models", default="llama2-7b")
ap.add_argument("--out", default=str(RESULTS))
ap.add_argument("--rotating-mb", type=int, default=0,
                help="rotate operands over this many MB while timing candidates (>256 MB defeats the "
                     "Infinity Cache: in-step conditions, where activations and weights arrive cold)")
ap.add_argument("--iters", type=int, default=40)
a = ap.parse_args()

from gke_ray_train_amd.models import get_config  # noqa: E402

tun = torch.cuda.tunable
tun.enable(True)
tun.tuning_enable(True)
tun.set_max_tuning_duration(30)
tun.set_max_tuning_iterations(a.iters)
if a.rotating_mb:
    tun.set_rotating_buffer_size(a.rotating_mb)
os.makedirs(os.path.dirname(a.out), exist_ok=True)
tun.set_filename(a.out)
T = a.tokens
for name in a.models.split(","):
    cfg = get_config(name)
    d, f, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
    hd = d // cfg.num_attention_heads
    qkv = (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * hd
    for (K, N) in [(d, qkv), (d, d), (d, 2 * f), (f, d), (d, V)]:
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        torch.nn.functional.linear(x, w)     # forward
        dy @ w                               # input gradient
        torch.cuda.synchronize()
        print(f"tuned {name}: K={K} N={N}", flush=True)
# write the CSV ourselves (TunableOp's own writer only runs at process exit)
with open(a.out, "w") as f:
    for k, v in tun.get_validators():
        f.write(f"Validator,{k},{v}\n")
    for op_sig, param_sig, kernel, ms in tun.get_results():
        f.write(f"{op_sig},{param_sig},{kernel},{ms}\n")
tun.tuning_enable(False)
print("results:", a.out, sum(1 for _ in open(a.out)), "lines", flush=True)
