#!/usr/bin/env python3
"""Weight gradient dW = dY^T X on the Llama-2-7B shapes (8192 tokens), three ways, interleaved rounds
in one process, median us:
  grt      the hand-written MFMA kernel on the token-major operands (csrc/kernels/gemm.hip)
  tn       hipBLASLt on explicitly transposed operands (F.linear(dY^T, X^T): the forward-like layout)
  tn+tr    the same including the two HIP transposes that would produce dY^T and X^T
Decides whether transposing the operands beats the hard layout (tools/, not shipped)."""
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402
from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms()
C = _native.kernels()
T, d, f, V = 8192, 4096, 11008, 32000
SHAPES = {"qkv": (3 * d, d), "o": (d, d), "gate_up": (2 * f, d), "down": (d, f), "lm_head": (V, d)}
cases = {}
for name, (N, K) in SHAPES.items():
    dy = torch.randn(T, N, device="cuda").bfloat16()
    x = torch.randn(T, K, device="cuda").bfloat16()
    cases[name] = dict(dy=dy, x=x, out=torch.empty(N, K, device="cuda", dtype=torch.bfloat16),
                       dyt=torch.empty(N, T, device="cuda", dtype=torch.bfloat16),
                       xt=torch.empty(K, T, device="cuda", dtype=torch.bfloat16), flops=2.0 * T * N * K)


def time_it(fn, iters=6):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1000


res = {n: {"grt": [], "tn": [], "tn+tr": [], "tr": [], "dyT_only": [], "xT_only": []} for n in cases}
for rnd in range(5):
    for n, c in cases.items():
        res[n]["grt"].append(time_it(lambda: C.gemm_wgrad(c["dy"], c["x"], c["out"], False)))
        C.transpose_into(c["dy"], c["dyt"])
        C.transpose_into(c["x"], c["xt"])
        res[n]["tn"].append(time_it(lambda: torch.mm(c["dyt"], c["xt"].t(), out=c["out"])))
        res[n]["tr"].append(time_it(lambda: (C.transpose_into(c["dy"], c["dyt"]), C.transpose_into(c["x"], c["xt"]))))
        res[n]["dyT_only"].append(time_it(lambda: torch.mm(c["dyt"], c["x"], out=c["out"])))
        res[n]["xT_only"].append(time_it(lambda: torch.mm(c["dy"].t(), c["xt"].t(), out=c["out"])))
        res[n]["tn+tr"].append(time_it(lambda: (C.transpose_into(c["dy"], c["dyt"]), C.transpose_into(c["x"], c["xt"]),
                                                torch.mm(c["dyt"], c["xt"].t(), out=c["out"]))))
# numerics: both layouts give the same product
for n, c in cases.items():
    C.gemm_wgrad(c["dy"], c["x"], c["out"], False)
    a = c["out"].float().clone()
    C.transpose_into(c["dy"], c["dyt"])
    C.transpose_into(c["x"], c["xt"])
    torch.mm(c["dyt"], c["xt"].t(), out=c["out"])
    rel = ((a - c["out"].float()).norm() / a.norm()).item()
    med = {k: statistics.median(v) for k, v in res[n].items()}
    print(json.dumps({"shape": n, **{k + "_us": round(v, 1) for k, v in med.items()},
                      "grt_tf": round(c["flops"] / med["grt"] / 1e6, 0), "tn_tf": round(c["flops"] / med["tn"] / 1e6, 0),
                      "rel_diff": rel}), flush=True)
