"""Forward-projection GEMM layouts on MI355X, hot and cold operands: Y = X W^T (NT, F.linear; what
the model runs) vs Y = X Wt with a pre-transposed weight (NN, the dgrad kernel family). 'cold'
rotates 6 independent operand sets (> the 256 MiB Infinity Cache) like a training step does."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms()
M = 8192
shapes = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}
for name, (K, N) in shapes.items():
    sets = [(torch.randn(M, K, device="cuda", dtype=torch.bfloat16), torch.randn(N, K, device="cuda", dtype=torch.bfloat16))
            for _ in range(6)]
    wts = [w.t().contiguous() for _, w in sets]
    for mode in ("hot", "cold"):
        for lay in ("NT_linear", "NN_pretransposed"):
            def run(i):
                x, w = sets[i % 6] if mode == "cold" else sets[0]
                return F.linear(x, w) if lay == "NT_linear" else x @ (wts[i % 6] if mode == "cold" else wts[0])
            for i in range(6):
                run(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(30):
                run(i)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 30
            print(json.dumps({"shape": name, "mode": mode, "layout": lay, "ms": round(ms, 4),
                              "tflops": round(2 * M * N * K / ms / 1e9, 1)}), flush=True)
