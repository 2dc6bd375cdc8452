"""Steady-state (power-limited) GEMM throughput: each projection GEMM run back to back for ~2 s, the
last second timed, vs a short 30-call burst. Shows how far a sustained load drops below burst
numbers on MI355X (the training step is a sustained GEMM load)."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms()
M = 8192
shapes = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}
for name, (K, N) in shapes.items():
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    for kind, fn in (("fwd", lambda: F.linear(x, w)), ("dgrad", lambda: dy @ w)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            fn()
        e1.record()
        torch.cuda.synchronize()
        burst = e0.elapsed_time(e1) / 30
        t_end = time.time() + 1.0
        while time.time() < t_end:  # heat up: ~1 s of continuous load
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
        n = 0
        e0.record()
        t_end = time.time() + 1.0
        while time.time() < t_end:
            for _ in range(20):
                fn()
            n += 20
            torch.cuda.synchronize()
        e1.record()
        torch.cuda.synchronize()
        steady = e0.elapsed_time(e1) / n
        fl = 2 * M * N * K
        print(json.dumps({"shape": name, "kind": kind, "burst_tflops": round(fl / burst / 1e9), "steady_tflops": round(fl / steady / 1e9)}), flush=True)
