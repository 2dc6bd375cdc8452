"""dX = dY W via the NN library GEMM (dy @ w, what autograd runs) vs the TN form on a transposed
weight copy (F.linear(dy, w^T contiguous)), burst and steady state, per Llama-2-7B projection."""
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
for name, (K, N) in {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096),
                     "lm_head": (4096, 32000)}.items():
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    wt = w.t().contiguous()
    ref = dy @ w
    assert torch.allclose(F.linear(dy, wt).float(), ref.float(), atol=0.5, rtol=2e-2)
    for kind, fn in (("NN dy@w", lambda: dy @ w), ("TN linear(dy, wT)", lambda: F.linear(dy, wt))):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t_end = time.time() + 0.7
        while time.time() < t_end:
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(40):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 40
        print(json.dumps({"shape": name, "kind": kind, "ms": round(ms, 4), "tflops": round(2 * M * N * K / ms / 1e9)}),
              flush=True)
