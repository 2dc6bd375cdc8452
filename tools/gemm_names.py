"""Which library kernels the projection GEMMs dispatch to (run under rocprofv3 --kernel-trace)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms  # noqa: E402

print("tuned:", enable_tuned_gemms(), flush=True)
M = 8192
for name, (K, N) in {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}.items():
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, requires_grad=False)
    for _ in range(3):
        F.linear(x, w)
    x3 = x.view(8, 1024, K)
    for _ in range(3):
        F.linear(x3, w)
    torch.cuda.synchronize()
    print("done", name, flush=True)
