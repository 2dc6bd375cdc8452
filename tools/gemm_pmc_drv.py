"""Workload for rocprofv3 PMC passes over the projection GEMM: hipBLASLt (tuned table) and the
hand-written kernel variants on one shape, a few dispatches each (scripts/gpu_gemm_pmc.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402
from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms  # noqa: E402

M, N, K = (int(v) for v in os.environ.get("GEMM_SHAPE", "8192,4096,4096").split(","))
variants = [int(v) for v in os.environ.get("GEMM_VARIANTS", "0,3").split(",")]
enable_tuned_gemms()
C = _native.kernels()
A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(int(os.environ.get("GEMM_REPS", "10"))):
    torch.mm(A, B.t(), out=out)
    for v in variants:
        C.gemm_nt(A, B, out, False, v)
torch.cuda.synchronize()
print("done")
