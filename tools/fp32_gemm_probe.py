#!/usr/bin/env python3
"""What precision and rate do torch's fp32 GEMMs run at on this GPU (BasicLLM's dtype)? Times
torch.mm in fp32 at the BasicLLM FFN shape (4096 tokens x 2048 -> 8192) and at 8192^3, reports TF/s
against the 157.3 TF/s fp32 matrix peak, and the error of a 1024^3 product against fp64: ~1e-7
relative = fp32 inputs and accumulation; ~1e-3 = a reduced-precision (tf32-like) input path."""
import json
import time

import torch


def tflops(m, n, k, reps=20):
    a = torch.randn(m, k, device="cuda")
    b = torch.randn(k, n, device="cuda")
    for _ in range(3):
        a @ b
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        a @ b
    torch.cuda.synchronize()
    return 2.0 * m * n * k * reps / (time.perf_counter() - t0) / 1e12


def main():
    out = {"allow_tf32": torch.backends.cuda.matmul.allow_tf32,
           "float32_matmul_precision": torch.get_float32_matmul_precision()}
    out["ffn_4096x8192x2048_TFs"] = round(tflops(4096, 8192, 2048), 1)
    out["sq_8192_TFs"] = round(tflops(8192, 8192, 8192, 10), 1)
    g = torch.Generator().manual_seed(0)
    a = torch.randn(1024, 1024, generator=g, dtype=torch.float64)
    b = torch.randn(1024, 1024, generator=g, dtype=torch.float64)
    ref = a @ b
    got = (a.float().cuda() @ b.float().cuda()).double().cpu()
    out["rel_err_vs_fp64"] = float((got - ref).norm() / ref.norm())
    cpu32 = (a.float() @ b.float()).double()
    out["cpu_fp32_rel_err_vs_fp64"] = float((cpu32 - ref).norm() / ref.norm())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
