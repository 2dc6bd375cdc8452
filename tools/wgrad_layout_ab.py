"""dW = dY^T X: the hand-written MFMA kernel on the M-major operands (gemm.hip, what training runs)
vs hipBLASLt TN on transposed copies (F.linear(dY^T, X^T), K = tokens) incl. the two transposes."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402
from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms  # noqa: E402
from gke_ray_train_amd.ops.linear import wgrad  # noqa: E402

enable_tuned_gemms()
C = _native.kernels()
M = 8192


def bench(fn, n=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t_end = time.time() + 0.5
    while time.time() < t_end:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for name, (K, N) in {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096),
                     "lm_head": (4096, 32000)}.items():
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    xt = torch.empty(K, M, device="cuda", dtype=torch.bfloat16)
    dyt = torch.empty(N, M, device="cuda", dtype=torch.bfloat16)
    C.transpose_into(x, xt)
    C.transpose_into(dy, dyt)
    ref = wgrad(dy, x)
    alt = F.linear(dyt, xt)
    rel = float((ref.float() - alt.float()).norm() / ref.float().norm())
    t_k = bench(lambda: wgrad(dy, x, out, False))
    t_tn = bench(lambda: torch.mm(dyt, xt.t(), out=out))
    t_tr = bench(lambda: (C.transpose_into(x, xt), C.transpose_into(dy, dyt)))
    fl = 2 * M * N * K
    print(json.dumps({"shape": name, "rel_err": round(rel, 5), "grt_kernel_ms": round(t_k, 4),
                      "grt_tflops": round(fl / t_k / 1e9), "tn_ms": round(t_tn, 4), "tn_tflops": round(fl / t_tn / 1e9),
                      "transposes_ms": round(t_tr, 4), "tn_plus_transposes_ms": round(t_tn + t_tr, 4)}), flush=True)
