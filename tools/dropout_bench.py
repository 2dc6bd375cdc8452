#!/usr/bin/env python3
"""Bandwidth of the seeded dropout kernels at the LoRA input shape (6144 x 4096 bf16)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402

C = _native.kernels()
x = torch.randn(6144, 4096, device="cuda", dtype=torch.bfloat16)
dx = torch.zeros_like(x)


def t(fn, it=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


f = t(lambda: C.dropout_fwd_seeded(x, 0.1, 7, 0))
b = t(lambda: C.dropout_bwd_seeded(x, dx, 0.1, 7, 0, True))
nb = x.numel() * 2
print(json.dumps({"fwd_us": round(f, 1), "fwd_TBps": round(2 * nb / f / 1e6, 2),
                  "bwd_accum_us": round(b, 1), "bwd_TBps": round(3 * nb / b / 1e6, 2)}))
