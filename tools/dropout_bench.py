#!/usr/bin/env python3
"""Bandwidth of the seeded dropout kernels at the LoRA input shape (6144 x 4096 bf16).

Cold-cache measurement: each launch works on the next of NBUF (x, dx) pairs whose total
(~1.2 GB) is several times the 256 MB Infinity Cache, so successive launches cannot hit in it
and the figure is an HBM bandwidth, not a cache bandwidth. ``--hot`` reuses one pair (the
round-1 figure, which the cache inflates)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--hot", action="store_true")
a = ap.parse_args()
C = _native.kernels()
NBUF = 1 if a.hot else 12
xs = [torch.randn(6144, 4096, device="cuda", dtype=torch.bfloat16) for _ in range(NBUF)]
dxs = [torch.zeros_like(xs[0]) for _ in range(NBUF)]


def t(fn, it=48):
    for i in range(NBUF):
        fn(i)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(it):
        fn(i % NBUF)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


f = t(lambda i: C.dropout_fwd_seeded(xs[i], 0.1, 7, 0))
b = t(lambda i: C.dropout_bwd_seeded(xs[i], dxs[i], 0.1, 7, 0, True))
nb = xs[0].numel() * 2
print(json.dumps({"cache": "hot" if a.hot else f"cold ({NBUF} rotating pairs, {2 * NBUF * nb / 2**30:.2f} GiB)",
                  "fwd_us": round(f, 1), "fwd_TBps": round(2 * nb / f / 1e6, 2),
                  "bwd_accum_us": round(b, 1), "bwd_TBps": round(3 * nb / b / 1e6, 2)}))
