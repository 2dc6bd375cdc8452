"""Isolated timing of the grad-norm partial-sum kernel (ops sumsq) on a bucket-sized bf16 buffer.
Run once per setting of GRT_SUMSQ_UNROLL (read once per process): scripts/r6/sumsq.sh."""
import argparse
import json
import os

import torch

from gke_ray_train_amd import _native


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=384)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    K = _native.kernels()
    x = torch.randn(a.mb * (1 << 20) // 2, device="cuda", dtype=torch.bfloat16)
    ws = torch.zeros(K.sumsq_blocks(), device="cuda", dtype=torch.float32)
    for _ in range(5):
        K.sumsq(x, ws, 0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        K.sumsq(x, ws, 0)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    print(json.dumps({"unroll": os.environ.get("GRT_SUMSQ_UNROLL", "1"), "mb": a.mb, "us": round(us, 1),
                      "TB_s": round(x.numel() * 2 / us / 1e6, 2)}))


if __name__ == "__main__":
    main()
