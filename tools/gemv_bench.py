#!/usr/bin/env python3
"""Decode-step projections of Llama-3.1-8B at batch 1 on the GEMV kernel (csrc/kernels/gemv.hip):
median time per call and the weight-stream bandwidth (N x K x 2 bytes / time), next to a pure
streaming read of the same bytes (grt sumsq) as the practical roofline; for the projections that
read a norm's output, the on-the-fly normalisation against the add_rms_norm kernel + GEMV, and for
the projections that produce the residual stream, the residual-add + rstd epilogue. One JSON line
per shape.

    python tools/gemv_bench.py [--m 1] [--reps 50] [--flush]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native, ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096, False), "o": (4096, 4096, False), "gate_up": (28672, 4096, False),
          "down_swiglu": (4096, 14336, True), "lm_head": (128256, 4096, False)}
NORM_INPUT = ("qkv", "gate_up", "lm_head")  # the projections that consume a norm's output
NORM_PRODUCER = ("o", "down_swiglu")         # ... and the ones whose output is the next residual


FLUSH = None  # --flush: a 1 GiB read between timed calls evicts the weights from L2 / the MALL


def med(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        if FLUSH is not None:
            FLUSH.sum()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--flush", action="store_true",
                    help="evict the weights between calls (the decode step reads 16 GB between two uses)")
    a = ap.parse_args()
    global FLUSH
    if a.flush:
        FLUSH = torch.ones(2 ** 28, device="cuda")
    C = _native.kernels()
    dev = torch.device("cuda")
    ws = torch.zeros(C.sumsq_blocks(), device=dev)
    tot_us = extra_fused = extra_sep = 0.0
    for name, (N, K, swi) in SHAPES.items():
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        x = torch.randn(a.m, 2 * K if swi else K, device=dev, dtype=torch.bfloat16)
        if swi and a.m > 4:  # the SwiGLU-folding GEMV takes 1-4 rows: time the plain MFMA path
            xk = x[:, :K].contiguous()
            us = med(lambda: C.gemv(xk, w), a.reps)
        else:
            us = med(lambda: C.gemv(x, w, swi), a.reps)
        xl = torch.randn(a.m, K, device=dev, dtype=torch.bfloat16)
        lib = med(lambda: torch.nn.functional.linear(xl, w), a.reps)  # hipBLASLt on the same weights
        ref = med(lambda: C.sumsq(w.view(-1), ws, 0), a.reps)
        nb = N * K * 2
        tot_us += us * (32 if name != "lm_head" else 1)
        print(json.dumps({"shape": name, "N": N, "K": K, "m": a.m, "gemv_us": round(us, 1), "library_us": round(lib, 1),
                          "gemv_TBps": round(nb / us / 1e6, 2), "stream_read_us": round(ref, 1),
                          "stream_read_TBps": round(nb / ref / 1e6, 2)}), flush=True)
        if name in NORM_INPUT and a.m <= 4:  # consumer of a norm: the input normalised on the fly (rstd, g)
            acc = torch.zeros(2, a.m, 64, dtype=torch.int64, device=dev)
            acc[:, :, 0] = K << 20
            g = torch.ones(K, device=dev, dtype=torch.bfloat16)
            r = torch.randn_like(x)
            fused = med(lambda: C.gemv_fused(x, w, acc, 0, g=g), a.reps)
            sep = med(lambda: C.gemv(ops.add_rms_norm(x, r, g, 1e-5)[0], w), a.reps)
            extra_fused += (fused - us) * (32 if name != "lm_head" else 1)
            extra_sep += (sep - us) * (32 if name != "lm_head" else 1)
            print(json.dumps({"shape": name + "+norm", "fused_us": round(fused, 1),
                              "add_rms_norm_kernel_then_gemv_us": round(sep, 1)}), flush=True)
        if name in NORM_PRODUCER and a.m <= 4:  # producer: + residual add and the next norm's rstd in the epilogue
            r = torch.randn(a.m, N, device=dev, dtype=torch.bfloat16)
            acc = torch.zeros(2, a.m, 64, dtype=torch.int64, device=dev)
            fused = med(lambda: C.gemv_fused(x, w, acc, 0, swiglu=swi, res=r), a.reps)
            extra_fused += (fused - us) * 32
            print(json.dumps({"shape": name + "+residual+rstd", "fused_us": round(fused, 1)}), flush=True)
        del w, x
    print(json.dumps({"projections_per_token_ms": round(tot_us / 1e3, 3),
                      "norms_fused_extra_ms": round(extra_fused / 1e3, 3),
                      "norms_separate_extra_ms": round(extra_sep / 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
