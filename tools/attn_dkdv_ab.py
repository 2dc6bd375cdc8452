#!/usr/bin/env python3
"""A/B of the two dK / dV kernel forms of the bf16 flash-attention backward (attention.hip):
1 = the 4-wave kernel (K, V, dK^T, dV^T of 32 keys in one wave, one wave per SIMD), 2 = the
wave-pair kernel (the same 32 keys split over an S-wave and a dP-wave on one SIMD).

Per shape: both forms' dQ / dK / dV are compared with each other (bitwise) and with the fp32 math
reference on a head slice; then the whole backward (pre + dK/dV + dQ) is timed, interleaved rounds,
median. TFLOP/s count the 5 algorithmic causal matmuls of the backward.
usage: python tools/attn_dkdv_ab.py [--rounds 7] [--iters 10]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402
from gke_ray_train_amd.ops import _ref  # noqa: E402

C = _native.kernels()


def ev_time(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us


def run(shape, rounds, iters, dropout):
    B, S, Hq, Hkv = shape
    D = 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q, do = (torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(2))
    k, v = (torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(2))
    scale = D ** -0.5
    o, lse = C.attn_fwd(q, k, v, None, scale, True, None, dropout, 7)
    res = {}
    for f in (1, 2):
        C.attn_set_dkdv_form(f)
        res[f] = C.attn_bwd(do, q, k, v, o, lse, None, None, None, scale, True, None, dropout, 7)
    torch.cuda.synchronize()
    tag = f"B{B} S{S} Hq{Hq} Hkv{Hkv} D128 causal p{dropout}"
    same = [torch.equal(a, b) for a, b in zip(res[1], res[2])]
    maxd = [float((a.float() - b.float()).abs().max()) for a, b in zip(res[1], res[2])]
    row = {"shape": tag, "bitwise_equal_dq_dk_dv": same, "max_abs_diff": maxd}
    if dropout == 0.0:
        hs = slice(0, min(Hq, 4))
        kv_hs = slice(0, max(1, (min(Hq, 4) * Hkv) // Hq))
        qr, kr, vr = (t.float().requires_grad_() for t in (q[:, :, hs], k[:, :, kv_hs], v[:, :, kv_hs]))
        _ref.attention(qr, kr, vr, causal=True, scale=scale).backward(do[:, :, hs].float())
        dq, dk, dv = res[2]
        row["form2_max_err_vs_fp32"] = [float((dq[:, :, hs].float() - qr.grad).abs().max()),
                                        float((dk[:, :, kv_hs].float() - kr.grad).abs().max()) if Hq == Hkv else None,
                                        float((dv[:, :, kv_hs].float() - vr.grad).abs().max()) if Hq == Hkv else None]
    ts = {1: [], 2: []}
    for _ in range(rounds):
        for f in (1, 2):
            C.attn_set_dkdv_form(f)
            ts[f].append(ev_time(lambda: C.attn_bwd(do, q, k, v, o, lse, None, None, None, scale, True, None,
                                                    dropout, 7), iters))
    flop = 5 * 2 * B * Hq * S * S * D / 2
    for f in (1, 2):
        t = statistics.median(ts[f])
        row[f"bwd_form{f}_us"] = round(t, 1)
        row[f"bwd_form{f}_tflops"] = round(flop / t / 1e6, 1)
    C.attn_set_dkdv_form(2)
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    for shape, p in (((8, 1024, 32, 32), 0.0), ((2, 2048, 32, 8), 0.0), ((4, 1024, 32, 8), 0.0),
                     ((2, 1024, 32, 32), 0.1)):
        run(shape, a.rounds, a.iters, p)
