#!/usr/bin/env python3
"""A/B of the LDS-DMA source addressing of the bf16 flash-attention kernels (attention.hip,
AttnParams::dma_fast): 1 = tiles inside the sequence take a uniform tile base + per-lane offsets
fixed for the sweep (one 64-bit add per DMA), 0 = the clamped per-lane row arithmetic on every tile
(two 32-bit multiplies + a 64-bit multiply-add per DMA, quarter-rate VALU).

Per shape both modes must give bit-identical O / lse / dQ / dK / dV (only addresses change); then
forward and backward are timed in interleaved rounds (median). Shapes: the Llama-2-7B headline
(B8 S1024 H32), a GQA shape, and a padding-free pack of odd-length sequences (the clamped tail
tiles) at the reference SFT job's Llama-3.1-8B heads.

``--flag skip_dead`` A/Bs AttnParams::skip_dead instead (attn_set_skip_dead: a wave skips the causal
tiles its rows mask entirely: forward, dQ and wave-pair dK / dV kernels), under the same bitwise-equality gate.
usage: python tools/attn_dma_ab.py [--rounds 7] [--iters 10] [--flag dma_fast|skip_dead]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402

C = _native.kernels()
SET, FLAG = C.attn_set_dma_fast, "dma"


def ev_time(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def run(tag, B, S, Hq, Hkv, lens, rounds, iters):
    D = 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q, do = (torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(2))
    k, v = (torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, generator=g) for _ in range(2))
    scale = D ** -0.5
    kw = {}
    if lens:
        cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), device="cuda", dtype=torch.int32)
        kw = dict(cu_seqlens=cu, max_seqlen=max(lens))
    fwd = lambda: C.attn_fwd(q, k, v, None, scale, True, None, 0.0, 0, **kw)  # noqa: E731
    res, fw, bw = {}, {0: [], 1: []}, {0: [], 1: []}
    for m in (0, 1):
        SET(m)
        o, lse = fwd()
        res[m] = (o, lse) + tuple(C.attn_bwd(do, q, k, v, o, lse, None, None, None, scale, True, None, 0.0, 0, **kw))
    torch.cuda.synchronize()
    same = [torch.equal(a, b) for a, b in zip(res[0], res[1])]
    if lens:  # packed lse is [nseq, H, max_seqlen]: rows past a sequence's length are never written
        same[1] = all(torch.equal(res[0][1][i, :, :n], res[1][1][i, :, :n]) for i, n in enumerate(lens))
    o, lse = res[1][:2]
    for _ in range(rounds):
        for m in (0, 1):
            SET(m)
            fw[m].append(ev_time(fwd, iters))
            bw[m].append(ev_time(lambda: C.attn_bwd(do, q, k, v, o, lse, None, None, None, scale, True, None,
                                                    0.0, 0, **kw), iters))
    SET(1)
    row = {"shape": tag, "bitwise_equal_o_lse_dq_dk_dv": same}
    for m in (0, 1):
        row[f"fwd_us_{FLAG}{m}"] = round(statistics.median(fw[m]), 1)
        row[f"bwd_us_{FLAG}{m}"] = round(statistics.median(bw[m]), 1)
    print(json.dumps(row), flush=True)
    return all(same)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--flag", choices=("dma_fast", "skip_dead"), default="dma_fast")
    a = ap.parse_args()
    SET, FLAG = getattr(C, f"attn_set_{a.flag}"), ("dma" if a.flag == "dma_fast" else "skip")
    ok = run("B8 S1024 Hq32 Hkv32 causal", 8, 1024, 32, 32, None, a.rounds, a.iters)
    ok &= run("B2 S2048 Hq32 Hkv8 causal", 2, 2048, 32, 8, None, a.rounds, a.iters)
    lens = [700, 1023, 517, 1301, 933, 1100, 429]
    ok &= run(f"packed {len(lens)} seqs ({sum(lens)} tokens) Hq32 Hkv8", 1, sum(lens), 32, 8, lens, a.rounds, a.iters)
    sys.exit(0 if ok else 1)
