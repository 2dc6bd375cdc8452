#!/usr/bin/env python3
"""bf16 flash-attention forward / backward timing (interleaved rounds, median) on random data at
the Llama-2-7B training shape (B8 S1024 H32 D128 causal) and a GQA shape, after a check against
the fp32 math reference (max abs error of O and of dQ / dK / dV). TFLOP/s count the algorithmic
causal FLOPs: 2 matmuls forward, 5 backward. The kernel generations compared in round 2
(profiles/r2_attention.md) were selected through a since-removed variant switch.
usage: python tools/attn_ab.py [--rounds 7]
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
SCHEDS = ""


def ev_time(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us


def run(shape, rounds, iters):
    B, S, Hq, Hkv = shape
    D = 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, generator=g)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, generator=g)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, generator=g)
    do = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16, generator=g)
    scale = D ** -0.5
    flop_mm = 2 * B * Hq * S * S * D / 2  # one causal matmul
    # reference on a slice of heads (fp32 math path)
    hs = slice(0, min(Hq, 4))
    kv_hs = slice(0, max(1, (min(Hq, 4) * Hkv) // Hq))
    qr, kr, vr = (t.float().requires_grad_() for t in (q[:, :, hs], k[:, :, kv_hs], v[:, :, kv_hs]))
    orf = _ref.attention(qr, kr, vr, causal=True, scale=scale)
    orf.backward(do[:, :, hs].float())
    out = {}
    o, lse = C.attn_fwd(q, k, v, None, scale, True, None)
    out["fwd"] = {"max_err": (o[:, :, hs].float() - orf.detach()).abs().max().item(), "t": []}
    dq, dk, dv = C.attn_bwd(do, q, k, v, o, lse, None, None, None, scale, True, None)
    out["bwd"] = {"max_err_dq_dk_dv": [(dq[:, :, hs].float() - qr.grad).abs().max().item(),
                                       (dk[:, :, kv_hs].float() - kr.grad).abs().max().item() if Hq == Hkv else None,
                                       (dv[:, :, kv_hs].float() - vr.grad).abs().max().item() if Hq == Hkv else None],
                  "t": []}
    scheds = [int(x) for x in SCHEDS.split(",")] if SCHEDS else [None]
    if len(scheds) > 1:  # every schedule must give bitwise the same outputs (same per-block math)
        res = []
        for sc in scheds:
            C.attn_set_schedule(sc)
            o_s, lse_s = C.attn_fwd(q, k, v, None, scale, True, None)
            res.append((o_s, lse_s, *C.attn_bwd(do, q, k, v, o_s, lse_s, None, None, None, scale, True, None)))
        for sc, r in zip(scheds[1:], res[1:]):
            same = all(torch.equal(x, y) for x, y in zip(res[0], r))
            print(json.dumps({"shape": f"B{B} S{S} Hq{Hq} Hkv{Hkv}", "sched": sc, "bitwise_equal_to": scheds[0],
                              "equal": same}), flush=True)
    for sc in scheds:
        for name in ("fwd", "bwd"):
            out.setdefault(f"{name}_s{sc}", {"t": []}) if sc is not None else None
    for _ in range(rounds):
        for sc in scheds:
            if sc is not None:
                C.attn_set_schedule(sc)
            kf, kb = ("fwd", "bwd") if sc is None else (f"fwd_s{sc}", f"bwd_s{sc}")
            out[kf]["t"].append(ev_time(lambda: C.attn_fwd(q, k, v, o, scale, True, None), iters))
            out[kb]["t"].append(ev_time(
                lambda: C.attn_bwd(do, q, k, v, o, lse, None, None, None, scale, True, None), iters))
    if scheds[0] is not None:
        del out["fwd"]["t"], out["bwd"]["t"]
        out["fwd"]["t"], out["bwd"]["t"] = [], []
        out = {k: v for k, v in out.items() if v["t"]} | {k: out[k] for k in ("fwd", "bwd")}
    for name, r in out.items():
        if not r.get("t"):
            r.pop("t", None)
            print(json.dumps({"shape": f"B{B} S{S} Hq{Hq} Hkv{Hkv} D128 causal", "kernel": name, **r}), flush=True)
            continue
        t = statistics.median(r.pop("t"))
        nmm = 2 if name.startswith("fwd") else 5
        r.update(us=round(t, 1), tflops=round(nmm * flop_mm / t / 1e6, 1))
        print(json.dumps({"shape": f"B{B} S{S} Hq{Hq} Hkv{Hkv} D128 causal", "kernel": name, **r}), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--scheds", default="", help="comma-separated workgroup schedules to A/B (attn_set_schedule)")
    a = ap.parse_args()
    SCHEDS = a.scheds
    for shape in ((8, 1024, 32, 32), (2, 2048, 32, 8)):
        run(shape, a.rounds, a.iters)
