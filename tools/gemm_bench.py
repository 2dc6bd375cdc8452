"""A/B microbench: hand-written gfx950 projection GEMM (csrc/kernels/gemm_mfma.hip) vs hipBLASLt
(torch.mm with the offline-tuned solution table) on the Llama-2-7B step shapes.

Both arms run on the same random operands, interleaved in one process (cdna_hip_programming.md
§5.4 rules 24/25). Every shape is first checked against an fp32 reference.

    python tools/gemm_bench.py [--set fwd,dgrad,wgrad] [--rounds 5] [--reps 20] [--out f.jsonl]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gke_ray_train_amd import _native  # noqa: E402
from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms  # noqa: E402

T = 8192  # tokens per step (8 x 1024)
# (name, M, N, K) of C[M, N] = A[M, K] B[N, K]^T
SETS = {
    "fwd": [("qkv", T, 12288, 4096), ("o", T, 4096, 4096), ("gate_up", T, 22016, 4096), ("down", T, 4096, 11008),
            ("lm_head", T, 32000, 4096)],
    # dX = dY (W^T)^T on the optimizer-written W^T
    "dgrad": [("qkv", T, 4096, 12288), ("o", T, 4096, 4096), ("gate_up", T, 4096, 22016), ("down", T, 11008, 4096),
              ("lm_head", T, 4096, 32000)],
    # dW = dY^T X on transposed (reduction-contiguous) operands
    "wgrad": [("qkv", 12288, 4096, T), ("o", 4096, 4096, T), ("gate_up", 22016, 4096, T), ("down", 4096, 11008, T),
              ("lm_head", 32000, 4096, T)],
}


def _time(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def check(C, a, b, out, accumulate=False, variant=0):
    ref = (out.float() if accumulate else 0) + a.float() @ b.float().t()
    ok = C.gemm_nt(a, b, out, accumulate, variant)
    assert ok, "shape not supported"
    torch.cuda.synchronize()
    err = (out.float() - ref).abs()
    rel = float((err.norm() / ref.norm()).item())
    bound = float((ref.abs() * 2 ** -7 + 1e-2).max().item())
    return rel, float(err.max().item()), bound


# weight gradient dW[N, K] = dY[T, N]^T X[T, K] on token-major operands: (name, N, K)
WGRAD_TT = [("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008),
            ("lm_head", 32000, 4096)]


def bench_tt(C, a, rows):
    """token-major weight gradient: production path (two HIP transposes + hipBLASLt TN with the tuned
    table), the round-1 gemm_tt kernel, and the half-tile TT kernel (gemm_wgrad2)."""
    dev = torch.device("cuda", 0)
    for name, N, K in WGRAD_TT:
        dy = torch.randn(T, N, device=dev).to(torch.bfloat16)
        x = torch.randn(T, K, device=dev).to(torch.bfloat16)
        out = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        ref = dy.float().t() @ x.float()
        assert C.gemm_wgrad2(dy, x, out, False)
        torch.cuda.synchronize()
        rel = float(((out.float() - ref).norm() / ref.norm()).item())
        print(f"tt {name:8s} check rel={rel:.2e}", flush=True)
        if not rel < 5e-3:
            raise SystemExit(f"tt {name}: wrong result rel={rel}")
        # accumulate (beta = 1)
        out2 = out.clone()
        assert C.gemm_wgrad2(dy, x, out2, True)
        torch.cuda.synchronize()
        rel2 = float(((out2.float() - 2 * ref).norm() / (2 * ref).norm()).item())
        if not rel2 < 5e-3:
            raise SystemExit(f"tt {name}: wrong accumulate rel={rel2}")
        dyt = torch.empty(N, T, device=dev, dtype=torch.bfloat16)
        xt = torch.empty(K, T, device=dev, dtype=torch.bfloat16)

        def prod():
            C.transpose_into(dy, dyt)
            C.transpose_into(x, xt)
            torch.mm(dyt, xt.t(), out=out)
        arms = {"transpose_tn": prod, "gemm_tt": lambda: C.gemm_wgrad(dy, x, out, False),
                "tt2": lambda: C.gemm_wgrad2(dy, x, out, False)}
        for f in list(arms.values()) * 2:
            f()
        torch.cuda.synchronize()
        ts = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, f in arms.items():
                ts[k].append(_time(f, a.reps))
        fl = 2.0 * T * N * K
        row = {"set": "wgrad_tt", "shape": name, "N": N, "K": K}
        for k, t in ts.items():
            m = statistics.median(t)
            row[f"{k}_us"] = round(m, 1)
            row[f"{k}_tf"] = round(fl / m / 1e6, 1)
        print(json.dumps(row), flush=True)
        rows.append(row)
        del dy, x, out, out2, dyt, xt
        torch.cuda.empty_cache()


def bench_nn(C, a, rows):
    """input gradient dX = dY W on W as stored: hipBLASLt NN, the production TN form on a W^T copy
    (its transpose not timed: the optimizer writes it), and the half-tile NN kernel (gemm_nn)."""
    dev = torch.device("cuda", 0)
    for name, M, N, K in SETS["dgrad"]:  # C[M, N] = A[M, K] B[K, N]; N = K_in, K = N_out
        dy = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(K, N, device=dev).to(torch.bfloat16)
        wt = w.t().contiguous()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = dy.float() @ w.float()
        assert C.gemm_nn(dy, w, out, False)
        torch.cuda.synchronize()
        rel = float(((out.float() - ref).norm() / ref.norm()).item())
        print(f"nn {name:8s} check rel={rel:.2e}", flush=True)
        if not rel < 5e-3:
            raise SystemExit(f"nn {name}: wrong result rel={rel}")
        arms = {"lib_nn": lambda: torch.mm(dy, w, out=out), "lib_tn": lambda: torch.mm(dy, wt.t(), out=out),
                "nn": lambda: C.gemm_nn(dy, w, out, False)}
        for f in list(arms.values()) * 2:
            f()
        torch.cuda.synchronize()
        ts = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, f in arms.items():
                ts[k].append(_time(f, a.reps))
        fl = 2.0 * M * N * K
        row = {"set": "dgrad_nn", "shape": name, "M": M, "N": N, "K": K}
        for k, t in ts.items():
            m = statistics.median(t)
            row[f"{k}_us"] = round(m, 1)
            row[f"{k}_tf"] = round(fl / m / 1e6, 1)
        print(json.dumps(row), flush=True)
        rows.append(row)
        del dy, w, wt, out
        torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="fwd,dgrad,wgrad")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--variants", default="0")
    a = ap.parse_args()
    enable_tuned_gemms()
    C = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    rows = []
    for sname in a.set.split(","):
        if sname == "tt":
            bench_tt(C, a, rows)
            continue
        if sname == "nn":
            bench_nn(C, a, rows)
            continue
        for name, M, N, K in SETS[sname]:
            A = torch.randn(M, K, device=dev).to(torch.bfloat16)
            B = torch.randn(N, K, device=dev).to(torch.bfloat16)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            out2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            variants = [int(v) for v in a.variants.split(",")]
            if not a.no_check:
                for v in variants:
                    rel, mx, bound = check(C, A, B, out, variant=v)
                    print(f"{sname:6s} {name:8s} v{v} check rel={rel:.2e} maxabs={mx:.3g} (bound {bound:.3g})",
                          flush=True)
                    if not (rel < 5e-3):
                        raise SystemExit(f"{sname} {name}: wrong result rel={rel}")
            arms = {"lib": lambda: torch.mm(A, B.t(), out=out2)}
            for v in variants:
                arms[f"v{v}"] = (lambda v=v: C.gemm_nt(A, B, out, False, v))
            for f in list(arms.values()) * 2:
                f()
            torch.cuda.synchronize()
            ts = {k: [] for k in arms}
            for _ in range(a.rounds):
                for k, f in arms.items():
                    ts[k].append(_time(f, a.reps))
            fl = 2.0 * M * N * K
            med = {k: statistics.median(t) for k, t in ts.items()}
            row = {"set": sname, "shape": name, "M": M, "N": N, "K": K}
            for k, t in med.items():
                row[f"{k}_us"] = round(t, 1)
                row[f"{k}_tf"] = round(fl / t / 1e6, 1)
            print(json.dumps(row), flush=True)
            rows.append(row)
            del A, B, out, out2
            torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
