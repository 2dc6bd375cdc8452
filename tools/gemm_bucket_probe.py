#!/usr/bin/env python3
"""Probe: does a TunableOp solution tuned at one token count M stay valid and fast at nearby M?

For each Llama projection GEMM (forward TN and transposed-weight dX TN), time the library default
at several M, tune at the bucket M0, then replay the winning solution at the other M through a
TunableOp results file written by this script (tuning off) and time again. Prints one JSON line
per (shape, M)."""
import json
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.models import get_config  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "llama3.1-8b"
    M0 = int(sys.argv[2]) if len(sys.argv) > 2 else 6144
    others = [M0 - 256, M0 - 64, M0 - 8, M0 + 8 * 13, M0 // 2]
    cfg = get_config(model)
    d, f, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
    hd = d // cfg.num_attention_heads
    qkv = (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * hd
    tun = torch.cuda.tunable
    shapes = []
    for (K, N) in [(d, qkv), (d, d), (d, 2 * f), (f, d), (d, V)]:
        shapes.append(("fwd", K, N))   # x [M,K] @ W[N,K]^T
        shapes.append(("dx", N, K))    # dy [M,N] @ Wt[K,N]^T
    Mmax = max([M0] + others)
    for kind, K, N in shapes:
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        xa = torch.randn(Mmax, K, device="cuda", dtype=torch.bfloat16)
        flops = lambda M: 2.0 * M * N * K
        tun.enable(False)
        base = {M: timeit(lambda: torch.nn.functional.linear(xa[:M], w)) for M in [M0] + others}
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(30)
        tun.set_max_tuning_iterations(30)
        torch.nn.functional.linear(xa[:M0], w)
        torch.cuda.synchronize()
        tun.tuning_enable(False)
        res = [r for r in tun.get_results() if f"_{M0}_{K}_" in r[1] and r[1].startswith(f"tn_{N}_")]
        if not res:
            print(json.dumps({"kind": kind, "K": K, "N": N, "error": "no tuned entry"}), flush=True)
            continue
        op_sig, param_sig, kernel, ms = res[0]
        tuned0 = timeit(lambda: torch.nn.functional.linear(xa[:M0], w))
        lines = [f"Validator,{k},{v}" for k, v in tun.get_validators()]
        for M in others:
            ps = param_sig.replace(f"_{M0}_{K}_", f"_{M}_{K}_", 1)
            lines.append(f"{op_sig},{ps},{kernel},{ms}")
        fd, path = tempfile.mkstemp(suffix=".csv")
        with os.fdopen(fd, "w") as fh:
            fh.write("\n".join(lines) + "\n")
        ok = tun.read_file(path)
        out = {"kind": kind, "K": K, "N": N, "M0": M0, "kernel": kernel, "read_ok": bool(ok),
               "default_ms": {M: round(t, 4) for M, t in base.items()},
               "tuned_ms": {M0: round(tuned0, 4)}, "errors": {}}
        for M in others:
            try:
                y = torch.nn.functional.linear(xa[:M], w)
                ref = torch.nn.functional.linear(xa[:M].float(), w.float())
                err = float((y.float() - ref).abs().max() / ref.abs().max())
                out["tuned_ms"][M] = round(timeit(lambda: torch.nn.functional.linear(xa[:M], w)), 4)
                if err > 2e-2:
                    out["errors"][M] = f"rel err {err:.3g}"
            except Exception as e:  # noqa: BLE001
                out["errors"][M] = str(e)[:200]
        out["pflops_default_M0"] = round(flops(M0) / base[M0] / 1e12, 3)
        out["pflops_tuned_M0"] = round(flops(M0) / tuned0 / 1e12, 3)
        print(json.dumps(out), flush=True)
        os.unlink(path)
        del w, xa
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
