#!/usr/bin/env python3
"""Tune the projection GEMMs of a model at a set of token counts M with TunableOp and keep only
the winners that beat the library default in THIS script's own back-to-back timing.

Used for the SFT path, whose fused batches keep M on multiples of 1024 (trainer/sft.py
``fuse_pad_multiple``): forward ``x[M,K] @ W[N,K]^T`` and the transposed-weight input gradient
``dy[M,N] @ Wt[K,N]^T`` (both TN). TunableOp's own pick is sometimes slower than the default in
practice (profiles/r1_gemm_bucket_probe.jsonl), hence the validation. Appends the kept entries to
``--out`` (default: the package's tuning file), preserving the existing ones.

    python tools/tune_gemm_buckets.py --model llama3.1-8b --ms 1024,2048,...,8192
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.models import get_config  # noqa: E402
from gke_ray_train_amd.ops.gemm_tuning import RESULTS  # noqa: E402


def timeit(fn, iters=25):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--ms", default=",".join(str(1024 * k) for k in range(1, 9)))
    ap.add_argument("--out", default=str(RESULTS))
    ap.add_argument("--keep-below", type=float, default=0.97, help="keep a winner if tuned/default < this")
    ap.add_argument("--log", default="")
    a = ap.parse_args()
    cfg = get_config(a.model)
    d, f, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
    hd = d // cfg.num_attention_heads
    qkv = (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * hd
    shapes = []
    for (K, N) in [(d, qkv), (d, d), (d, 2 * f), (f, d), (d, V)]:
        shapes.append(("fwd", K, N))
        shapes.append(("dx", N, K))
    Ms = [int(x) for x in a.ms.split(",")]
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    if os.path.exists(a.out):
        tun.read_file(a.out)
    existing = {(o, p) for o, p, _, _ in tun.get_results()}
    kept = []
    log = open(a.log, "a") if a.log else None
    t_start = time.time()
    for kind, K, N in shapes:
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        xa = torch.randn(max(Ms), K, device="cuda", dtype=torch.bfloat16)
        for M in Ms:
            x = xa[:M]
            key_hint = f"_{M}_{K}_"
            if any(p.startswith(f"tn_{N}_") and key_hint in p for _, p in existing):
                continue
            tun.enable(False)
            base = timeit(lambda: torch.nn.functional.linear(x, w))
            tun.enable(True)
            tun.tuning_enable(True)
            tun.set_max_tuning_duration(20)
            tun.set_max_tuning_iterations(25)
            torch.nn.functional.linear(x, w)
            torch.cuda.synchronize()
            tun.tuning_enable(False)
            res = [r for r in tun.get_results() if r[1].startswith(f"tn_{N}_{M}_{K}_")]
            tuned = timeit(lambda: torch.nn.functional.linear(x, w))
            rec = {"kind": kind, "M": M, "N": N, "K": K, "default_ms": round(base, 4), "tuned_ms": round(tuned, 4),
                   "kernel": res[0][2] if res else None, "kept": bool(res) and tuned < a.keep_below * base,
                   "elapsed_s": round(time.time() - t_start, 1)}
            if rec["kept"]:
                kept.append(res[0])
            print(json.dumps(rec), flush=True)
            if log:
                log.write(json.dumps(rec) + "\n")
                log.flush()
        del w, xa
        torch.cuda.empty_cache()
    # rewrite the file: validators + previous entries + kept new entries
    prev = []
    if os.path.exists(a.out):
        prev = [ln.rstrip("\n") for ln in open(a.out) if ln.strip() and not ln.startswith("Validator")]
    with open(a.out, "w") as fh:
        for k, v in tun.get_validators():
            fh.write(f"Validator,{k},{v}\n")
        for ln in prev:
            fh.write(ln + "\n")
        for op_sig, param_sig, kernel, ms in kept:
            fh.write(f"{op_sig},{param_sig},{kernel},{ms}\n")
    print(f"kept {len(kept)} new entries -> {a.out}", flush=True)


if __name__ == "__main__":
    main()
