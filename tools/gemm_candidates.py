#!/usr/bin/env python3
"""Rank ALL TunableOp candidates for the input-gradient (NN) GEMMs by a realistic timing.

TunableOp's own ranking times candidates on hot, tiny loops; the dX GEMMs of a training step run
on operands that have just been written elsewhere and on a power-loaded chip. Step 1 (one process)
runs TunableOp with verbose logging to list every candidate for each shape; step 2 pins each
candidate in a fresh process (a one-line results file) and times it over 3 rotating operand sets
for ~0.5 s; the fastest per shape is written to --out (merged with the existing forward entries).
"""
import argparse
import csv
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096),
          "lm_head": (4096, 32000)}
M = 8192


def list_candidates(tmp):
    env = dict(os.environ, PYTORCH_TUNABLEOP_ENABLED="1", PYTORCH_TUNABLEOP_TUNING="1",
               PYTORCH_TUNABLEOP_VERBOSE="3", PYTORCH_TUNABLEOP_FILENAME=os.path.join(tmp, "all.csv"),
               PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS="3", PYTORCH_TUNABLEOP_MAX_WARMUP_ITERATIONS="1")
    code = ("import torch\n"
            f"for K, N in {list(SHAPES.values())!r}:\n"
            f"    dy = torch.randn({M}, N, device='cuda', dtype=torch.bfloat16)\n"
            "    w = torch.randn(N, K, device='cuda', dtype=torch.bfloat16)\n"
            "    dy @ w\n"
            "    torch.cuda.synchronize()\n")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    cands = {}
    sig = None
    for line in out.splitlines():
        m = re.search(r"(nn_\d+_\d+_\d+_ld_\d+_\d+_\d+)", line)
        if m:
            sig = m.group(1)
        c = re.search(r"(Gemm_(?:Hipblaslt|Rocblas)_\d+|Default)", line)
        if sig and c:
            cands.setdefault(sig, set()).add(c.group(1))
    return cands, out


TIME_CODE = r'''
import sys, torch, json
K, N, path = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
tun = torch.cuda.tunable
tun.enable(True); tun.tuning_enable(False); tun.record_untuned_enable(False)
ok = tun.read_file(path)
sets = [(torch.randn(%d, N, device="cuda", dtype=torch.bfloat16), torch.randn(N, K, device="cuda", dtype=torch.bfloat16)) for _ in range(3)]
for i in range(6): sets[i %% 3][0] @ sets[i %% 3][1]
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
n = 60
for i in range(n): sets[i %% 3][0] @ sets[i %% 3][1]
e1.record(); torch.cuda.synchronize()
print(json.dumps({"ok": bool(ok), "ms": e0.elapsed_time(e1) / n}))
''' % M


def time_candidate(K, N, sig, cand, validators, tmp):
    path = os.path.join(tmp, "pin.csv")
    with open(path, "w") as f:
        for k, v in validators:
            f.write(f"Validator,{k},{v}\n")
        f.write(f"GemmTunableOp_BFloat16_NN,{sig},{cand},0.1\n")
    r = subprocess.run([sys.executable, "-c", TIME_CODE, str(K), str(N), path], capture_output=True, text=True,
                       timeout=300)
    try:
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception:
        return {"ok": False, "err": (r.stdout + r.stderr)[-300:]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tmp", default="gpurun_out/cand")
    ap.add_argument("--max", type=int, default=12, help="candidates timed per shape (TunableOp's fastest first)")
    ap.add_argument("--out", default="gpurun_out/cand/tunableop_nn_ranked.csv")
    a = ap.parse_args()
    os.makedirs(a.tmp, exist_ok=True)
    import torch
    cands, log = list_candidates(a.tmp)
    open(os.path.join(a.tmp, "tuning_log.txt"), "w").write(log)
    validators = [tuple(r[1:3]) for r in csv.reader(open(os.path.join(a.tmp, "all.csv"))) if r and r[0] == "Validator"]
    best = {}
    for name, (K, N) in SHAPES.items():
        sig = f"nn_{K}_{M}_{N}_ld_{K}_{N}_{K}"
        cs = sorted(cands.get(sig, []))
        print(json.dumps({"shape": name, "sig": sig, "n_candidates": len(cs)}), flush=True)
        res = []
        for c in cs[: a.max] if len(cs) <= a.max else cs:
            t = time_candidate(K, N, sig, c, validators, a.tmp)
            if t.get("ok"):
                res.append((t["ms"], c))
                print(json.dumps({"shape": name, "cand": c, "ms": round(t["ms"], 4),
                                  "tflops": round(2 * M * N * K / t["ms"] / 1e9)}), flush=True)
        if res:
            best[sig] = min(res)
            print(json.dumps({"shape": name, "best": best[sig][1], "ms": round(best[sig][0], 4)}), flush=True)
    with open(a.out, "w") as f:
        for k, v in validators:
            f.write(f"Validator,{k},{v}\n")
        for sig, (ms, c) in best.items():
            f.write(f"GemmTunableOp_BFloat16_NN,{sig},{c},{ms}\n")
    print("wrote", a.out, flush=True)


if __name__ == "__main__":
    main()
