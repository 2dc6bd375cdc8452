#!/usr/bin/env python3
"""Offline-tune the GEMM shapes a run logged as missing from the shipped table.

Step 1 (the run): ``GRT_TUNED_GEMM_RECORD_UNTUNED=gpurun_out/x/untuned.csv <job>`` makes
``enable_tuned_gemms`` log every library GEMM whose (layout, m, n, k, ld) has no table row.
Step 2 (this tool, on an MI355X): tune each logged shape once with TunableOp on top of the base
table (``tune_gemm_in_file``), write the merged table to --out, then validate every row of it on
NaN-poisoned operands against fp32 (``check_tuned_table``) and drop rows that fail. A/B the result
with ``GRT_TUNED_GEMM_FILE=<out>`` before shipping it.
"""
import argparse
import glob
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.ops.gemm_tuning import RESULTS, check_tuned_table  # noqa: E402


def write_results(tun, path):
    with open(path + ".tmp", "w") as fh:
        for k, v in tun.get_validators():
            fh.write(f"Validator,{k},{v}\n")
        for op_sig, param_sig, kernel, ms in tun.get_results():
            fh.write(f"{op_sig},{param_sig},{kernel},{ms}\n")
    os.replace(path + ".tmp", path)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("untuned", help="untuned-shape file(s), glob allowed")
    ap.add_argument("--out", required=True)
    ap.add_argument("--base", default=str(RESULTS))
    ap.add_argument("--duration", type=int, default=30, help="max tuning ms per candidate solution")
    ap.add_argument("--only", default="", help="comma-separated substrings; tune only matching shapes")
    a = ap.parse_args(argv)
    # TunableOp's rotating operand copies are sized from the leading dimensions and overrun
    # column-block views (the round-2 'invalid argument' abort): tune without them
    os.environ.setdefault("PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE", "0")
    lines = set()
    for f in glob.glob(a.untuned):
        for ln in open(f):
            if ln.startswith("Gemm"):
                lines.add(ln.strip())
    known = {tuple(ln.split(",")[:2]) for ln in open(a.base) if ln.startswith("Gemm")}
    todo = sorted(ln for ln in lines if tuple(ln.split(",")[:2]) not in known)
    if a.only:
        keys = a.only.split(",")
        todo = [ln for ln in todo if any(k in ln for k in keys)]
    print(f"{len(lines)} logged shapes, {len(todo)} not in the base table", flush=True)
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.read_file(a.base)
    tun.tuning_enable(True)
    tun.record_untuned_enable(False)
    tun.set_max_tuning_duration(a.duration)
    tun.set_max_tuning_iterations(30)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    tmp = a.out + ".todo"
    for i, ln in enumerate(todo):
        with open(tmp, "w") as fh:
            fh.write(ln + "\n")
        t0 = time.time()
        tun.tune_gemm_in_file(tmp)
        torch.cuda.synchronize()
        print(f"[{i + 1}/{len(todo)}] {ln.split(',')[1]} tuned in {time.time() - t0:.1f} s", flush=True)
        write_results(tun, a.out)  # after every shape: a time-limited run keeps what it tuned
    os.remove(tmp) if os.path.exists(tmp) else None
    tun.tuning_enable(False)
    write_results(tun, a.out)
    res = check_tuned_table(a.out)
    bad = [r for r in res if not r[3]]
    for ln, fin, rel, ok in bad:
        print(f"DROP (finite={fin} rel={rel:.3g}): {ln}", flush=True)
    if bad:
        drop = {r[0] for r in bad}
        kept = [ln for ln in open(a.out).read().splitlines() if ln not in drop]
        with open(a.out, "w") as fh:
            fh.write("\n".join(kept) + "\n")
    print(f"results: {a.out}: rows {len(res)} bad {len(bad)}", flush=True)


if __name__ == "__main__":
    main()
