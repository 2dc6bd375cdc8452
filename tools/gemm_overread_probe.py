#!/usr/bin/env python3
"""Validate every GEMM of a TunableOp results table on an MI355X (ops/gemm_tuning.py
check_tuned_table: each row's exact BLAS problem on NaN-poisoned operand padding/tails vs an fp32
reference) and optionally write the table without the failing rows. Tuning itself only times the
candidates, so a solution that reads outside its operands or computes a wrong product can win;
run this after every tuning pass."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.ops.gemm_tuning import RESULTS, check_tuned_table  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--table", default=str(RESULTS))
ap.add_argument("--prune", default="", help="write the table without failing rows here")
ap.add_argument("--out", default="", help="per-row JSON lines")
a = ap.parse_args()
rows = check_tuned_table(a.table)
recs = []
for ln, finite, rel, ok in rows:
    f = ln.split(",")
    recs.append({"op": f[0], "params": f[1], "solution": f[2], "finite": finite, "rel": rel, "ok": ok})
    print(json.dumps(recs[-1]), flush=True)
bad = {ln for ln, _, _, ok in rows if not ok}
print(f"rows {len(rows)}, failing: {len(bad)}", flush=True)
if a.out:
    with open(a.out, "w") as fh:
        fh.writelines(json.dumps(r) + "\n" for r in recs)
if a.prune:
    lines = open(a.table).read().splitlines()
    with open(a.prune, "w") as fh:
        fh.write("\n".join(ln for ln in lines if ln not in bad) + "\n")
    print("pruned table:", a.prune, flush=True)
