#!/usr/bin/env python3
"""Summarise scripts/gpu_pmc_zoo.sh output: per kernel, mean duration (kernel trace), MFMA busy share,
wave-state split, LDS bank-conflict cycles, HBM-side bytes and bandwidth.

Derived columns (MI355X: 256 CUs x 4 SIMDs):
* effective clock: GRBM_GUI_ACTIVE is summed over the 8 XCDs, so GRBM_GUI_ACTIVE / 8 / duration is the
  clock the kernel ran at — but only for dispatches of >= 0.3 ms (MI355X_MICROARCH.md 'DVFS give-back':
  the quotient reads high on shorter ones; round 3's zoo showed 3.3-6.2 GHz there). Shorter dispatches
  get the median clock of the run's long dispatches (column `clk src` = "run"), and no clock ever
  exceeds the 2.4 GHz maximum;
* cycles = duration x that clock; mfma % = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles) — share of
  the time the matrix cores are busy at the clock the kernel actually ran;
* wait / issue-stall / active = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES;
* read GB = 2 x FETCH_SIZE KiB (gfx950 FETCH_SIZE counts half of a wide coalesced read,
  MI355X_MICROARCH.md §HBM), write GB = WRITE_SIZE KiB; GB/s over the trace duration.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    n = name.replace("void ", "").replace("grt::(anonymous namespace)::", "")
    m = re.match(r"_ZN3grt12_GLOBAL__N_1\d+(\w+?)I(\w*?)EE", n)
    if m:  # keep the template arguments (Lb0E = false, Lb1E = true, Li2E = 2) to tell variants apart
        args = re.sub(r"L[bi](\d+)E?", r"\1,", m.group(2)).rstrip(",")
        return f"{m.group(1)}<{args}>"
    return re.sub(r"\(.*", "", n)[:60]


def load_counters(path):
    """-> {kernel: {counter: [per-dispatch values]}}"""
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    names = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[k][r["Counter_Name"]][did] += float(r["Counter_Value"])
        names[k] = 1
    out = {}
    for k, cs in per.items():
        out[k] = {c: sum(v.values()) / max(1, len(v)) for c, v in cs.items()}
    return out


def main(d):
    tr = glob.glob(os.path.join(d, "**", "trace_kernel_trace.csv"), recursive=True)
    dur = defaultdict(list)
    if tr:
        for r in csv.DictReader(open(tr[0])):
            dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9)
    else:  # no separate kernel trace: the (serialised) dispatch times of the first counter pass
        seen = set()
        for r in csv.DictReader(open(glob.glob(os.path.join(d, "**", "sq_counter_collection.csv"), recursive=True)[0])):
            if r["Dispatch_Id"] not in seen:
                seen.add(r["Dispatch_Id"])
                dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9)
    ctr = {}
    for tag in ("sq", "fetch", "write"):
        f = glob.glob(os.path.join(d, "**", f"{tag}_counter_collection.csv"), recursive=True)
        if f:
            for k, cs in load_counters(f[0]).items():
                ctr.setdefault(k, {}).update(cs)
    LONG_S, MAX_GHZ = 3e-4, 2.4
    med = {k: sorted(ds)[len(ds) // 2] for k, ds in dur.items()}
    own = {}
    for k, t in med.items():
        gui = ctr.get(k, {}).get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if gui and t >= LONG_S:
            own[k] = min(MAX_GHZ, gui / t / 1e9)
    run_clk = sorted(own.values())[len(own) // 2] if own else 2.1
    rows = []
    for k, ds in dur.items():
        if not any(s in k for s in ("grt", "gemm_tt", "Cijk")):
            continue
        c = ctr.get(k, {})
        t = med[k]
        clk, src = (own[k], "own") if k in own else (run_clk, "run")
        cyc = t * clk * 1e9
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        rd = 2 * c.get("FETCH_SIZE", 0.0) * 1024 / 1e9
        wr = c.get("WRITE_SIZE", 0.0) * 1024 / 1e9
        hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        rows.append((short(k), len(ds), t * 1e6, 100 * mf / (1024 * cyc) if cyc else 0.0, clk, src,
                     100 * c.get("SQ_WAIT_ANY", 0) / wc, 100 * c.get("SQ_WAIT_INST_ANY", 0) / wc,
                     100 * c.get("SQ_ACTIVE_INST_ANY", 0) / wc, c.get("SQ_LDS_BANK_CONFLICT", 0.0),
                     rd, wr, (rd + wr) / t if t else 0.0, 100 * hit / (hit + miss) if hit + miss else 0.0))
    rows.sort(key=lambda r: -r[2])
    print("| kernel | calls | median us | mfma % | clk GHz | clk src | wait % | issue-stall % | active % | "
          "LDS bank-conflict cycles | read GB | write GB | HBM GB/s | L2 hit % |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| `{r[0]}` | {r[1]} | {r[2]:.1f} | {r[3]:.1f} | {r[4]:.2f} | {r[5]} | {r[6]:.0f} | {r[7]:.0f} | "
              f"{r[8]:.0f} | {r[9]:.3g} | {r[10]:.3f} | {r[11]:.3f} | {r[12]:.0f} | {r[13]:.0f} |")
    extra = glob.glob(os.path.join(d, "**", "sq2_counter_collection.csv"), recursive=True)
    if extra:
        cs2 = load_counters(extra[0])
        names = sorted({n for v in cs2.values() for n in v})
        print()
        print("| kernel | " + " | ".join(names) + " |")
        print("|---" * (len(names) + 1) + "|")
        for k, v in sorted(cs2.items(), key=lambda kv: -med.get(kv[0], 0)):
            if any(s in k for s in ("grt", "gemm_tt", "Cijk")):
                print(f"| `{short(k)}` | " + " | ".join(f"{v.get(n, 0):.4g}" for n in names) + " |")


if __name__ == "__main__":
    main(sys.argv[1])
