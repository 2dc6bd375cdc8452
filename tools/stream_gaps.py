#!/usr/bin/env python3
"""Idle time of each stream inside whole training steps of a rocprofv3 kernel trace: per stream,
busy time, idle time, and the largest gaps with the kernels on either side (where the compute
stream waits for a side stream's event, or for the host).
usage: tools/stream_gaps.py run_kernel_trace.csv TOTAL_STEPS [--top 15]"""
import csv
import sys
from collections import defaultdict


def main(path, total_steps, top=15):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    per = len(ad) // total_steps
    t0 = int(rows[ad[per - 1]]["End_Timestamp"])
    t1 = int(rows[ad[-1]]["End_Timestamp"])
    nsteps = total_steps - 1
    by = defaultdict(list)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s >= t0 and e <= t1:
            by[r["Stream_Id"]].append((s, e, r["Kernel_Name"][:70]))
    print(f"window {(t1 - t0) / 1e6 / nsteps:.1f} ms/step over {nsteps} steps")
    for sid, ks in sorted(by.items(), key=lambda kv: -len(kv[1])):
        busy = sum(e - s for s, e, _ in ks)
        gaps = [(ks[i + 1][0] - ks[i][1], ks[i][2], ks[i + 1][2]) for i in range(len(ks) - 1)]
        idle = sum(g for g, _, _ in gaps if g > 0)
        print(f"\nstream {sid}: {len(ks) / nsteps:.0f} kernels/step, busy {busy / 1e6 / nsteps:.1f} ms/step, "
              f"idle between its kernels {idle / 1e6 / nsteps:.1f} ms/step")
        agg = defaultdict(lambda: [0, 0])
        for g, a, b in gaps:
            if g > 20_000:  # > 20 us
                k = (a, b)
                agg[k][0] += g
                agg[k][1] += 1
        for (a, b), (g, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
            print(f"  {g / 1e6 / nsteps:6.2f} ms/step  {n / nsteps:5.1f}x/step  after {a}  ->  {b}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), *(int(x) for x in sys.argv[4:5]))
