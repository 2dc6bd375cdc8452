#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --stats run: python tools/prof_top.py <kernel_stats.csv> <steps> [N] [filter]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
flt = sys.argv[4] if len(sys.argv) > 4 else ""
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6 / steps:.2f} ms/step over {steps:g} steps")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if flt and flt not in r["Name"]:
        continue
    n -= 1
    if n < 0:
        break
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.2f} ms/step {int(r['Calls']) / steps:6.1f}/step "
          f"{float(r['AverageNs']) / 1e3:8.1f} us avg  {r['Name'][:100]}")
