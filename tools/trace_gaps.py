#!/usr/bin/env python3
"""Idle-gap analysis of a rocprofv3 kernel trace (``run_kernel_trace.csv``).

Splits the trace into steps at a marker kernel (default: the AdamW update), then reports per step
the wall span, summed kernel time, the device-idle time (union of kernel intervals subtracted from
the span) and the largest idle gaps with the kernels on either side — where the host, a
synchronisation or a copy leaves the GPU waiting.

usage: trace_gaps.py run_kernel_trace.csv [--marker adamw] [--skip 2] [--top 12]
"""
import argparse
import csv
from collections import Counter


def short(name: str) -> str:
    n = name.split("(")[0]
    return n[-90:]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="adamw")
    ap.add_argument("--skip", type=int, default=2, help="steps to skip at the start")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args(argv)
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    steps = list(zip(marks, marks[1:]))[a.skip:]
    if not steps:
        print("no steps found")
        return
    gaps = Counter()
    gap_t = Counter()
    tot_span = tot_busy = 0
    for i0, i1 in steps:
        seg = rows[i0 + 1:i1 + 1]
        span = seg[-1][1] - rows[i0][1]
        busy = 0
        cur_s, cur_e = None, None
        prev_name = short(rows[i0][2])
        for s, e, n in seg:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    g = s - cur_e
                    key = (prev_name, short(n))
                    gaps[key] += 1
                    gap_t[key] += g
                else:
                    g = s - rows[i0][1]
                    if g > 0:
                        key = (prev_name, short(n))
                        gaps[key] += 1
                        gap_t[key] += g
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            prev_name = short(n)
        busy += cur_e - cur_s
        tot_span += span
        tot_busy += busy
    n = len(steps)
    print(f"steps {n}: wall {tot_span / n / 1e6:.2f} ms/step, device busy {tot_busy / n / 1e6:.2f} ms/step, "
          f"idle {(tot_span - tot_busy) / n / 1e6:.2f} ms/step")
    print(f"\n| idle ms/step | gaps/step | before | after |\n|---|---|---|---|")
    for key, t in gap_t.most_common(a.top):
        print(f"| {t / n / 1e6:.3f} | {gaps[key] / n:.1f} | `{key[0]}` | `{key[1]}` |")


if __name__ == "__main__":
    main()
