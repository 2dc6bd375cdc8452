#!/usr/bin/env python3
"""Host-link timeline of an offloaded-optimizer run from a rocprofv3 `--kernel-trace
--memory-copy-trace` directory: for each full step (update start to next update start, the update
start being the first AdamW kernel after a gap) the wall time, GPU kernel busy time, and per copy
direction the bytes, busy time (union of copy intervals), achieved GB/s while busy, and how much
of it falls in the forward window (update start .. first attention-backward kernel) vs the
backward window.

    python tools/offload_timeline.py gpurun_out/r5offtrace/prof
"""
import csv
import glob
import os
import sys


def _rows(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    if not fs:
        return []
    return list(csv.DictReader(open(fs[0])))


def _union(iv):
    iv = sorted(iv)
    out, cs, ce = [], None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                out.append((cs, ce))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        out.append((cs, ce))
    return out


def _busy(iv, lo, hi):
    return sum(max(0, min(e, hi) - max(s, lo)) for s, e in _union(iv))


def main(d):
    ks = _rows(d, "*kernel_trace.csv")
    cs = _rows(d, "*memory_copy_trace.csv")
    if not ks:
        print("no kernel trace under", d)
        return 1
    kiv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in ks]
    kiv.sort()
    # update starts: an adamw kernel more than 200 ms after the previous adamw kernel
    starts, last = [], None
    for s, e, n in kiv:
        if "adamw" in n:
            if last is None or s - last > 200e6:
                starts.append(s)
            last = e
    bwd = [s for s, e, n in kiv if "attn_bwd" in n]
    copies = {}
    for r in cs:
        dirn = r.get("Direction") or r.get("Kind") or "?"
        size = int(r.get("Bytes") or r.get("Size") or 0)
        copies.setdefault(dirn, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), size))
    print(f"copy directions: {sorted(copies)}; steps found: {max(0, len(starts) - 1)}; "
          f"copy trace columns: {list(cs[0].keys()) if cs else []}\n")
    blits = [(s, e) for s, e, n in kiv if "copyBuffer" in n]
    print("| step | wall ms | kernel busy ms | blit-copy kernel busy ms | fwd window ms | " +
          " | ".join(f"{k} GB / busy ms / GB/s / in fwd window ms" for k in sorted(copies)) + " |")
    print("|---|---|---|---|---|" + "---|" * len(copies))
    for i in range(len(starts) - 1):
        lo, hi = starts[i], starts[i + 1]
        b0 = next((s for s in bwd if s > lo), hi)
        kb = _busy([(s, e) for s, e, _ in kiv], lo, hi)
        cells = []
        for k in sorted(copies):
            iv = [(s, e) for s, e, _ in copies[k] if s < hi and e > lo]
            by = sum(z for s, e, z in copies[k] if lo <= s < hi)
            busy = _busy(iv, lo, hi)
            fw = _busy(iv, lo, b0)
            cells.append(f"{by / 1e9:.1f} / {busy / 1e6:.0f} / {by / max(busy, 1):.1f} / {fw / 1e6:.0f}")
        bb = _busy(blits, lo, hi)
        print(f"| {i} | {(hi - lo) / 1e6:.0f} | {kb / 1e6:.0f} | {bb / 1e6:.0f} | {(b0 - lo) / 1e6:.0f} | "
              + " | ".join(cells) + " |")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
