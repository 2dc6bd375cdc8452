#!/usr/bin/env python3
"""Per-step kernel breakdown from a rocprofv3 ``--kernel-trace`` CSV: only kernels that start after
the end of the first optimizer kernel (``adamw``), i.e. whole training steps with model init and
the first (warm-up) step excluded. Groups kernels into families and prints a markdown table."""
import csv
import re
import sys
from collections import defaultdict

FAMILIES = [
    ("gemm wgrad (grt MFMA)", r"gemm_tt_kernel"),
    ("gemm hipBLASLt", r"^Cijk_|^Custom_Cijk"),
    ("attention fwd", r"attn_fwd"),
    ("attention bwd", r"attn_bwd"),
    ("adamw", r"adamw"),
    ("rmsnorm/layernorm", r"norm_(fwd|bwd)|colsum"),
    ("swiglu", r"swiglu"),
    ("rope", r"rope"),
    ("cross-entropy", r"ce_(fwd|bwd)"),
    ("grad norm", r"sumsq|clip"),
    ("embedding", r"embedding|compute_grad_weight|sum_and_scatter|gather"),
    ("lora", r"lora"),
    ("nf4 dequant", r"nf4"),
    ("transpose", r"transpose"),
    ("rccl", r"ncclDevKernel|rccl|nccl"),
    ("copies/fills", r"copyBuffer|fillBuffer|FillFunctor|copy_kernel"),
]


def main(path, total_steps, top=25):
    """total_steps = warm-up + timed steps of the profiled run (the optimizer launches one AdamW
    kernel per parameter group, or one per module chunk when overlapped)."""
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    per = len(ad) // total_steps
    if total_steps < 2 or per < 1 or len(ad) % total_steps:
        sys.exit(f"{len(ad)} optimizer kernels do not split into {total_steps} steps")
    t_begin = int(rows[ad[per - 1]]["End_Timestamp"])
    t_end = int(rows[ad[-1]]["End_Timestamp"])
    steps = total_steps - 1
    fam = defaultdict(float)
    perk = defaultdict(lambda: [0.0, 0])
    busy = 0.0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t_begin or s > t_end:
            continue
        d = (e - s) / 1e6
        busy += d
        n = r["Kernel_Name"]
        perk[n][0] += d
        perk[n][1] += 1
        for f, pat in FAMILIES:
            if re.search(pat, n):
                fam[f] += d
                break
        else:
            fam["other"] += d
    wall = (t_end - t_begin) / 1e6
    print(f"steps: {steps}; wall {wall / steps:.1f} ms/step; summed kernel time {busy / steps:.1f} ms/step\n")
    print("| family | ms/step | % of kernel time |\n|---|---|---|")
    for f, v in sorted(fam.items(), key=lambda x: -x[1]):
        print(f"| {f} | {v / steps:.2f} | {100 * v / busy:.1f} |")
    print("\n| ms/step | calls/step | avg us | kernel |\n|---|---|---|---|")
    for n, (t, c) in sorted(perk.items(), key=lambda x: -x[1][0])[:top]:
        print(f"| {t / steps:.2f} | {c / steps:.0f} | {1000 * t / c:.1f} | `{n[:110]}` |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
