#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy table of one .hip file (hipcc -Rpass-analysis remarks).

usage: python tools/kernel_resources.py gke_ray_train_amd/csrc/kernels/attention.hip [-DFOO=1 ...]
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
src = sys.argv[1]
extra = sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast",
       "-munsafe-fp-atomics", "-I", str(ROOT / "gke_ray_train_amd/csrc/include"), *extra, "-c", src,
       "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True).stdout
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(.*?): (.*) \[-Rpass", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
print(f"{'kernel':70s} {'VGPR':>5} {'AGPR':>5} {'spill':>5} {'LDS':>6} {'occ':>4}")
for r in rows:
    if "Occupancy [waves/SIMD]" not in r:
        continue
    name = subprocess.run(["c++filt", r["name"]], stdout=subprocess.PIPE, text=True).stdout.strip()
    name = re.sub(r"grt::\(anonymous namespace\)::", "", name)[:70]
    print(f"{name:70s} {r.get('VGPRs', '?'):>5} {r.get('AGPRs', '?'):>5} {r.get('VGPRs Spill', '?'):>5} "
          f"{r.get('LDS Size [bytes/block]', '?'):>6} {r.get('Occupancy [waves/SIMD]', '?'):>4}")
