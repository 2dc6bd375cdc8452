"""List library GEMM / marker kernels of a rocprofv3 kernel trace in launch order (name, grid, us)."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    n = r["Kernel_Name"]
    if "Cijk" in n or "FillFunctor<float>" in n or "gemm_tt" in n:
        print(n[:100], r["Grid_Size_X"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) // 1000)
