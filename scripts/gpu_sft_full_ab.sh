#!/bin/bash
# Full-FT reference SFT job (Llama-2-7B) and bench.py --batch 6 on the shipped vs the merged tuned
# table (gpurun_out/r4ft/tuned.csv from scripts/gpu_sft_full_tune.sh): validate the merged table on
# NaN-poisoned operands (rows that fail are dropped), then interleaved runs.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ftab}; rm -rf $O; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
T=$PWD/${2:-gke_ray_train_amd/tuning/tunableop_mi355x_candidate.csv}
timeout -k 10 300 python3 - "$T" > $O/validate.log 2>&1 <<'PY'
import sys
sys.path.insert(0, ".")
from gke_ray_train_amd.ops.gemm_tuning import check_tuned_table
p = sys.argv[1]
res = check_tuned_table(p)
bad = {r[0] for r in res if not r[3]}
for r in res:
    if not r[3]:
        print("DROP", r)
if bad:
    kept = [ln for ln in open(p).read().splitlines() if ln not in bad]
    open(p, "w").write("\n".join(kept) + "\n")
print(f"rows {len(res)} bad {len(bad)}")
PY
rc=$?; tail -2 $O/validate.log; fatal $rc; [ $rc = 0 ] || exit $rc
cp $T $O/validated.csv
export GRT_STORAGE_PATH=/tmp/grt_ft
FT="python3 tools/sft_inproc.py --set USE_QLORA=false --set MODEL_ID=llama2-7b --set SAVE_STRATEGY=no --set REPORT_TO=none --set NUM_TRAIN_SAMPLES=400 --set LEARNING_RATE=2e-5 --set OUTPUT_DIR_BASE=/tmp/grt_ft/out"
for r in 1 2; do
  timeout -k 10 300 $FT > $O/ab_old_$r.log 2>&1; rc=$?; fatal $rc
  GRT_TUNED_GEMM_FILE=$T timeout -k 10 300 $FT > $O/ab_new_$r.log 2>&1; rc=$?; fatal $rc
  echo "old $r"; grep -h "tokens_per_sec" $O/ab_old_$r.log | tail -3 | cut -c1-150
  echo "new $r"; grep -h "tokens_per_sec" $O/ab_new_$r.log | tail -3 | cut -c1-150
done
timeout -k 10 200 python3 bench.py --batch 6 --steps 20 --warmup 5 > $O/b6_old.log 2>&1; rc=$?; tail -1 $O/b6_old.log | cut -c1-200; fatal $rc
GRT_TUNED_GEMM_FILE=$T timeout -k 10 200 python3 bench.py --batch 6 --steps 20 --warmup 5 > $O/b6_new.log 2>&1; rc=$?; tail -1 $O/b6_new.log | cut -c1-200; fatal $rc
echo done
