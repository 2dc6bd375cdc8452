#!/bin/bash
# SFT-job GEMM coverage: (1) run the SFT worker loop logging every library GEMM the shipped table
# misses, (2) tune those shapes offline and validate the merged table on poisoned operands,
# (3) A/B the worker loop on the shipped vs the merged table (same box, interleaved).
# SFT_ENV="K=V ..." is passed to every worker-loop run (e.g. GRT_SFT_PADDING_FREE=1).
set -o pipefail
O=gpurun_out/${1:-sfttune}
mkdir -p $O
export GRT_STORAGE_PATH=/tmp/grt_sftt
SFT="env ${SFT_ENV:-GRT_X=0} python3 tools/sft_inproc.py --set NUM_TRAIN_SAMPLES=320 --set EVAL_STEPS_SFT=20 --set SAVE_STEPS_SFT=1000 --set OUTPUT_DIR_BASE=/tmp/grt_sftt/out"
GRT_TUNED_GEMM_RECORD_UNTUNED=$PWD/$O/untuned.csv timeout -k 10 300 $SFT > $O/record.log 2>&1 || exit $?
ls $O
timeout -k 10 ${TUNE_S:-900} python3 tools/tune_untuned.py "$O/untuned*.csv" --out $O/tuned.csv --only "${TUNE_ONLY:-}" > $O/tune.log 2>&1 || exit $?
tail -3 $O/tune.log
for r in 1 2; do
  timeout -k 10 300 $SFT > $O/ab_old_$r.log 2>&1 || exit $?
  GRT_TUNED_GEMM_FILE=$PWD/$O/tuned.csv timeout -k 10 300 $SFT > $O/ab_new_$r.log 2>&1 || exit $?
  grep -h "training finished" $O/ab_old_$r.log $O/ab_new_$r.log | cut -c1-200
done
