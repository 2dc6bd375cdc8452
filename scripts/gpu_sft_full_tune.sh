#!/bin/bash
# BASELINE config #2 through the reference SFT job (full FT, Llama-2-7B): log every library GEMM the
# shipped table misses (padding-free packed steps of 4.5-8 K tokens, multiples of 512), tune them
# offline (poison-checked), then A/B the job and bench.py at the job's tokens/step on both tables.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ft}; rm -rf $O; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
export GRT_STORAGE_PATH=/tmp/grt_ft
FT="python3 tools/sft_inproc.py --set USE_QLORA=false --set MODEL_ID=llama2-7b --set SAVE_STRATEGY=no --set REPORT_TO=none --set NUM_TRAIN_SAMPLES=400 --set LEARNING_RATE=2e-5 --set OUTPUT_DIR_BASE=/tmp/grt_ft/out"
GRT_TUNED_GEMM_RECORD_UNTUNED=$PWD/$O/untuned.csv timeout -k 10 300 $FT > $O/record.log 2>&1; rc=$?
grep -E "tokens_per_sec|training finished" $O/record.log | cut -c1-200; fatal $rc; [ $rc = 0 ] || exit $rc
GRT_TUNED_GEMM_RECORD_UNTUNED=$PWD/$O/untuned_b6.csv timeout -k 10 200 python3 bench.py --batch 6 --steps 3 --warmup 2 > $O/record_b6.log 2>&1; rc=$?; fatal $rc
ls $O; cat $O/untuned*.csv | grep -c Gemm
timeout -k 10 1500 python3 tools/tune_untuned.py "$O/untuned*.csv" --out $O/tuned.csv > $O/tune.log 2>&1; rc=$?
tail -3 $O/tune.log; fatal $rc; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 $FT > $O/ab_old_$r.log 2>&1; rc=$?; fatal $rc
  GRT_TUNED_GEMM_FILE=$PWD/$O/tuned.csv timeout -k 10 300 $FT > $O/ab_new_$r.log 2>&1; rc=$?; fatal $rc
  grep -h "tokens_per_sec" $O/ab_old_$r.log | tail -3 | cut -c1-160
  grep -h "tokens_per_sec" $O/ab_new_$r.log | tail -3 | cut -c1-160
done
timeout -k 10 200 python3 bench.py --batch 6 --steps 20 --warmup 5 > $O/b6_old.log 2>&1; rc=$?; tail -1 $O/b6_old.log | cut -c1-200; fatal $rc
GRT_TUNED_GEMM_FILE=$PWD/$O/tuned.csv timeout -k 10 200 python3 bench.py --batch 6 --steps 20 --warmup 5 > $O/b6_new.log 2>&1; rc=$?; tail -1 $O/b6_new.log | cut -c1-200; fatal $rc
echo done
