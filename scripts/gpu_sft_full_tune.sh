#!/bin/bash
# BASELINE config #2 through the reference SFT job (full FT, Llama-2-7B): log every library GEMM the
# shipped table misses (padding-free packed steps of 4.5-8 K tokens, multiples of 512), tune them
# offline (poison-checked). The A/B of the job / bench.py on both tables is scripts/gpu_sft_full_ab.sh.
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
timeout -k 10 ${TUNE_S:-840} python3 tools/tune_untuned.py "$O/untuned*.csv" --out $O/tuned.csv > $O/tune.log 2>&1; rc=$?
tail -3 $O/tune.log; fatal $rc
echo done
