#!/bin/bash
# Round 4 batch 6: which GEMM shapes of the QLoRA reference SFT job miss the table; HIP API trace of
# its worker loop (host calls that block between steps).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r4b6; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
export GRT_STORAGE_PATH=/tmp/grt_sftu
GRT_TUNED_GEMM_RECORD_UNTUNED=$PWD/$OUT/untuned.csv timeout -k 10 300 python3 tools/sft_inproc.py --set OUTPUT_DIR_BASE=/tmp/grt_sftu/out > $OUT/record.log 2>&1; rc=$?
grep "train_samples_per_second" $OUT/record.log | tail -1 | cut -c1-200; fatal $rc
cat $OUT/untuned*.csv 2>/dev/null | grep -c Gemm
rm -rf /tmp/grt_sftu
bash scripts/gpu_sft_hiptrace.sh r4b6/hip; rc=$?; fatal $rc
echo done
