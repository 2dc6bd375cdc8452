#!/bin/bash
# NF4 v2 dequant + streamed K-concatenated QLoRA: tests, then QLoRA bench cache on / off (streamed) /
# off without the streamed path, 2 rounds; kernel stats of the streamed step.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-nf4b}; rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_jobs.py -q -k "nf4 or kcat or qlora or lora" \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/test.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR" $OUT/test.log | head; tail -1 $OUT/test.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for arm in "auto 1" "0 1" "0 0"; do
    set -- $arm
    GRT_NF4_CACHE=$1 GRT_NF4_STREAM_KCAT=$2 timeout -k 10 300 python bench.py --peft qlora --steps 10 --warmup 3 > $OUT/b_$1$2_$r.log 2>&1; rc=$?
    echo "cache=$1 stream=$2 r$r $(tail -1 $OUT/b_$1$2_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"hbm_peak_gib": [0-9.]*\|"hbm_plan_gib": [0-9.]*' | tr '\n' ' ')"
    fatal $rc; [ $rc -eq 0 ] || exit $rc
  done
done
GRT_NF4_CACHE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --peft qlora --steps 4 --warmup 2 > $OUT/prof.log 2>&1; rc=$?
echo "prof rc $rc"; fatal $rc
echo done
