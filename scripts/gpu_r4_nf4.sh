#!/bin/bash
# QLoRA with and without the resident NF4 dequant cache (bench --peft qlora), + kernel stats of the
# cache-off step.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-nf4}; rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
for r in 1 2; do
  for c in auto 0; do
    GRT_NF4_CACHE=$c timeout -k 10 300 python bench.py --peft qlora --steps 10 --warmup 3 > $OUT/b_${c}_$r.log 2>&1; rc=$?
    echo "cache=$c r$r $(tail -1 $OUT/b_${c}_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"hbm_peak_gib": [0-9.]*\|"hbm_plan_gib": [0-9.]*' | tr '\n' ' ')"
    fatal $rc; [ $rc -eq 0 ] || exit $rc
  done
done
GRT_NF4_CACHE=${2:-0} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --peft qlora --steps 4 --warmup 2 > $OUT/prof.log 2>&1; rc=$?
echo "prof rc $rc"; fatal $rc
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
echo done
