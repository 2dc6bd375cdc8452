#!/bin/bash
# Overlapped vs serial per-module transposing AdamW on the headline step (A/B, interleaved).
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-optser}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
for r in 1 2; do
  for sr in 0 1; do
    GRT_OVERLAP_OPT_SERIAL=$sr timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/b_${sr}_$r.log 2>&1; rc=$?
    echo "serial=$sr r$r $(tail -1 $OUT/b_${sr}_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"loss": [0-9.]*' | tr '\n' ' ')"; fatal $rc
  done
done
echo done
