#!/bin/bash
# GPU_MAX_HW_QUEUES (hardware queues per process; HIP default 4) on the headline.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-envab3}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
for r in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/b_${q}_$r.log 2>&1; rc=$?
    echo "queues=$q r$r $(tail -1 $OUT/b_${q}_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"; fatal $rc
  done
done
echo done
