#!/bin/bash
# A/B: training step on a high-priority stream (side streams at default priority) vs default
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5prio}; rm -rf $OUT; mkdir -p $OUT
for r in 1 2; do
  for v in normal high; do
    GRT_COMPUTE_STREAM_PRIORITY=$v timeout -k 10 300 python bench.py > $OUT/bench_${v}_$r.log 2>&1; rc=$?
    echo "prio=$v run $r: $(tail -1 $OUT/bench_${v}_$r.log | cut -c100-200)"; [ $rc = 0 ] || exit $rc
  done
done
