#!/bin/bash
# memory-bound kernel table + A/B of the transposing kernels' store / walk variants
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5membw}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u tools/membw_bench.py --reps 30 --md > $OUT/membw.log 2>&1; rc=$?
grep -v "^{" $OUT/membw.log; echo "rc=$rc"; exit $rc
