#!/bin/bash
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5adamw}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u tools/adamw_bench.py --reps 20 > $OUT/adamw.log 2>&1; rc=$?; cat $OUT/adamw.log | grep "^{"; exit $rc
