#!/bin/bash
# GEMV per-projection times with and without evicting the weights between calls (MALL effect)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5gemvflush}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 python -u tools/gemv_bench.py > $OUT/warm.log 2>&1; rc=$?; grep "^{" $OUT/warm.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u tools/gemv_bench.py --flush > $OUT/flush.log 2>&1; rc=$?; grep "^{" $OUT/flush.log; [ $rc = 0 ] || exit $rc
