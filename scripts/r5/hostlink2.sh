#!/bin/bash
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5hostlink2}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 python3 tools/hostlink_bench.py > $OUT/plain.log 2>&1; rc=$?; tail -1 $OUT/plain.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python3 tools/fp32_gemm_probe.py > $OUT/fp32.log 2>&1; rc=$?; tail -1 $OUT/fp32.log; exit $rc
