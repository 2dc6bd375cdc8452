#!/bin/bash
# round-5 baseline on a fresh box: headline bench + library-vs-hand GEMM microbench (fwd shapes)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5base}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1; rc=$?; tail -1 $OUT/bench.log | cut -c1-300; fatal $rc
timeout -k 10 300 python tools/gemm_bench.py --set fwd --variants 3,4 --rounds 3 --reps 10 > $OUT/gemm.log 2>&1; rc=$?; grep '^{' $OUT/gemm.log; fatal $rc
echo done
