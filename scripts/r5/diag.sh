#!/bin/bash
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5diag}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 python -u tools/gemm_diag.py --variant ${2:-9} > $OUT/diag.log 2>&1; rc=$?; cat $OUT/diag.log | tail -60; exit $rc
