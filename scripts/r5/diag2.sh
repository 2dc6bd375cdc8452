#!/bin/bash
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5diag2}; rm -rf $OUT; mkdir -p $OUT
GRT_DIAG_TILES=${2:-9} timeout -k 10 200 python -u tools/gemm_diag.py > $OUT/diag.log 2>&1; rc=$?; cat $OUT/diag.log | tail -40; exit $rc
