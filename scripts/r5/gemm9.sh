#!/bin/bash
# k64 GEMM (variant 9) correctness + A/B vs hipBLASLt on the Llama-2-7B step shapes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5gemm9}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 python -u tools/gemm_bench.py --set fwd,dgrad,wgrad --variants 9,10 --rounds 5 --reps 10 > $OUT/gemm.log 2>&1; rc=$?
grep -E '^\{|check|wrong|Error|error' $OUT/gemm.log | head -60; echo "rc=$rc"; exit $rc
