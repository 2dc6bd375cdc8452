#!/bin/bash
# k64 GEMM wait-source experiment: variants 13-16 drop the vmcnt wait / lgkmcnt waits / barriers
# (results wrong, timing only) next to variant 9 and the library
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5gemmdiag}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u tools/gemm_bench.py --set fwd,dgrad --variants ${VARIANTS:-9,13,14,15,16} --no-check --rounds 3 --reps 10 > $OUT/gemm.log 2>&1; rc=$?
grep -E '^\{|Error|error' $OUT/gemm.log | head -40; echo "rc=$rc"; exit $rc
