#!/bin/bash
# round-5 batch: gemm_k64 + IPC data-plane GPU tests, AdamW kernel bandwidth
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5batch1}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k k64 tests/test_ipc_gpu.py > $OUT/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|passed|failed" $OUT/tests.log | tail -40; fatal $rc
timeout -k 10 300 python -u tools/adamw_bench.py --reps 20 > $OUT/adamw.log 2>&1; rc=$?; grep "^{" $OUT/adamw.log; fatal $rc
echo done
