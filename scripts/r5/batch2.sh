#!/bin/bash
# IPC data-plane GPU tests + memory-bound kernel bandwidth table
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5batch2}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ipc_gpu.py > $OUT/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|passed|failed" $OUT/tests.log | tail -40; fatal $rc
timeout -k 10 300 python -u tools/membw_bench.py --reps 30 --md > $OUT/membw.log 2>&1; rc=$?; cat $OUT/membw.log; fatal $rc
echo done
