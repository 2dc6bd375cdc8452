#!/bin/bash
# offload prefetch GPU tests, then the 70B proxy-8 offload runs (scripts/r5/offload70.sh)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5batch3}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_parallel_gpu.py -k "offload" > $OUT/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|passed|failed" $OUT/tests.log | tail -20; [ $rc = 0 ] || exit $rc
bash scripts/r5/offload70.sh ${OFF_OUT:-r5off70}
