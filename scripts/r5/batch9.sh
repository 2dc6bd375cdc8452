#!/bin/bash
# deferred owned-slot write-backs: offload tests, then the 70B proxy-8 runs
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r5batch9; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_parallel_gpu.py -k "offload" > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -3; [ $rc = 0 ] || exit $rc
CFGS="auto:auto 0:auto 0.5:auto" bash scripts/r5/offload70.sh r5off70d
