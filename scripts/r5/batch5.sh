#!/bin/bash
# dedicated prefetch slots: offload tests + 70B resident 0 / 0.5 runs + memory-copy trace; BasicLLM in-process kernel trace
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r5batch5; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_parallel_gpu.py -k "overlapped_offload" > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -3; [ $rc = 0 ] || exit $rc
CFGS="0:auto 0.5:auto" bash scripts/r5/offload70.sh r5off70c || exit $?
bash scripts/r5/offtrace.sh r5offtrace || exit $?
bash scripts/r5/basicllm_prof.sh r5basicllm
