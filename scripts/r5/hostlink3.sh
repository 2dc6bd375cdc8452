#!/bin/bash
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5hostlink3}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hostcopy_gpu.py "tests/test_ipc_gpu.py::test_ddp_small_bucket_over_ipc" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 tools/hostlink_bench.py > $OUT/hostlink.log 2>&1; rc=$?; tail -1 $OUT/hostlink.log; exit $rc
