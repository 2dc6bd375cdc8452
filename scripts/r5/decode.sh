#!/bin/bash
# decode step: GEMV bandwidth per projection, decode throughput, kernel stats of the decode loop
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5decode}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemv or decode" > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u tools/gemv_bench.py > $OUT/gemv.log 2>&1; rc=$?; grep "^{" $OUT/gemv.log; [ $rc = 0 ] || exit $rc

timeout -k 10 300 python -u tools/decode_bench.py > $OUT/decode.log 2>&1; rc=$?; grep "^{" $OUT/decode.log; [ $rc = 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o dec -- python3 $GRAFT_REPO_ROOT/tools/decode_bench.py > $GRAFT_REPO_ROOT/$OUT/decode_prof.log 2>&1; rc=$?
cd $GRAFT_REPO_ROOT; f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv; head -16 $OUT/kernel_stats.csv | cut -c1-180; rm -rf $OUT/prof; exit $rc
