#!/bin/bash
# Full GPU test suite + smoke + headline bench (state check)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4full}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR" $OUT/tests.log | head -20; tail -2 $OUT/tests.log; fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -2 $OUT/smoke.log; fatal $rc
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1; rc=$?; tail -1 $OUT/bench.log | cut -c1-400; fatal $rc
echo done
