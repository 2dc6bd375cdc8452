#!/bin/bash
# round-5 state check on one box: full GPU suite, smoke, headline bench, kernel trace of the bench
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5final}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -5 $OUT/gpu_tests.log; fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -2 $OUT/smoke.log; fatal $rc
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1; rc=$?; tail -1 $OUT/bench.log | cut -c1-400; fatal $rc
timeout -k 10 300 python bench.py > $OUT/bench2.log 2>&1; rc=$?; tail -1 $OUT/bench2.log | cut -c1-200; fatal $rc
bash scripts/gpu_prof.sh $OUT/prof --steps 6 --warmup 3; rc=$?; fatal $rc
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steps.py "$f" 9 > $OUT/step_breakdown.md 2>&1; head -40 $OUT/step_breakdown.md
rm -rf $OUT/prof
