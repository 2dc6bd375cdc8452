#!/bin/bash
# adamw_t 128-row tiles: numerics, isolated bandwidth (64 vs 128), headline A/B
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5adamw2}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adamw" > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed" $OUT/tests.log | tail -2; fatal $rc
for t in 64 128; do
  GRT_ADAMW_T_ROWS=$t timeout -k 10 200 python -u tools/adamw_bench.py --reps 20 > $OUT/adamw_$t.log 2>&1; rc=$?
  echo "rows=$t"; grep "^{" $OUT/adamw_$t.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['param'], d['adamw_t_sr1_us'], d['adamw_t_sr1_TBps'])"; fatal $rc
done
for r in 1 2; do
  for t in 64 128; do
    GRT_ADAMW_T_ROWS=$t timeout -k 10 300 python bench.py > $OUT/bench_${t}_$r.log 2>&1; rc=$?
    echo "rows=$t run $r: $(tail -1 $OUT/bench_${t}_$r.log | cut -c100-200)"; fatal $rc
  done
done
