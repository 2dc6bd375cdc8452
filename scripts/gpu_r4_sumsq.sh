#!/bin/bash
# grad-norm sumsq with 4 loads in flight: clip / optimizer tests, headline x2, kernel stats.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4sumsq}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_parallel_gpu.py -q -k "clip or norm or adamw or overlap or ddp or sumsq" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $OUT/test.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR" $OUT/test.log | head; tail -1 $OUT/test.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/b_$r.log 2>&1; rc=$?
  echo "bench r$r $(tail -1 $OUT/b_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"loss": [0-9.]*' | tr '\n' ' ')"; fatal $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 2 > $OUT/prof.log 2>&1; rc=$?
grep -h "sumsq\|colsum" $OUT/prof/run_kernel_stats.csv | cut -c1-200; fatal $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log; fatal $rc
echo done
