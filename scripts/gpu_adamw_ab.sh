#!/bin/bash
# AdamW microbench A/B of the plain update's grid cap, then the headline bench with the new adamw_t.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-adamwab}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
for cap in 2048 16384 65536; do
  GRT_ADAMW_GRID_CAP=$cap timeout -k 10 200 python -u tools/adamw_bench.py > $OUT/cap$cap.jsonl 2>&1; rc=$?
  echo "cap $cap"; grep -o '"param": "[a-z_]*"\|"adamw_sr1_us": [0-9.]*' $OUT/cap$cap.jsonl | tr '\n' ' '; echo; fatal $rc
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "adamw" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/test.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR" $OUT/test.log | head; tail -1 $OUT/test.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_$r.log 2>&1; rc=$?
  echo "bench r$r $(tail -1 $OUT/bench_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"; fatal $rc
done
echo done
