#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2pace
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_parallel_gpu.py -k "overlap" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
rm -f $O/ab.txt
for r in 1 2; do
  for v in 0 2 4 8; do
    GRT_OPT_PACE=$v timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
    echo "GRT_OPT_PACE=$v round $r: $(tail -1 $O/run.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')" | tee -a $O/ab.txt
  done
done
