#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2sr
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_parallel_gpu.py tests/test_kernels_gpu.py -k "adamw or overlap or offload or fsdp or early or stochastic" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 1; do
  GRT_ADAMW_SR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 2 --metrics-jsonl $O/m$v.jsonl > $O/b$v.log 2>&1 || exit 1
  echo "SR=$v $(tail -1 $O/b$v.log | cut -c 150-260)"
  python3 -c "import json; print('losses', [round(json.loads(l)['loss'], 3) for l in open('$O/m$v.jsonl')])"
done
