#!/bin/bash
# decode tests + batch 1 / 2 / 4 decode (GEMV up to 2 rows, library GEMM beyond)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2g2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_jobs.py -k "gemv or decode or generation or graph" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for b in 2 1; do
  DECODE_B=$b timeout -k 10 300 python tools/decode_bench.py > $O/bench_$b.log 2>&1 || { tail -20 $O/bench_$b.log; exit 1; }
  grep tokens_per_s $O/bench_$b.log
done
