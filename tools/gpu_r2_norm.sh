#!/bin/bash
# norm kernels: numerics, then headline bench + kernel profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2norm
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels_gpu_sweep.py \
  -k "norm or layer" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/bench.log 2>&1 && tail -1 $O/bench.log && bash tools/gpu_prof_bench.sh r2norm/prof
