#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2enorm
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_parallel_gpu.py tests/test_kernels_gpu.py -k "early or fsdp or overlap or adamw" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab_env.sh r2enorm/ab "GRT_EARLY_GRAD_NORM=0" "GRT_EARLY_GRAD_NORM=1" 2
