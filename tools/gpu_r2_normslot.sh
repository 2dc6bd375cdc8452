#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2normslot
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_parallel_gpu.py tests/test_parallel_gpu_multiproc.py tests/test_kernels_gpu.py -k "norm or fsdp or overlap or early or llama or ranks or sequence" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab_env.sh r2normslot/ab "GRT_NORM_DIRECT_GRAD=0" "GRT_NORM_DIRECT_GRAD=1" 2
