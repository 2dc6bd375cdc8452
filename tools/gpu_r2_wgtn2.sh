#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2wgtn2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_parallel_gpu.py tests/test_parallel_gpu_multiproc.py -k "wgrad or llama or overlap or fsdp or early or ranks or zero or sequence" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab_env.sh r2wgtn2/ab "GRT_WGRAD_TN_OVERLAP=0" "GRT_WGRAD_TN_OVERLAP=1" 2
