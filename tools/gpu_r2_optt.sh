#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2optt
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_parallel_gpu.py tests/test_kernels_gpu.py -k "adamw or overlap or early or fsdp or llama" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab_env.sh r2optt/ab "GRT_OPT_TRANSPOSE=0" "GRT_OPT_TRANSPOSE=1" 2
