#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2prodt
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_parallel_gpu.py -k "swiglu or llama or overlap or fsdp or wgrad" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab_env.sh r2prodt/ab "GRT_PRODUCER_T=0" "GRT_PRODUCER_T=1" 2
