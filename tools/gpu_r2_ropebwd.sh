#!/bin/bash
# RoPE backward fused into the attention backward epilogues: attention / model GPU tests + headline A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2rb
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels_gpu_sweep.py tests/test_parallel_gpu.py -k "attention or llama or rope or sequence or flash" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab_env.sh r2rb "GRT_ROPE_BWD_FUSED=0" "GRT_ROPE_BWD_FUSED=1" 2
