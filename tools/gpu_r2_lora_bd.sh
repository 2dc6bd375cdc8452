#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2lorabd
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "lora" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab_env.sh r2lorabd/ab "GRT_LORA_BLOCKDIAG=0" "GRT_LORA_BLOCKDIAG=1" 2 --peft lora
