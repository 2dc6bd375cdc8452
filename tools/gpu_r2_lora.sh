#!/bin/bash
# LoRA adapter kernels: GPU numerics, then LoRA bench A/B (torch path vs lora.hip) on one box.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2lora
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "lora or dropout" > gpurun_out/r2lora/tests.log 2>&1 || { tail -40 gpurun_out/r2lora/tests.log; exit 1; }
tail -3 gpurun_out/r2lora/tests.log
bash tools/gpu_ab_env.sh r2lora "GRT_LORA_KERNELS=0" "GRT_LORA_KERNELS=1" 2 --peft lora
