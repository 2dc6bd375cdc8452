#!/bin/bash
# LoRA gradients written straight into the DDP slots: GPU LoRA tests, then A/B on the LoRA bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2ld
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_jobs.py -k "lora or sft or peft" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab_env.sh r2ld "GRT_LORA_DIRECT_GRAD=0" "GRT_LORA_DIRECT_GRAD=1" ${ROUNDS:-2} --peft lora
