#!/bin/bash
# SFT job (reference config, 1000 samples) on one MI355X: fused accumulation + NF4 dequant cache
# vs the unfused / transient-dequant paths; then the new kernel tests.
set -o pipefail
mkdir -p gpurun_out
export GRT_STORAGE_PATH=/tmp/grt_sft
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lm_head" > gpurun_out/sft_fuse_tests.log 2>&1 || exit $?
for mode in fused_cache fused_nocache; do
  case $mode in
    fused_cache) envs="GRT_SFT_FUSE_ACCUM=1 GRT_NF4_CACHE=auto";;
    fused_nocache) envs="GRT_SFT_FUSE_ACCUM=1 GRT_NF4_CACHE=0";;
  esac
  env $envs timeout -k 10 400 python -u jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sft/$mode > gpurun_out/sft_$mode.log 2>&1 || exit $?
  grep -E "^\{'loss'|eval_loss|training finished" gpurun_out/sft_$mode.log | cut -c1-260
done
