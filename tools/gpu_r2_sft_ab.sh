#!/bin/bash
# SFT job (reference fine_tune_llama_ray.py workload: Llama-3.1-8B QLoRA, 1 GPU) with the LoRA
# adapter kernels on vs off, same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2sft
mkdir -p $O
for v in 1 0; do
  export GRT_STORAGE_PATH=/tmp/grt_sft_$v
  GRT_LORA_KERNELS=$v timeout -k 10 400 python -u jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sft_$v/out > $O/sft_$v.log 2>&1 || { echo "sft $v failed"; tail -30 $O/sft_$v.log; exit 1; }
  echo "GRT_LORA_KERNELS=$v: $(grep -E "train_samples_per_second" $O/sft_$v.log | tail -1 | cut -c1-260)"
done
