#!/bin/bash
# Full GPU suite, then the reference SFT job (Llama-3.1-8B QLoRA, 1 GPU) with LoRA direct-grad on/off
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2sftd
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0; do
  export GRT_STORAGE_PATH=/tmp/grt_sft_$v
  GRT_LORA_DIRECT_GRAD=$v timeout -k 10 400 python -u jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sft_$v/out > $O/sft_$v.log 2>&1 || { echo "sft $v failed"; tail -30 $O/sft_$v.log; exit 1; }
  echo "GRT_LORA_DIRECT_GRAD=$v: $(grep -E "train_samples_per_second" $O/sft_$v.log | tail -1 | cut -c1-260)"
done
