#!/bin/bash
# reference SFT job with the eval forward under no_grad (eval_runtime / train_samples_per_second)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2sfte
mkdir -p $O
export GRT_STORAGE_PATH=/tmp/grt_sft_e
timeout -k 10 400 python -u jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sft_e/out > $O/sft.log 2>&1 || { echo "sft failed"; tail -30 $O/sft.log; exit 1; }
grep -E "eval_runtime|train_samples_per_second" $O/sft.log | cut -c1-220
