#!/bin/bash
# SFT job A/B: padded length multiple of the fused batch (8 = collator default, 64, 128).
set -o pipefail
mkdir -p gpurun_out
export GRT_STORAGE_PATH=/tmp/grt_sft
for m in 64 8 128; do
  GRT_SFT_PAD_MULTIPLE=$m timeout -k 10 300 python -u tools/sft_inproc.py --set OUTPUT_DIR_BASE=/tmp/grt_sft/p$m --set NUM_TRAIN_SAMPLES=480 --set NUM_EVAL_SAMPLES=16 --set SAVE_STRATEGY=no > gpurun_out/sft_pad$m.log 2>&1 || exit $?
  echo "pad $m"; grep -E "^\{'loss'|training finished" gpurun_out/sft_pad$m.log | cut -c1-240
done
