#!/bin/bash
# SFT job with the bucket-tuned GEMMs, PMC zoo, bench modes
set -o pipefail
mkdir -p gpurun_out
cd jobs && GRT_STORAGE_PATH=/tmp/grt_sft timeout -k 10 400 python -u fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sft/out > ../gpurun_out/sft_ref_v5.log 2>&1 || exit $?
cd .. && grep -E "training finished" gpurun_out/sft_ref_v5.log | cut -c1-250
bash tools/gpu_pmc_zoo.sh || exit $?
bash tools/gpu_bench_modes.sh || exit $?
