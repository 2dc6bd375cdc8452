#!/bin/bash
# Round-3 batch 3: tune the padding-free SFT step's odd-512 GEMM shapes, then the reference SFT job
# end to end: padded (shipped table) vs padding-free on the merged table.
set -o pipefail
O=gpurun_out/${1:-r3batch3}
mkdir -p $O
SFT_ENV=GRT_SFT_PADDING_FREE=1 TUNE_S=900 TUNE_ONLY="_5632_,_6656_,_7680_,_4608_" \
  bash scripts/gpu_sft_tune.sh ${1:-r3batch3}/pfree_tune || exit $?
bash scripts/gpu_sft_job_trace.sh ${1:-r3batch3}/sft_padded || exit $?
bash scripts/gpu_sft_job_trace.sh ${1:-r3batch3}/sft_pfree_tuned GRT_SFT_PADDING_FREE=1 \
  GRT_TUNED_GEMM_FILE=$PWD/$O/pfree_tune/tuned.csv || exit $?
