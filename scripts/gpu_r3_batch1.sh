#!/bin/bash
# Round-3 measurement batch: attention / LoRA correctness, per-kernel attention schedule A/B,
# LoRA dX-epilogue A/B on the LoRA bench, SFT job padded vs padding-free at 1024-token multiples.
set -o pipefail
O=gpurun_out/${1:-r3batch1}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "lora or kcat or attn or attention or varlen or flash" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/attn_ab.py --scheds 0,1,3,5,7 --rounds 7 > $O/attn_ab.jsonl 2>&1 || { cat $O/attn_ab.jsonl; exit 1; }
grep -v max_err $O/attn_ab.jsonl
bash scripts/gpu_env_ab.sh ${1:-r3batch1}/epi GRT_LORA_DX_EPI 0 1 2 --peft lora || exit $?
bash scripts/gpu_sft_job_trace.sh ${1:-r3batch1}/sft_padded || exit $?
bash scripts/gpu_sft_job_trace.sh ${1:-r3batch1}/sft_pfree1024 GRT_SFT_PADDING_FREE=1 GRT_SFT_PAD_MULTIPLE=1024 || exit $?
