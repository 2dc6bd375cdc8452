#!/bin/bash
# after the lora_down / lora_dx changes: LoRA tests, LoRA + headline bench, reference SFT job (packed default)
set -o pipefail
O=gpurun_out/${1:-r3c2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_lora_grad_gpu.py tests/test_varlen.py -x -q -k "lora or kcat or varlen" --timeout 120 --timeout-method thread > $O/t.log 2>&1 \
  || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python bench.py --peft lora > $O/b_lora.log 2>&1 || { tail -20 $O/b_lora.log; exit 1; }
echo "lora: $(tail -1 $O/b_lora.log | cut -c100-175)"
timeout -k 10 300 python bench.py > $O/b_head.log 2>&1 || { tail -20 $O/b_head.log; exit 1; }
echo "head: $(tail -1 $O/b_head.log | cut -c100-175)"
bash scripts/gpu_sft_job_trace.sh ${1:-r3c2}/sft1 || exit $?
bash scripts/gpu_sft_job_trace.sh ${1:-r3c2}/sft2 || exit $?
