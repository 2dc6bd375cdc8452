#!/bin/bash
# LoRA adapter-gradient kernels (lora_grad.hip): numerics vs fp32, LoRA tests, LoRA bench A/B
# (GRT_LORA_GRAD_KERNELS=1 / 0 / 1), kernel profile of the LoRA step with the kernels on.
set -o pipefail
O=gpurun_out/${1:-r3lg}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lora_grad_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_grad.log 2>&1 \
  || { tail -30 $O/t_grad.log; exit 1; }
tail -1 $O/t_grad.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "lora or kcat" --timeout 120 --timeout-method thread > $O/t_lora.log 2>&1 \
  || { tail -30 $O/t_lora.log; exit 1; }
tail -1 $O/t_lora.log
for v in 1 0 1; do
  GRT_LORA_GRAD_KERNELS=$v timeout -k 10 300 python bench.py --peft lora > $O/bench_lora_k$v.log 2>&1 || { tail -20 $O/bench_lora_k$v.log; exit 1; }
  echo "lora grad kernels=$v: $(tail -1 $O/bench_lora_k$v.log | cut -c1-190)"
done
bash scripts/gpu_prof.sh $O/prof_lora --peft lora --steps 6 --warmup 3 || exit $?
# padding-free SFT steps on the candidate GEMM table (odd multiples of 512 tokens tuned)
timeout -k 10 300 python -u tools/varlen_probe.py \
  --cfgs 5632,6144,6656 --padded "" > $O/varlen_probe_cand.jsonl 2> $O/varlen_probe_cand.err || { tail $O/varlen_probe_cand.err; exit 1; }
cat $O/varlen_probe_cand.jsonl
bash scripts/gpu_sft_job_trace.sh ${1:-r3lg}/sft_padded || exit $?
bash scripts/gpu_sft_job_trace.sh ${1:-r3lg}/sft_packed GRT_SFT_PADDING_FREE=1 || exit $?
