#!/bin/bash
# lora_g with B^T through a private LDS image: numerics, LoRA bench, LoRA step kernel profile
set -o pipefail
O=gpurun_out/${1:-r3lg2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lora_grad_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_grad.log 2>&1 \
  || { tail -30 $O/t_grad.log; exit 1; }
tail -1 $O/t_grad.log
timeout -k 10 300 python bench.py --peft lora > $O/bench_lora.log 2>&1 || { tail -20 $O/bench_lora.log; exit 1; }
echo "lora: $(tail -1 $O/bench_lora.log | cut -c1-190)"
bash scripts/gpu_prof.sh $O/prof_lora --peft lora --steps 6 --warmup 3 || exit $?
