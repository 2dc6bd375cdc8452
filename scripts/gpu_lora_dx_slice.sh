#!/bin/bash
# lora_dx with R sliced by 64 at R > 128 (4 workgroups per CU): LoRA tests, bench, LoRA step profile
set -o pipefail
O=gpurun_out/${1:-r3ldx}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_lora_grad_gpu.py -x -q -k "lora or kcat" --timeout 120 --timeout-method thread > $O/t.log 2>&1 \
  || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python bench.py --peft lora > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
echo "lora: $(tail -1 $O/b.log | cut -c100-175)"
bash scripts/gpu_prof.sh $O/prof_lora --peft lora --steps 6 --warmup 3 || exit $?
