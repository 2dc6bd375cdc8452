#!/bin/bash
# lora_down with two 32-token tiles per workgroup (A chunk loads halved): LoRA tests, bench A/B
set -o pipefail
O=gpurun_out/${1:-r3ldt}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_lora_grad_gpu.py -x -q -k "lora or kcat" --timeout 120 --timeout-method thread > $O/t.log 2>&1 \
  || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for cfg in "GRT_LORA_DOWN_TB=2" "GRT_LORA_DOWN_TB=1" "GRT_LORA_DOWN_TB=2 GRT_LORA_DOWN_KC=64" "GRT_LORA_DOWN_TB=2" "GRT_LORA_DOWN_TB=1"; do
  env $cfg timeout -k 10 300 python bench.py --peft lora > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  echo "$cfg: $(tail -1 $O/b.log | cut -c100-175)"
done
