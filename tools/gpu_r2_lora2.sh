#!/bin/bash
# tuned-table correctness gate + LoRA kernel tests, per-step losses, LoRA bench A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2lora2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_tuning_gpu.py \
  tests/test_kernels_gpu.py -k "tuned or poisoned or lora" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0; do
  GRT_LORA_KERNELS=$v timeout -k 10 200 python bench.py --peft lora --steps 4 --warmup 0 --metrics-jsonl $O/m$v.jsonl > $O/m$v.log 2>&1 || exit 1
  python3 -c "import json; print('kernels=$v losses', [round(json.loads(l)['loss'], 4) for l in open('$O/m$v.jsonl')])"
done
bash tools/gpu_ab_env.sh r2lora2/ab "GRT_LORA_KERNELS=0" "GRT_LORA_KERNELS=1" 2 --peft lora
