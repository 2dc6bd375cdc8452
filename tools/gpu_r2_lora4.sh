#!/bin/bash
# split-K lora_down + one-pass dL/dh: numerics, LoRA bench A/B, kernel profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2lora4
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "lora" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
rm -f $O/ab3.jsonl
for r in 1 2; do
  for v in 0 down,dx down,dx,g; do
    GRT_LORA_KERNELS=$v timeout -k 10 300 python bench.py --steps 15 --warmup 4 --peft lora > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
    echo "GRT_LORA_KERNELS=$v round $r: $(tail -1 $O/run.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["loss"])')" | tee -a $O/ab3.txt
  done
done
bash tools/gpu_prof_bench.sh r2lora4/prof --peft lora || exit 1
python3 tools/prof_top.py $O/prof/prof/run_kernel_stats.csv 9 10 lora
