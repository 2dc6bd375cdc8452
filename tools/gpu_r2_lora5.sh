#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2lora5
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "lora" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_ab_env.sh r2lora5/ab "GRT_LORA_DOWN_KC=128" "GRT_LORA_DOWN_KC=64" 2 --peft lora || exit 1
GRT_LORA_DOWN_KC=64 bash tools/gpu_prof_bench.sh r2lora5/prof --peft lora || exit 1
python3 tools/prof_top.py $O/prof/prof/run_kernel_stats.csv 9 10 lora
