#!/bin/bash
# headline + bench modes on one MI355X (one JSON line per mode -> gpurun_out/bench_modes.jsonl)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/bench_modes.jsonl
for mode in "" "--parallel fsdp" "--peft lora" "--peft qlora" "--peft lora --data pipeline"; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 3 $mode > gpurun_out/bench_mode.log 2>&1 || { echo "bench $mode failed"; tail -20 gpurun_out/bench_mode.log; exit 1; }
  tail -1 gpurun_out/bench_mode.log >> gpurun_out/bench_modes.jsonl
  echo "$mode: $(tail -1 gpurun_out/bench_mode.log | cut -c100-190)"
done
