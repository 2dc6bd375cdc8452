#!/bin/bash
# final bench modes on one GPU: LoRA, QLoRA, FSDP (BASELINE configs #4, #3)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2mf
mkdir -p $O
rm -f $O/modes.jsonl
for args in "--peft lora" "--peft qlora" "--parallel fsdp"; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 $args > $O/run.log 2>&1 || { echo "[$args] failed"; tail -20 $O/run.log; exit 1; }
  tail -1 $O/run.log >> $O/modes.jsonl
  echo "$args: $(tail -1 $O/run.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["config"]["parallelism"], d["loss"])')"
done
