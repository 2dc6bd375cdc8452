#!/bin/bash
# Same-box A/B of two full bench configurations (env + args per arm), alternating, 2 rounds:
#   A = default (overlapped AdamW writing W^T), B = serial AdamW + side-stream W^T transposes in the forward
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2modeab
mkdir -p $O
rm -f $O/ab.txt
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
  echo "A default round $r: $(tail -1 $O/run.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["loss"])')" | tee -a $O/ab.txt
  GRT_TRANSPOSED_DGRAD_TRAINABLE=1 timeout -k 10 300 python bench.py --steps 15 --warmup 4 --overlap-opt off > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
  echo "B serial+fwdT round $r: $(tail -1 $O/run.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["loss"])')" | tee -a $O/ab.txt
  timeout -k 10 300 python bench.py --steps 15 --warmup 4 --overlap-opt off > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
  echo "C serial round $r: $(tail -1 $O/run.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["loss"])')" | tee -a $O/ab.txt
done
