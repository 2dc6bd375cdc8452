#!/bin/bash
# headline bench: optimizer placement A/B (overlapped chunks vs serial vs ZeRO machinery at world 1)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/optmode_ab.txt
for mode in "--overlap-opt off" "--overlap-opt on" "--zero on" "--overlap-opt off" "--overlap-opt on" "--zero on"; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 $mode > gpurun_out/optmode.log 2>&1 || exit $?
  echo "$mode $(tail -1 gpurun_out/optmode.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["parallelism"], d["config"]["optimizer_overlap"])')" | tee -a gpurun_out/optmode_ab.txt
done
