#!/bin/bash
# A/B of an environment switch on the 1-GPU headline bench, same box, alternating runs:
#   bash tools/gpu_ab_env.sh <outdir> "<env A>" "<env B>" [rounds] [bench args...]
# e.g. bash tools/gpu_ab_env.sh r2ab "GRT_WGRAD_STREAM=0" "GRT_WGRAD_STREAM=1" 2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
A=$2
B=$3
R=${4:-2}
shift 4
mkdir -p $O
rm -f $O/ab.jsonl
for r in $(seq 1 $R); do
  for v in "$A" "$B"; do
    env $v timeout -k 10 300 python bench.py --steps 15 --warmup 4 "$@" > $O/run.log 2>&1 || { echo "bench [$v] failed"; tail -20 $O/run.log; exit 1; }
    echo "{\"env\": \"$v\", \"round\": $r, \"result\": $(tail -1 $O/run.log)}" >> $O/ab.jsonl
    echo "$v round $r: $(tail -1 $O/run.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
