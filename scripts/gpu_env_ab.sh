#!/bin/bash
# Generic interleaved A/B of one environment switch on the 1-GPU bench (and optionally the SFT
# worker loop): scripts/gpu_env_ab.sh <out-subdir> <VAR> <valueA> <valueB> <rounds> [bench args...]
# Set SFT_AB=1 to A/B the SFT worker loop (320 samples) instead of bench.py.
set -o pipefail
O=gpurun_out/$1; VAR=$2; A=$3; B=$4; N=$5
shift 5
mkdir -p $O
export GRT_STORAGE_PATH=/tmp/grt_envab
for r in $(seq 1 $N); do
  for v in $A $B; do
    if [ "${SFT_AB:-0}" = "1" ]; then
      env $VAR=$v timeout -k 10 300 python3 tools/sft_inproc.py --set NUM_TRAIN_SAMPLES=320 \
        --set OUTPUT_DIR_BASE=/tmp/grt_envab/out > $O/${VAR}_${v}_$r.log 2>&1 || exit $?
      echo "$VAR=$v r$r: $(grep -h 'training finished' $O/${VAR}_${v}_$r.log | cut -c1-160)"
    else
      env $VAR=$v timeout -k 10 300 python3 bench.py "$@" > $O/${VAR}_${v}_$r.log 2>&1 || exit $?
      echo "$VAR=$v r$r: $(tail -1 $O/${VAR}_${v}_$r.log | cut -c1-150)"
    fi
  done
done
