#!/bin/bash
# reference SFT job: padded vs padding-free steps (varlen attention without causal pairs), interleaved
set -o pipefail
O=gpurun_out/${1:-r3pk}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_varlen.py tests/test_lora_grad_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for mode in packed padded packed padded; do
  if [ $mode = packed ]; then E=GRT_SFT_PADDING_FREE=1; else E=GRT_SFT_PADDING_FREE=0; fi
  bash scripts/gpu_sft_job_trace.sh ${1:-r3pk}/$mode$((++n)) $E || exit $?
done
