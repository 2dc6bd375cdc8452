#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2tr2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "transpose or wgrad or llama" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0; do GRT_TRANSPOSE_V1=$v timeout -k 10 300 python -u tools/wgrad_transpose_ab.py > $O/mb_v1_$v.log 2>&1 || exit 1; echo "V1=$v"; grep shape $O/mb_v1_$v.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(' ', d['shape'], 'tr', d['tr_us'], 'tn+tr', d['tn+tr_us'])
"; done
bash tools/gpu_ab_env.sh r2tr2/ab "GRT_TRANSPOSE_V1=1" "GRT_TRANSPOSE_V1=0" 2
