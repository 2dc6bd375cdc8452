#!/bin/bash
# decode A/B on one box: RMSNorm folded into the GEMV (GRT_DECODE_NORM_GEMV) on / off, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2decab
mkdir -p $O
rm -f $O/ab.txt
for r in 1 2; do
  for v in 0 1; do
    GRT_DECODE_NORM_GEMV=$v timeout -k 10 300 python tools/decode_bench.py > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
    echo "GRT_DECODE_NORM_GEMV=$v round $r: $(grep hip_graph+gemv $O/run.log)" | tee -a $O/ab.txt
  done
done
