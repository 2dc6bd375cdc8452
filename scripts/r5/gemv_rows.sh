#!/bin/bash
# GEMV (1-2 rows FMA, 3-16 rows MFMA) vs hipBLASLt per projection, weights evicted between calls
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5gemvrows}; rm -rf $OUT; mkdir -p $OUT
for m in 1 4 8 16; do
  timeout -k 10 200 python -u tools/gemv_bench.py --m $m --flush > $OUT/m$m.log 2>&1; rc=$?; grep '"shape"' $OUT/m$m.log | grep -v "+" | cut -c1-170; [ $rc = 0 ] || exit $rc
done
