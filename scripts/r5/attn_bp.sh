#!/bin/bash
# flash-attention forward: one workgroup barrier per tile (BP 1, default) vs per two tiles (BP 2,
# 5-slot ring); numerics tests under BP 2, then tools/attn_ab.py under each
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5attnbp}; rm -rf $OUT; mkdir -p $OUT
GRT_ATTN_FWD_BP=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention or flash" > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for bp in 1 2; do
    GRT_ATTN_FWD_BP=$bp timeout -k 10 200 python -u tools/attn_ab.py --rounds 5 > $OUT/ab_${bp}_$i.log 2>&1; rc=$?
    echo "BP=$bp run $i: $(grep -i "fwd\|forward" $OUT/ab_${bp}_$i.log | head -3 | tr '\n' ' ' | cut -c1-300)"; [ $rc = 0 ] || exit $rc
  done
done
