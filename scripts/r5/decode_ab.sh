#!/bin/bash
# decode A/B of one env switch (default: the fused decode-attention combine), interleaved on one box
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5decab}; VAR=${2:-GRT_DECODE_ATTN_FUSE}; rm -rf $OUT; mkdir -p $OUT
env $VAR=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "decode or gemv" > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 300 python -u tools/decode_bench.py > $OUT/decode_${v}_$i.log 2>&1; rc=$?
    echo "$VAR=$v run $i: $(grep hip_graph+gemv $OUT/decode_${v}_$i.log)"; [ $rc = 0 ] || exit $rc
  done
done
