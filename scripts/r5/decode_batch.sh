#!/bin/bash
# batched decode: skinny MFMA GEMM (3-16 rows) vs the library GEMM, Llama-3.1-8B, batch 4 / 8 / 16
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5decbatch}; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemv" > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log; [ $rc = 0 ] || exit $rc
for b in 4 8 16; do
  DECODE_B=$b timeout -k 10 300 python -u tools/decode_bench.py > $OUT/decode_b$b.log 2>&1; rc=$?; grep "^{" $OUT/decode_b$b.log; [ $rc = 0 ] || exit $rc
done
