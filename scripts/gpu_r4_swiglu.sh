#!/bin/bash
# Transposing SwiGLU (h^T / dgu^T for the TN weight gradients): tests, then headline A/B.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4swiglu}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "swiglu or direct_grad or wgrad or transposed_dgrad" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $OUT/test.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR|Error|assert" $OUT/test.log | head -20; tail -1 $OUT/test.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 1 0; do
    GRT_SWIGLU_T=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/b_${f}_$r.log 2>&1; rc=$?
    echo "swiglu_t=$f r$r $(tail -1 $OUT/b_${f}_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"hbm_peak_gib": [0-9.]*' | tr '\n' ' ')"; fatal $rc
  done
done
echo done
