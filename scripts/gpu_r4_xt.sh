#!/bin/bash
# Transpose placement of the TN weight gradient: X^T in the forward (+ dY^T first) vs inside wgrad.
# Correctness test, then interleaved headline A/B (3 rounds).
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-xt}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "direct_grad_linear or wgrad" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $OUT/test.log 2>&1; rc=$?; tail -1 $OUT/test.log; fatal $rc
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for arm in "0 0" "1 0" "1 1"; do
    set -- $arm
    GRT_WGRAD_XT_FWD=$1 GRT_WGRAD_DYT_FIRST=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/b_$1$2_$r.log 2>&1; rc=$?
    echo "xt=$1 dyt=$2 r$r $(tail -1 $OUT/b_$1$2_$r.log | grep -o '"value": [0-9.]*, [^,]*, [^,]*, [^,]*, [^,]*, "ms_per_step": [0-9.]*' | sed 's/"unit.*warmup": [0-9]*,//') $(tail -1 $OUT/b_$1$2_$r.log | grep -o '"hbm_peak_gib": [0-9.]*')"
    fatal $rc; [ $rc -eq 0 ] || exit $rc
  done
done
echo done
