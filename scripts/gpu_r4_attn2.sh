#!/bin/bash
# attention A/B after a build change (no SLP vectorizer in attention.hip): forms 1 / 2 + forward
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4attn2; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "dkdv or flash_attention_production or rope_attention" > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; fatal $rc; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/attn_dkdv_ab.py > $OUT/ab.log 2>&1; rc=$?; grep '^{' $OUT/ab.log; fatal $rc
timeout -k 10 300 python -u tools/attn_ab.py --rounds 5 > $OUT/attn_ab.log 2>&1; rc=$?; grep '^{' $OUT/attn_ab.log; fatal $rc
echo done
