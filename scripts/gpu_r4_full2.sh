#!/bin/bash
# full GPU suite twice: the 4-wave dK/dV kernel forced (GRT_ATTN_DKDV=1), then the default
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4full2; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
GRT_ATTN_DKDV=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_form1.log 2>&1; rc=$?
echo "form1:"; grep -E "^FAILED|^ERROR" $OUT/tests_form1.log | head -10; tail -1 $OUT/tests_form1.log; fatal $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_form2.log 2>&1; rc=$?
echo "form2:"; grep -E "^FAILED|^ERROR" $OUT/tests_form2.log | head -10; tail -1 $OUT/tests_form2.log; fatal $rc
echo done
