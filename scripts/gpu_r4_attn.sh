#!/bin/bash
# Round 4: wave-pair dK / dV kernel: parity tests vs the 4-wave kernel and the fp32 math path, A/B timing.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4attn; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "dkdv or flash_attention or rope_attention" > $OUT/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error" $OUT/tests.log | tail -40; fatal $rc; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/attn_dkdv_ab.py > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log | tail -8; fatal $rc
echo done
