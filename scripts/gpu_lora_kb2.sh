#!/bin/bash
# lora_down with A chunks one vs two ahead (GRT_LORA_DOWN_AD), interleaved microbench
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-lorakb2}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
GRT_LORA_DOWN_AD=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lora" > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log; fatal $rc; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for ad in 1 2; do
    GRT_LORA_DOWN_AD=$ad timeout -k 10 120 python -u tools/lora_kernel_bench.py --tag ad$ad > $OUT/ad$ad.$r.jsonl 2>&1; rc=$?; fatal $rc
    grep lora_down $OUT/ad$ad.$r.jsonl | python3 -c "import sys,json; print('ad$ad', [(json.loads(l)['module'], json.loads(l)['us']) for l in sys.stdin])"
  done
done
