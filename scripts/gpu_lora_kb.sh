#!/bin/bash
# LoRA kernel microbench (tools/lora_kernel_bench.py) under launch-time variants, interleaved
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-lorakb}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lora_grad_gpu.py > $OUT/tests.log 2>&1; rc=$?; tail -1 $OUT/tests.log; fatal $rc; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  GRT_LORA_G_NS=4 GRT_LORA_TRED_WPC=1 timeout -k 10 120 python -u tools/lora_kernel_bench.py --tag old > $OUT/old$r.jsonl 2>&1; rc=$?; tail -1 $OUT/old$r.jsonl; fatal $rc
  GRT_LORA_G_NS=3 GRT_LORA_TRED_WPC=2 timeout -k 10 120 python -u tools/lora_kernel_bench.py --tag new > $OUT/new$r.jsonl 2>&1; rc=$?; tail -1 $OUT/new$r.jsonl; fatal $rc
done
