#!/bin/bash
# round-aware lora_g / lora_tred splits vs the former rules: tests, microbench (interleaved), QLoRA bench
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-lorakb5}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lora_grad_gpu.py tests/test_kernels_gpu.py -k "lora or kcat" > $OUT/tests.log 2>&1; rc=$?
tail -1 $OUT/tests.log; fatal $rc; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  GRT_LORA_G_SPLITS=old GRT_LORA_TRED_SPLITS=old timeout -k 10 120 python -u tools/lora_kernel_bench.py --tag old > $OUT/old$r.jsonl 2>&1; rc=$?; tail -1 $OUT/old$r.jsonl; fatal $rc
  timeout -k 10 120 python -u tools/lora_kernel_bench.py --tag new > $OUT/new$r.jsonl 2>&1; rc=$?; tail -1 $OUT/new$r.jsonl; fatal $rc
done
