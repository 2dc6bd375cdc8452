#!/bin/bash
# LDS-DMA lora_down: GPU tests, then the LoRA kernel microbench with it off / on, then the LoRA bench
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-lorakb3}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lora or kcat" > $OUT/tests.log 2>&1; rc=$?
grep -E "FAIL|Error" $OUT/tests.log | head -5; tail -1 $OUT/tests.log; fatal $rc; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for d in 0 1; do
    GRT_LORA_DOWN_DMA=$d timeout -k 10 120 python -u tools/lora_kernel_bench.py --tag dma$d > $OUT/dma$d.$r.jsonl 2>&1; rc=$?; fatal $rc
    grep '"kernel": "lora_down"' $OUT/dma$d.$r.jsonl | python3 -c "import sys,json; print('dma$d', [(json.loads(l)['module'], json.loads(l)['us']) for l in sys.stdin])"
  done
done
for d in 0 1; do
  GRT_LORA_DOWN_DMA=$d timeout -k 10 300 python bench.py --peft qlora --steps 10 --warmup 3 > $OUT/bench_q$d.log 2>&1; rc=$?; echo "dma$d $(tail -1 $OUT/bench_q$d.log | cut -c1-140)"; fatal $rc
done
