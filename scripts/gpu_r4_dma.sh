#!/bin/bash
# Hoisted LDS-DMA addressing in the attention kernels: attention GPU tests, then the in-process A/B
# (bitwise equality + timing), then the headline bench.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4dma}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_varlen.py -m gpu -q -k "attn or attention or varlen or flash or dkdv or rope" \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/test.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR" $OUT/test.log | head; tail -1 $OUT/test.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/attn_dma_ab.py > $OUT/ab.jsonl 2>&1; rc=$?; cat $OUT/ab.jsonl | cut -c1-400; fatal $rc
[ $rc -eq 0 ] || exit $rc
for m in 1 0 1 0; do
  GRT_ATTN_DMA_FAST=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_$m.log 2>&1; rc=$?
  echo "dma_fast=$m $(tail -1 $OUT/bench_$m.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"; fatal $rc
done
echo done
