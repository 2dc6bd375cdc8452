#!/bin/bash
# BASELINE config #5 at per-rank volume on one GPU: Llama-3-70B (80 layers) FSDP full-shard, proxy
# rank 0 of 8, activation checkpointing, AdamW moments offloaded to pinned host memory with
# resident share auto / 0.5 / 0 (0 = every unit's moments stream over the host link each step)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5off70}; rm -rf $OUT; mkdir -p $OUT
COMMON="--model llama3-70b --parallel fsdp --offload --proxy-world 8 --checkpointing --steps ${STEPS:-2} --warmup 1"
timeout -k 10 120 python bench.py $COMMON --plan-only > $OUT/plan.log 2>&1; rc=$?; tail -1 $OUT/plan.log | cut -c1-600; [ $rc = 0 ] || exit $rc
for r in ${RESIDENT:-auto 0 0.5}; do
  timeout -k 10 420 python -u bench.py $COMMON --offload-resident $r > $OUT/res_$r.log 2>&1; rc=$?
  tail -1 $OUT/res_$r.log | cut -c1-400; [ $rc = 0 ] || exit $rc
done
echo done
