#!/bin/bash
# BASELINE config #5 at per-rank volume on one GPU: Llama-3-70B (80 layers) FSDP full-shard, proxy
# rank 0 of 8, activation checkpointing, AdamW moments offloaded to pinned host memory with
# resident share auto / 0 / 0.5 (0 = every unit's moments stream over the host link each step) and
# the streamed moments' device ring prefetched during the backward (auto) or not (0 GiB)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5off70}; rm -rf $OUT; mkdir -p $OUT
COMMON="--model llama3-70b --parallel fsdp --offload --proxy-world 8 --checkpointing --steps ${STEPS:-3} --warmup 1"
timeout -k 10 120 python bench.py $COMMON --plan-only > $OUT/plan.log 2>&1; rc=$?; tail -1 $OUT/plan.log | cut -c1-900; [ $rc = 0 ] || exit $rc
for cfg in ${CFGS:-auto:auto 0:auto 0:0 0.5:auto}; do
  r=${cfg%%:*}; pf=${cfg##*:}
  timeout -k 10 420 python -u bench.py $COMMON --offload-resident $r --offload-prefetch-gib $pf > $OUT/res_${r}_pf${pf}.log 2>&1; rc=$?
  echo "--- resident $r prefetch $pf"; tail -1 $OUT/res_${r}_pf${pf}.log | cut -c1-1500; [ $rc = 0 ] || exit $rc
done
echo done
