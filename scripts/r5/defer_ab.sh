#!/bin/bash
# A/B on one box: owned-slot write-backs deferred to the forward tail (1) or issued at step() (0)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5defer}; rm -rf $OUT; mkdir -p $OUT
COMMON="--model llama3-70b --parallel fsdp --offload --proxy-world 8 --checkpointing --steps 3 --warmup 1 --offload-prefetch-gib auto"
for r in 0 0.5; do
  for d in 0 1; do
    GRT_OFFLOAD_DEFER_WRITEBACK=$d timeout -k 10 420 python -u bench.py $COMMON --offload-resident $r > $OUT/res${r}_defer$d.log 2>&1; rc=$?
    echo "resident $r defer $d: $(tail -1 $OUT/res${r}_defer$d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"])')"; [ $rc = 0 ] || exit $rc
  done
done
timeout -k 10 200 python3 tools/hostlink_bench.py > $OUT/hostlink.log 2>&1; tail -1 $OUT/hostlink.log
