#!/bin/bash
# Llama-3-70B proxy-8 FSDP + offload (resident 0, prefetch ring) under rocprofv3 kernel + memory-copy
# trace: where the host-link copies sit relative to the forward / backward kernels
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5offtrace}; rm -rf $OUT; mkdir -p $OUT
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof -o off -- python3 -u $GRAFT_REPO_ROOT/bench.py --model llama3-70b --parallel fsdp --offload --proxy-world 8 --checkpointing --steps 2 --warmup 1 --offload-resident ${RES:-0} --offload-prefetch-gib ${PF:-auto} > $OUT/bench.log 2>&1; rc=$?
tail -1 $OUT/bench.log | cut -c1-300; [ $rc = 0 ] || { echo "rc=$rc"; exit $rc; }
cd $GRAFT_REPO_ROOT && python3 tools/offload_timeline.py $OUT/prof > $OUT/timeline.md 2>&1; cat $OUT/timeline.md | head -60
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv; head -12 $OUT/kernel_stats.csv | cut -c1-160
f=$(find $OUT/prof -name "*memory_copy_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/memory_copy_stats.csv && cat $OUT/memory_copy_stats.csv
rm -rf $OUT/prof  # raw traces exceed what gpurun copies back
