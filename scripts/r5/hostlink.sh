#!/bin/bash
# host-link engines and rates (tools/hostlink_bench.py), plain and under a kernel + memory-copy trace
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5hostlink}; rm -rf $OUT; mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 tools/hostlink_bench.py > $OUT/plain.log 2>&1; rc=$?; tail -1 $OUT/plain.log; [ $rc = 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof -o hl -- python3 $GRAFT_REPO_ROOT/tools/hostlink_bench.py > $OUT/traced.log 2>&1; rc=$?
tail -1 $OUT/traced.log; [ $rc = 0 ] || exit $rc
for k in kernel_stats memory_copy_stats; do f=$(find $OUT/prof -name "*${k}.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/$k.csv && echo "== $k" && head -8 $OUT/$k.csv | cut -c1-220; done
f=$(find $OUT/prof -name "*memory_copy_trace.csv" | head -1); [ -n "$f" ] && head -3 "$f" | cut -c1-400
rm -rf $OUT/prof
