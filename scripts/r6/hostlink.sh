# host link: torch copy_ vs copy_sdma (hipMemcpyDeviceToDeviceNoCU), plus an engine trace
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6host; mkdir -p $O
timeout -k 10 200 python3 $R/tools/hostlink_bench.py --mib 512 --reps 4 > $O/bench.json 2> $O/bench.err && \
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o run -- \
   python3 $R/tools/hostlink_bench.py --mib 256 --reps 2 > $O/trace.log 2>&1)
rc=$?; cat $O/bench.json; find $O/trace -name "*stats*.csv" | xargs -r head -20; exit $rc
