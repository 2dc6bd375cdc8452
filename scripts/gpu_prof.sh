# kernel-time profile of the 1-GPU headline bench (rocprofv3 kernel trace + stats only)
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
shift
mkdir -p $OUT
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $GRAFT_REPO_ROOT/$OUT/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"
cd $GRAFT_REPO_ROOT && find $OUT -name "*stats*.csv" | head
exit $rc
