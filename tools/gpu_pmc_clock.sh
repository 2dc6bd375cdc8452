# effective shader clock per kernel family: GRBM_GUI_ACTIVE cycles / kernel duration
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc/bench.log 2>&1
rc=$?; echo "rc=$rc"; cd $GRAFT_REPO_ROOT; find gpurun_out/pmc -name "*.csv" | head; exit $rc
