# does the autograd thread now use the tuned dX GEMMs? probe trace + headline bench
export TMPDIR=/tmp
mkdir -p gpurun_out/pi2
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pi2 -o run -- python3 $GRAFT_REPO_ROOT/tools/gemm_insitu_probe.py > $GRAFT_REPO_ROOT/gpurun_out/pi2/log.txt 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/prof_names.py gpurun_out/pi2 | tail -24
for i in 1 2; do
timeout -k 10 400 python bench.py --steps 8 --warmup 3 > gpurun_out/tb.log 2>&1 || { tail -20 gpurun_out/tb.log; exit 1; }
tail -1 gpurun_out/tb.log | cut -c1-200
done
