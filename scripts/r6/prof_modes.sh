# rocprofv3 kernel tables of the per-rank 8-GPU steps (ZeRO proxy-8, FSDP proxy-8) + the headline
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {  # name, bench args...
  n=$1; shift; mkdir -p $R/gpurun_out/r6prof2/$n
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6prof2/$n -o run -- \
      python3 $R/bench.py --steps 6 --warmup 3 "$@" > $R/gpurun_out/r6prof2/$n/bench.log 2>&1) || return 1
  f=$(find $R/gpurun_out/r6prof2/$n -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/prof_steps.py $f 9 > $R/gpurun_out/r6prof2/$n/steps.md 2>&1
  tail -1 $R/gpurun_out/r6prof2/$n/bench.log
}
run zero8 --proxy-world 8 && run fsdp8 --parallel fsdp --proxy-world 8 && run head
rc=$?
find $R/gpurun_out/r6prof2 -name "*.csv" -size +20M -delete
exit $rc
