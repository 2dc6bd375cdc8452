export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6d2h; mkdir -p $O
for cfg in "torch" "nocu" "registered" "torch GPU_BLIT_ENGINE_TYPE=1" "torch GPU_BLIT_ENGINE_TYPE=2" "nocu GPU_BLIT_ENGINE_TYPE=2" "torch HSA_ENABLE_SDMA=1 GPU_FORCE_BLIT_COPY_SIZE=0"; do
  set -- $cfg; mode=$1; shift
  tag=$(echo "$cfg" | tr ' =' '__')
  (cd /tmp && env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/$tag -o run -- python3 $R/tools/d2h_engine_probe.py $mode > $O/$tag.log 2>&1) || { echo "FAIL $cfg"; exit 1; }
  echo "== $cfg: $(grep GB/s $O/$tag.log) | blit kernels: $(grep -c copyBuffer $O/$tag/run_kernel_trace.csv 2>/dev/null) | D2H SDMA copies: $(grep -c DEVICE_TO_HOST $O/$tag/run_memory_copy_trace.csv 2>/dev/null)"
done
