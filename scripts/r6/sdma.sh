# SDMA device->host write-backs: GPU tests, engine probe under the memory-copy trace, then the
# full-depth Llama-3-70B FSDP offload (proxy rank 0 of 8, moments streamed) with blit vs SDMA write-backs
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6sdma; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_sdma_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -8
for mode in hsa torch; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/$mode -o run -- python3 $R/tools/d2h_engine_probe.py $mode > $O/$mode.log 2>&1) || { echo "FAIL probe $mode"; tail -5 $O/$mode.log; exit 1; }
  echo "== $mode: $(grep GB/s $O/$mode.log) | blit kernels: $(grep -c copyBuffer $O/$mode/run_kernel_trace.csv 2>/dev/null) | D2H SDMA copies: $(grep -c DEVICE_TO_HOST $O/$mode/run_memory_copy_trace.csv 2>/dev/null)"
done
for eng in sdma blit; do
  GRT_OFFLOAD_D2H=$eng timeout -k 10 600 python3 bench.py --model llama3-70b --parallel fsdp --offload --proxy-world 8 --checkpointing --offload-resident 0 --offload-prefetch-gib 32 --steps 3 --warmup 1 > $O/off_$eng.json 2> $O/off_$eng.err || { echo "FAIL offload $eng"; tail -20 $O/off_$eng.err; exit 1; }
  echo "offload resident 0, d2h=$eng: $(python3 -c "import json;d=json.load(open('$O/off_$eng.json'));print(d['value'], d['ms_per_step'], d['loss'])")"
done
