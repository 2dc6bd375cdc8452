# full GPU suite + bench modes (incl. FSDP+offload) + rocprof of the headline
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/s5_gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/s5_gpu_tests.log; exit 1; }
tail -2 gpurun_out/s5_gpu_tests.log
rm -f gpurun_out/s5_bench.jsonl
for mode in "" "--parallel fsdp --offload"; do
  timeout -k 10 600 python bench.py --steps 6 --warmup 2 $mode > gpurun_out/s5_bench.log 2>&1 || { echo "bench $mode failed"; tail -20 gpurun_out/s5_bench.log; exit 1; }
  tail -1 gpurun_out/s5_bench.log >> gpurun_out/s5_bench.jsonl; tail -1 gpurun_out/s5_bench.log | cut -c1-200
done
bash tools/gpu_prof.sh gpurun_out/prof6 --steps 3 --warmup 1
