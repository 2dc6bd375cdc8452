# FSDP / offload GPU tests + full GPU suite + bench in every mode
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_parallel_gpu.py -q -rf -x > gpurun_out/s4_parallel.log 2>&1 || { echo "parallel rc=$?"; tail -30 gpurun_out/s4_parallel.log; exit 1; }
tail -2 gpurun_out/s4_parallel.log
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/s4_gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/s4_gpu_tests.log; exit 1; }
tail -2 gpurun_out/s4_gpu_tests.log
for mode in "--parallel ddp" "--parallel fsdp" "--peft lora" "--peft qlora"; do
  timeout -k 10 420 python bench.py --steps 5 --warmup 2 $mode > gpurun_out/s4_bench.log 2>&1 || { echo "bench $mode failed"; tail -20 gpurun_out/s4_bench.log; exit 1; }
  tail -1 gpurun_out/s4_bench.log | tee -a gpurun_out/s4_bench_all.jsonl
done
