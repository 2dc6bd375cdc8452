export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_gpu_jobs.py -q -rf -x > gpurun_out/lo_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/lo_tests.log; exit 1; }
tail -1 gpurun_out/lo_tests.log
for mode in "--peft lora" "--peft qlora"; do
  timeout -k 10 500 python bench.py --steps 6 --warmup 2 $mode > gpurun_out/lo_b.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/lo_b.log; exit 1; }
  tail -1 gpurun_out/lo_b.log | cut -c1-200
done
