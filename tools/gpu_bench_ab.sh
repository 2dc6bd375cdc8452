export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -rf -x > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for i in 1 2; do
timeout -k 10 400 env GRT_WGRAD_GEMM=0 python bench.py --steps 8 --warmup 2 > gpurun_out/ab_b0.log 2>&1 || { echo "bench0 failed"; tail -20 gpurun_out/ab_b0.log; exit 1; }
tail -1 gpurun_out/ab_b0.log | cut -c1-190
timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/ab_b1.log 2>&1 || { echo "bench1 failed"; tail -20 gpurun_out/ab_b1.log; exit 1; }
tail -1 gpurun_out/ab_b1.log | cut -c1-190
done
