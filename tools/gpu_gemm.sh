# wgrad GEMM: numerics, microbench vs hipBLASLt, bench A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -rf -x -k "gemm or wgrad" > gpurun_out/g_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/g_tests.log; exit 1; }
tail -2 gpurun_out/g_tests.log
timeout -k 10 300 python tools/microbench.py --what gemm > gpurun_out/g_micro.jsonl 2>&1 || { echo "micro failed"; tail -20 gpurun_out/g_micro.jsonl; exit 1; }
grep wgrad gpurun_out/g_micro.jsonl
timeout -k 10 400 env GRT_WGRAD_GEMM=0 python bench.py --steps 5 --warmup 2 > gpurun_out/g_bench0.log 2>&1 || { echo "bench0 failed"; tail -20 gpurun_out/g_bench0.log; exit 1; }
tail -1 gpurun_out/g_bench0.log | cut -c1-200
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/g_bench1.log 2>&1 || { echo "bench1 failed"; tail -20 gpurun_out/g_bench1.log; exit 1; }
tail -1 gpurun_out/g_bench1.log | cut -c1-200
