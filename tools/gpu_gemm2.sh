export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -rf -x -k "gemm or wgrad" > gpurun_out/g_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/g_tests.log; exit 1; }
tail -2 gpurun_out/g_tests.log
timeout -k 10 300 env GRT_GEMM_DIAG=1 python tools/microbench.py --what gemm > gpurun_out/g_micro.jsonl 2>&1 || { echo "micro failed"; tail -20 gpurun_out/g_micro.jsonl; exit 1; }
grep wgrad gpurun_out/g_micro.jsonl
