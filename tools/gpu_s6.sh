# session 6 sanity: GPU suite + headline bench on the restored tree
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/s6_gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/s6_gpu_tests.log; exit 1; }
tail -2 gpurun_out/s6_gpu_tests.log
timeout -k 10 600 python bench.py --steps 8 --warmup 3 > gpurun_out/s6_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/s6_bench.log; exit 1; }
tail -1 gpurun_out/s6_bench.log
