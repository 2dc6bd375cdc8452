export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -rf -x -k "gemm or wgrad" > gpurun_out/g_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/g_tests.log; exit 1; }
tail -1 gpurun_out/g_tests.log
timeout -k 10 400 python tools/gemm_ab.py ${MODES:-1,2,3,4,5,6} > gpurun_out/g_ab.jsonl 2>&1 || { echo "ab failed"; tail -20 gpurun_out/g_ab.jsonl; exit 1; }
cat gpurun_out/g_ab.jsonl
