export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_gpu_jobs.py -q -rf -x > gpurun_out/ad_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/ad_tests.log; exit 1; }
tail -2 gpurun_out/ad_tests.log
timeout -k 10 300 python tools/microbench.py --what attn > gpurun_out/ad_micro.jsonl 2>&1 || { echo "micro failed"; tail -20 gpurun_out/ad_micro.jsonl; exit 1; }
cat gpurun_out/ad_micro.jsonl | grep attn
