export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -rf -x > gpurun_out/s3_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/s3_gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/s3_bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/s3_bench.log
