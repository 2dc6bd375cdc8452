export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -k "attention or rope or llama" > gpurun_out/attn_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/attn_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/microbench.py --what attn > gpurun_out/attn_micro.log 2>&1; echo "micro rc=$?"
grep -v amdgpu gpurun_out/attn_micro.log
