# first MI355X session: device check, kernel numerics, 1-GPU bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import torch; print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0).gcnArchName)" > gpurun_out/s1_dev.log 2>&1 || exit $?
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -rf > gpurun_out/s1_kt.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/s1_bench.log 2>&1
echo "bench rc=$?"
