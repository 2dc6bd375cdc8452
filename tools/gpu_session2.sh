export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/microbench.py > gpurun_out/s2_micro.log 2>&1 || exit $?
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv timeout -k 10 900 python tools/microbench.py --what gemm > gpurun_out/s2_micro_tuned.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/s2_bench.log 2>&1
echo "bench rc=$?"
