# 2 ranks sharing the one GPU over gloo: engine tests + bench rehearsal (DDP+ZeRO, FSDP)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_parallel_gpu_multiproc.py -q -rf -x > gpurun_out/mp_tests.log 2>&1 || { echo "mp tests failed rc=$?"; tail -40 gpurun_out/mp_tests.log; exit 1; }
tail -2 gpurun_out/mp_tests.log
for par in ddp fsdp; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --model llama-125m --batch 4 --seq 512 --steps 3 --warmup 1 --parallel $par > gpurun_out/mp_bench_$par.log 2>&1 || { echo "bench $par failed"; tail -30 gpurun_out/mp_bench_$par.log; exit 1; }
grep metric gpurun_out/mp_bench_$par.log | cut -c1-200
done
timeout -k 10 400 python bench.py --steps 6 --warmup 2 > gpurun_out/mp_bench1.log 2>&1 || { echo "bench 1gpu failed"; tail -30 gpurun_out/mp_bench1.log; exit 1; }
tail -1 gpurun_out/mp_bench1.log | cut -c1-200
