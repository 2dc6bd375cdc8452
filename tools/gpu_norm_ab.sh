export TMPDIR=/tmp
mkdir -p gpurun_out
for nb in 256 512 1024 2048; do
  GRT_NORM_BWD_BLOCKS=$nb timeout -k 10 120 python tools/microbench.py --what normbwd 2>/dev/null | sed "s/^/nb=$nb /" || { echo "nb $nb failed"; exit 1; }
done
timeout -k 10 300 python -m pytest tests/test_parallel_gpu.py -q -x > gpurun_out/na_par.log 2>&1 || { echo "par tests failed"; tail -30 gpurun_out/na_par.log; exit 1; }
tail -1 gpurun_out/na_par.log
timeout -k 10 600 python bench.py --steps 4 --warmup 2 --parallel fsdp --offload > gpurun_out/na_off.log 2>&1 || { echo "offload bench failed"; tail -20 gpurun_out/na_off.log; exit 1; }
tail -1 gpurun_out/na_off.log | cut -c1-200
