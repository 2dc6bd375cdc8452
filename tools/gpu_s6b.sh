export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parallel_gpu.py -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/s6b_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/s6b_tests.log; exit 1; }
tail -2 gpurun_out/s6b_tests.log
timeout -k 10 600 python bench.py --steps 8 --warmup 3 --peft lora --data pipeline > gpurun_out/s6b_lora_pipe.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/s6b_lora_pipe.log; exit 1; }
tail -1 gpurun_out/s6b_lora_pipe.log | cut -c1-400
timeout -k 10 600 python bench.py --steps 8 --warmup 3 --data pipeline > gpurun_out/s6b_ddp_pipe.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/s6b_ddp_pipe.log; exit 1; }
tail -1 gpurun_out/s6b_ddp_pipe.log | cut -c1-200
