# block-diagonal LoRA op: GPU numerics + LoRA/QLoRA bench (compare with profiles/r1_transposed_dgrad_ab.txt)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_jobs.py -q -rf -x -k "lora" --timeout 200 --timeout-method thread > gpurun_out/lora_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/lora_tests.log; exit 1; }
tail -2 gpurun_out/lora_tests.log
for mode in "--peft lora" "--peft qlora" "--peft lora"; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 3 $mode > gpurun_out/lora_b.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/lora_b.log; exit 1; }
  echo "[$mode] $(tail -1 gpurun_out/lora_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
