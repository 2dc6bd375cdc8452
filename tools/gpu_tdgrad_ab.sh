# transposed-weight dX GEMMs: kernel tests + A/B on the headline, LoRA and QLoRA benches
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_peft.py -q -rf -x -k "transpose or dgrad or nf4 or lora or qlora" --timeout 200 --timeout-method thread > gpurun_out/td_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/td_tests.log; exit 1; }
tail -2 gpurun_out/td_tests.log
rm -f gpurun_out/td_ab.txt
for mode in "" "--peft lora" "--peft qlora"; do
for f in 0 1; do
  GRT_TRANSPOSED_DGRAD=$f timeout -k 10 400 python bench.py --steps 8 --warmup 3 $mode > gpurun_out/td_b.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/td_b.log; exit 1; }
  echo "[$mode] tdgrad=$f $(tail -1 gpurun_out/td_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/td_ab.txt
done
done
