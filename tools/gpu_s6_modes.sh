# full GPU suite + headline/bench modes + BasicLLM (reference workload #1, fp32) on one MI355X
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/s6m_gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/s6m_gpu_tests.log; exit 1; }
tail -2 gpurun_out/s6m_gpu_tests.log
rm -f gpurun_out/s6m_modes.jsonl
for mode in "" "--parallel fsdp" "--peft lora" "--peft qlora"; do
  timeout -k 10 600 python bench.py --steps 8 --warmup 3 $mode > gpurun_out/s6m_bench.log 2>&1 || { echo "bench $mode failed"; tail -20 gpurun_out/s6m_bench.log; exit 1; }
  tail -1 gpurun_out/s6m_bench.log >> gpurun_out/s6m_modes.jsonl; tail -1 gpurun_out/s6m_bench.log | cut -c1-160
done
timeout -k 10 600 python jobs/pytorch_llm_ray.py --workers 1 --max-windows 3200 --pvc /tmp/grt_pvc > gpurun_out/s6m_basicllm_fp32.log 2>&1 || { echo "basicllm failed"; tail -30 gpurun_out/s6m_basicllm_fp32.log; exit 1; }
grep -i "tokens_per_sec\|metrics" gpurun_out/s6m_basicllm_fp32.log | tail -3
