# attention forward variants: numerics (env-selected variant) + microbench
export TMPDIR=/tmp
mkdir -p gpurun_out
for nw in 4 8; do
  GRT_ATTN_FWD_WAVES=$nw timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "flash_attention or rope_attention" --timeout 200 --timeout-method thread > gpurun_out/attn_nw$nw.log 2>&1 || { echo "nw=$nw tests failed"; tail -30 gpurun_out/attn_nw$nw.log; exit 1; }
  echo "nw=$nw $(tail -1 gpurun_out/attn_nw$nw.log)"
  GRT_ATTN_FWD_WAVES=$nw timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn_b$nw.jsonl 2>&1 || { tail -5 gpurun_out/attn_b$nw.jsonl; exit 1; }
  grep llama2 gpurun_out/attn_b$nw.jsonl
done
