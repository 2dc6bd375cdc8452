export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k embedding > gpurun_out/emb_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/emb_tests.log; exit 1; }
tail -1 gpurun_out/emb_tests.log
for e in 0 1 0 1; do
  GRT_NATIVE_EMBEDDING=$e timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/emb_b.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/emb_b.log; exit 1; }
  tail -1 gpurun_out/emb_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('native_emb=$e', d['value'], d['ms_per_step'])"
done
