export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "attention or attn" > gpurun_out/aab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/aab_tests.log; exit 1; }
tail -1 gpurun_out/aab_tests.log
for nq in 1 2 1 2; do
  GRT_ATTN_BWD_NQ=$nq timeout -k 10 120 python tools/microbench.py --what attn 2>/dev/null | grep bwd | sed "s/^/nq=$nq /" || { echo "nq $nq failed"; exit 1; }
done
