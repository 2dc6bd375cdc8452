# overlapped optimizer: GPU equivalence test + bench A/B (serial vs overlapped), interleaved
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parallel_gpu.py -x -q -k overlapped --timeout 200 --timeout-method thread > gpurun_out/ovl_test.log 2>&1 || { echo "test failed"; tail -30 gpurun_out/ovl_test.log; exit 1; }
tail -2 gpurun_out/ovl_test.log
rm -f gpurun_out/ovl_ab.txt
for i in 1 2; do
for m in off on; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 3 --overlap-opt $m > gpurun_out/ovl_b.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/ovl_b.log; exit 1; }
  echo "$m $(tail -1 gpurun_out/ovl_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ovl_ab.txt
done
done
