# overlapped optimizer at projection granularity: GPU tests + interleaved headline A/B (GRT_OVERLAP_FINE 1 / 0)
O=gpurun_out/r6fine; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_parallel_gpu.py -x -q -k overlapped_optimizer --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for f in 1 0; do
    GRT_OVERLAP_FINE=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/b$f.$i.json 2> $O/b$f.$i.err || exit 1
    echo "fine=$f round $i: $(python3 -c "import json;d=json.load(open('$O/b$f.$i.json'));print(d['value'], d['ms_per_step'], d['loss'])")"
  done
done
