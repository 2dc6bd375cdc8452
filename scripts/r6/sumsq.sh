# Grad-norm partial sums with 4 loads in flight per lane: float64 test, isolated timing, interleaved headline A/B
O=gpurun_out/r6sumsq; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q -k "sumsq or adamw_and_clip" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for u in 1 0 1 0; do
  GRT_SUMSQ_UNROLL=$u PYTHONPATH=. timeout -k 10 120 python3 tools/sumsq_ab.py >> $O/time.log 2>&1 || { cat $O/time.log; exit 1; }
done
cat $O/time.log
for i in 1 2 3; do
  for u in 1 0; do
    GRT_SUMSQ_UNROLL=$u timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/b$u.$i.json 2> $O/b$u.$i.err || exit 1
    echo "sumsq_unroll=$u round $i: $(python3 -c "import json;d=json.load(open('$O/b$u.$i.json'));print(d['value'], d['ms_per_step'], d['loss'])")"
  done
done
