# Grad-norm partial sums with U = 4 / 2 / 1 loads in flight per lane (GRT_SUMSQ_UNROLL=4|2|0):
# float64 test per U, isolated timing, interleaved headline A/B
O=${O:-gpurun_out/r6sumsq2}; mkdir -p $O
for u in ${US:-4 2 0}; do
  GRT_SUMSQ_UNROLL=$u timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q -k "sumsq or adamw_and_clip" --timeout 200 --timeout-method thread > $O/tests$u.log 2>&1 || { tail -30 $O/tests$u.log; exit 1; }
  echo "U=$u: $(tail -1 $O/tests$u.log)"
done
for u in ${US:-4 2 0} ${US:-4 2 0}; do
  GRT_SUMSQ_UNROLL=$u PYTHONPATH=. timeout -k 10 120 python3 tools/sumsq_ab.py >> $O/time.log 2>&1 || { cat $O/time.log; exit 1; }
done
grep unroll $O/time.log
for i in 1 2 3; do
  for u in ${US:-4 2 0}; do
    GRT_SUMSQ_UNROLL=$u timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/b$u.$i.json 2> $O/b$u.$i.err || exit 1
    echo "sumsq_unroll=$u round $i: $(python3 -c "import json;d=json.load(open('$O/b$u.$i.json'));print(d['value'], d['ms_per_step'], d['loss'])")"
  done
done
