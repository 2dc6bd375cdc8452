# ZeRO proxy-8: forward-time W^T transposes (TN dX GEMMs) vs NN dX GEMMs, interleaved
O=gpurun_out/r6zerot; mkdir -p $O
for i in 1 2; do
  for f in 1 0; do
    GRT_ZERO_FWD_TRANSPOSE=$f timeout -k 10 300 python3 bench.py --proxy-world 8 --steps 20 --warmup 5 > $O/z$f.$i.json 2> $O/z$f.$i.err || exit 1
    echo "zero_fwd_transpose=$f round $i: $(python3 -c "import json;d=json.load(open('$O/z$f.$i.json'));print(d['value'], d['ms_per_step'], d['loss'])")"
  done
done
