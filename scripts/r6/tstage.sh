# LDS-staged transposed epilogue copies (o^T, dq^T, dk^T, dv^T): attention GPU tests (NaN-filled
# outputs, transposed == row-major^T bit for bit, stale-LDS), isolated A/B, interleaved headline A/B
O=gpurun_out/r6tstage; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_lds_poison_gpu.py -x -q -k "attn or attention or dkdv or transposed" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 tools/attn_dma_ab.py --flag tstage --rounds 7 --iters 10 > $O/ab.jsonl 2> $O/ab.err || { cat $O/ab.jsonl; tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
for i in 1 2 3; do
  for f in 1 0; do
    GRT_ATTN_TSTAGE=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/b$f.$i.json 2> $O/b$f.$i.err || exit 1
    echo "tstage=$f round $i: $(python3 -c "import json;d=json.load(open('$O/b$f.$i.json'));print(d['value'], d['ms_per_step'], d['loss'])")"
  done
done
