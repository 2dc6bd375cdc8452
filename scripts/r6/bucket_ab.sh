# 1 GPU: early grad-norm granularity (bucket size) A/B — smaller buckets read their gradients while hot in the Infinity Cache
O=gpurun_out/r6bucket; mkdir -p $O
for i in 1 2; do
  for mb in 256 64 32; do
    GRT_BUCKET_MB=$mb timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/b$mb.$i.json 2> $O/b$mb.$i.err || exit 1
    echo "bucket=$mb round $i: $(python3 -c "import json;d=json.load(open('$O/b$mb.$i.json'));print(d['value'], d['ms_per_step'])")"
  done
done
