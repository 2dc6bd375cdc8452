# FSDP (config #3) per-rank step: record the library GEMM shapes the table misses, tune them, A/B
export TMPDIR=/tmp
O=gpurun_out/r6fsdp; mkdir -p $O
GRT_TUNED_GEMM_RECORD_UNTUNED=$O/untuned.csv timeout -k 10 300 python3 bench.py --parallel fsdp --proxy-world 8 --steps 6 --warmup 2 > $O/rec.json 2> $O/rec.err || exit 1
echo "record run: $(python3 -c "import json;d=json.load(open('$O/rec.json'));print(d['value'], d['ms_per_step'])")"
ls -la $O
timeout -k 10 900 python3 tools/tune_untuned.py "$O/untuned.csv*" --out $O/tuned.csv > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -5 $O/tune.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --parallel fsdp --proxy-world 8 --steps 10 --warmup 3 > $O/base$i.json 2>/dev/null || exit 1
  GRT_TUNED_GEMM_FILE=$O/tuned.csv timeout -k 10 300 python3 bench.py --parallel fsdp --proxy-world 8 --steps 10 --warmup 3 > $O/new$i.json 2>/dev/null || exit 1
  echo "round $i: base $(python3 -c "import json;d=json.load(open('$O/base$i.json'));print(d['ms_per_step'])") new $(python3 -c "import json;d=json.load(open('$O/new$i.json'));print(d['ms_per_step'])")"
done
