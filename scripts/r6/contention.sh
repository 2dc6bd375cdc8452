# price of the overlapped AdamW beside the forward: headline vs the same step without update kernels
O=gpurun_out/r6cont; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/head$i.json 2> $O/head$i.err || exit 1
  timeout -k 10 300 python3 tools/no_update_probe.py --steps 20 --warmup 5 > $O/noupd$i.json 2> $O/noupd$i.err || exit 1
  echo "round $i: head $(python3 -c "import json;d=json.load(open('$O/head$i.json'));print(d['ms_per_step'])") ms, no-update $(python3 -c "import json;d=json.load(open('$O/noupd$i.json'));print(d['ms_per_step'])") ms"
done
