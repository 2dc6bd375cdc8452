O=gpurun_out/r6fsdpab; mkdir -p $O
for i in 1 2; do
  for z in 0 1; do
    GRT_FSDP_ZERO_FULL_GRAD=$z timeout -k 10 300 python3 bench.py --parallel fsdp --proxy-world 8 --steps 10 --warmup 3 > $O/z$z.$i.json 2>/dev/null || exit 1
    echo "zero_full=$z round $i: $(python3 -c "import json;d=json.load(open('$O/z$z.$i.json'));print(d['ms_per_step'])")"
  done
done
