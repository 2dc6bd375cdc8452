# single-pass RoPE / SwiGLU kernels: bitwise tests vs the grid-stride kernels, LoRA / QLoRA / headline A/B
O=gpurun_out/r6ew; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q -k "rope or swiglu" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for f in 1 0; do
    for m in "lora:--peft lora" "qlora:--peft qlora"; do
      n=${m%%:*}; args=${m#*:}
      GRT_EW_FAST=$f timeout -k 10 300 python3 bench.py $args --steps 20 --warmup 5 > $O/$n$f.$i.json 2> $O/$n$f.$i.err || { tail -5 $O/$n$f.$i.err; exit 1; }
      echo "$n ew_fast=$f round $i: $(python3 -c "import json;d=json.load(open('$O/$n$f.$i.json'));print(d['value'], d['ms_per_step'], d['loss'])")"
    done
  done
done
