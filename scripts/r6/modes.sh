# round-6 tree: the other bench modes (LoRA, QLoRA, FSDP world 1, BasicLLM job config) on one box
O=gpurun_out/r6modes; mkdir -p $O
for m in "lora:--peft lora" "qlora:--peft qlora" "fsdp:--parallel fsdp" "head:"; do
  n=${m%%:*}; args=${m#*:}
  timeout -k 10 400 python3 bench.py $args --steps 10 --warmup 3 > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -5 $O/$n.err; exit 1; }
  echo "$n: $(python3 -c "import json;d=json.load(open('$O/$n.json'));print(d['value'], d['ms_per_step'], d.get('mfu_bf16_dense'))")"
done
