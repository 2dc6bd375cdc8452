# full-depth Llama-3-70B FSDP offload, proxy rank 0 of 8, moments streamed (resident 0): prefetch ring
# 32 vs 48 vs 64 GiB (uploads moved into the backward window), plus resident auto as the reference
O=gpurun_out/r6ring2; mkdir -p $O
for r in 64 32 48; do
  timeout -k 10 300 python3 bench.py --model llama3-70b --parallel fsdp --offload --proxy-world 8 --checkpointing --offload-resident 0 --offload-prefetch-gib $r --steps 3 --warmup 1 --heartbeat 30 > $O/r$r.json 2> $O/r$r.err || { echo "FAIL ring $r"; tail -5 $O/r$r.err; exit 1; }
  echo "resident 0 ring $r GiB: $(python3 -c "import json;d=json.load(open('$O/r$r.json'));print(d['value'], d['ms_per_step'], d['hbm_peak_gib'], d['loss'])")"
done
timeout -k 10 300 python3 bench.py --model llama3-70b --parallel fsdp --offload --proxy-world 8 --checkpointing --steps 3 --warmup 1 --heartbeat 30 > $O/auto.json 2> $O/auto.err || { echo "FAIL auto"; tail -5 $O/auto.err; exit 1; }
echo "resident auto: $(python3 -c "import json;d=json.load(open('$O/auto.json'));print(d['value'], d['ms_per_step'], d['hbm_peak_gib'], d['loss'])")"
