# full-depth 70B, moments streamed, 64 GiB ring: blit vs SDMA write-backs, interleaved (after the FSDP budget fix)
O=gpurun_out/r6sdma64; mkdir -p $O
for i in 1 2; do
  for eng in sdma blit; do
    GRT_OFFLOAD_D2H=$eng timeout -k 10 300 python3 bench.py --model llama3-70b --parallel fsdp --offload --proxy-world 8 --checkpointing --offload-resident 0 --offload-prefetch-gib 64 --steps 3 --warmup 1 --heartbeat 30 > $O/$eng.$i.json 2> $O/$eng.$i.err || { echo "FAIL $eng"; tail -5 $O/$eng.$i.err; exit 1; }
    echo "ring 64, d2h=$eng round $i: $(python3 -c "import json;d=json.load(open('$O/$eng.$i.json'));print(d['value'], d['ms_per_step'], d['hbm_peak_gib'], d['loss'])")"
  done
done
