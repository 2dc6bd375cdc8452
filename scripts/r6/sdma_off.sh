# full-depth Llama-3-70B FSDP offload (proxy rank 0 of 8, moments streamed, 32 GiB prefetch ring):
# blit vs SDMA moment write-backs, interleaved
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6sdma; mkdir -p $O
for i in 1 2; do
  for eng in sdma blit; do
    GRT_OFFLOAD_D2H=$eng timeout -k 10 300 python3 bench.py --model llama3-70b --parallel fsdp --offload --proxy-world 8 --checkpointing --offload-resident 0 --offload-prefetch-gib 32 --steps 3 --warmup 1 --heartbeat 30 > $O/off_$eng.$i.json 2> $O/off_$eng.$i.err || { echo "FAIL offload $eng"; tail -20 $O/off_$eng.$i.err; exit 1; }
    echo "offload resident 0, d2h=$eng round $i: $(python3 -c "import json;d=json.load(open('$O/off_$eng.$i.json'));print(d['value'], d['ms_per_step'], d['loss'])")"
  done
done
