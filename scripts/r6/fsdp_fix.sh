# FSDP forward-transpose budget on full weight sizes: FSDP GPU tests, then 70B offload memory / speed
O=gpurun_out/r6fsdpfix; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_parallel_gpu.py -x -q -k "fsdp" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in auto 0; do
  timeout -k 10 300 python3 bench.py --model llama3-70b --parallel fsdp --offload --proxy-world 8 --checkpointing --offload-resident $r --offload-prefetch-gib 32 --steps 3 --warmup 1 --heartbeat 30 > $O/r$r.json 2> $O/r$r.err || { echo "FAIL $r"; tail -5 $O/r$r.err; exit 1; }
  echo "resident $r ring 32: $(python3 -c "import json;d=json.load(open('$O/r$r.json'));print(d['value'], d['ms_per_step'], d['hbm_plan_gib'], d['hbm_peak_gib'], d['loss'])")"
done
timeout -k 10 300 python3 bench.py --parallel fsdp --proxy-world 8 --steps 10 --warmup 3 > $O/fsdp7.json 2>/dev/null && echo "fsdp proxy-8 7B: $(python3 -c "import json;d=json.load(open('$O/fsdp7.json'));print(d['value'], d['ms_per_step'], d['hbm_peak_gib'])")"
