# FSDP forward-time W^T: GPU tests of the FSDP paths, then the proxy-8 A/B
O=gpurun_out/r6fsdpt; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_parallel_gpu.py tests/test_force_collectives.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for t in auto 0; do
    GRT_FSDP_FWD_TRANSPOSE=$t timeout -k 10 300 python3 bench.py --parallel fsdp --proxy-world 8 --steps 10 --warmup 3 > $O/t$t.$i.json 2>/dev/null || exit 1
    echo "fwd_transpose=$t round $i: $(python3 -c "import json;d=json.load(open('$O/t$t.$i.json'));print(d['ms_per_step'], d['hbm_peak_gib'], d['loss'])")"
  done
done
GRT_FSDP_FWD_TRANSPOSE=auto timeout -k 10 300 python3 bench.py --parallel fsdp --steps 10 --warmup 3 > $O/fsdp1.json 2>/dev/null && echo "fsdp1 (world 1): $(python3 -c "import json;d=json.load(open('$O/fsdp1.json'));print(d['value'], d['ms_per_step'])")"
