O=gpurun_out/r6bisect; mkdir -p $O
T="tests/test_parallel_gpu.py::test_ddp_early_grad_norm_matches_full_norm"
for f in tests/test_force_collectives.py tests/test_optim_state.py "tests/test_force_collectives.py tests/test_optim_state.py"; do
  n=$(echo $f | tr ' /' '__')
  timeout -k 10 400 python3 -u -m pytest $f $T -q -m gpu --timeout 200 --timeout-method thread > $O/$n.log 2>&1
  echo "$f -> rc=$? $(tail -1 $O/$n.log)"; grep -E "^E .*non-finite|^E  " $O/$n.log | head -3
done
