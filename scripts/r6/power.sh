# clocks / power during the headline step with and without the optimizer kernels (smi sampling)
O=gpurun_out/r6power; mkdir -p $O
sample() { while true; do rocm-smi --showpower --showclocks --showtemp --json 2>/dev/null | tr -d '\n'; echo; sleep 0.25; done; }
for mode in head noupd; do
  sample > $O/$mode.smi & sp=$!
  if [ $mode = head ]; then timeout -k 10 300 python3 bench.py --steps 60 --warmup 5 > $O/$mode.json 2> $O/$mode.err
  else timeout -k 10 300 python3 tools/no_update_probe.py --steps 60 --warmup 5 > $O/$mode.json 2> $O/$mode.err; fi
  rc=$?; kill $sp; wait $sp 2>/dev/null; [ $rc = 0 ] || exit $rc
done
head -c 1500 $O/head.smi
