# device->host GB/s per pinned SDMA engine (tools/d2h_engine_probe.py hsa), then full depth with the chosen one
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6sdmaeng; mkdir -p $O
for e in auto 1 2 3 8 15; do
  GRT_SDMA_TRACE=0 GRT_SDMA_ENGINE=$e timeout -k 10 60 python3 tools/d2h_engine_probe.py hsa > $O/e$e.log 2>&1 || { echo "FAIL engine $e"; tail -3 $O/e$e.log; exit 1; }
  echo "engine $e: $(grep GB/s $O/e$e.log)"
done
