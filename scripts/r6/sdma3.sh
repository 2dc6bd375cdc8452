# SDMA copier with bounded producer polling and fail-fast: SDMA tests, stress loop, suite with SDMA x2
O=gpurun_out/r6sdma5; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_sdma_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
sed -i 's#gpurun_out/r6sdmastress#gpurun_out/r6sdma5/stress#' scripts/r6/sdma_stress.sh
bash scripts/r6/sdma_stress.sh || exit 1
for i in 1 2; do
  GRT_OFFLOAD_D2H=sdma timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/suite$i.log 2>&1 || { grep -E "FAILED|Timeout" $O/suite$i.log | head -5; tail -3 $O/suite$i.log; exit 1; }
  tail -1 $O/suite$i.log
done
