# SDMA copier v2 (worker polls a stream-written ready word; no HIP call on the worker): SDMA tests,
# the full GPU suite with SDMA write-backs for every offload test, the stress loop, full-depth 70B A/B
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6sdma2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_sdma_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
GRT_OFFLOAD_D2H=sdma timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { grep -E "FAILED|Error" $O/suite.log | head; tail -5 $O/suite.log; exit 1; }
tail -1 $O/suite.log
sed -i 's#gpurun_out/r6sdmastress#gpurun_out/r6sdma2/stress#' scripts/r6/sdma_stress.sh
bash scripts/r6/sdma_stress.sh || exit 1
sed -i 's#O=$R/gpurun_out/r6sdma;#O=$R/gpurun_out/r6sdma2;#' scripts/r6/sdma_off.sh
bash scripts/r6/sdma_off.sh
