# full GPU suite with SDMA write-backs in every offload test (stall hunt), verbose, per-copy trace off
O=gpurun_out/r6suitesdma; mkdir -p $O
GRT_OFFLOAD_D2H=sdma timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|Timeout" $O/pytest.log | head -5; tail -2 $O/pytest.log; exit $rc
