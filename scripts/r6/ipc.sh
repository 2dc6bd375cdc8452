# IPC fail-stop + self-test GPU tests
OUT=gpurun_out/r6ipc; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ipc_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -30 $OUT/pytest.log; exit $rc
