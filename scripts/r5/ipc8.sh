cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5ipc8
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ipc_gpu.py -s > gpurun_out/r5ipc8/tests.log 2>&1; rc=$?; grep -E "passed|failed|world" gpurun_out/r5ipc8/tests.log | tail -12; exit $rc
