O=gpurun_out/r6lds; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_lds_poison_gpu.py -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|^E " $O/pytest.log | head -30; exit $rc
