O=gpurun_out/r6suite; mkdir -p $O
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "^E " $O/pytest.log | head -8; tail -3 $O/pytest.log; exit $rc
