# full GPU test suite + smoke (what the driver runs at round end), then the FSDP gap-clear A/B
O=gpurun_out/r6suite; mkdir -p $O
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/r6/fsdp_ab.sh
