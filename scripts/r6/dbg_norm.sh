O=gpurun_out/r6dbg; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest "tests/test_parallel_gpu.py::test_ddp_early_grad_norm_matches_full_norm" -x -q --timeout 120 --timeout-method thread > $O/alone.log 2>&1; echo "alone rc=$?"; tail -3 $O/alone.log
timeout -k 10 600 python3 -u -m pytest tests/test_parallel_gpu.py -x -v --timeout 120 --timeout-method thread > $O/file.log 2>&1; echo "file rc=$?"; grep -E "PASSED|FAILED" $O/file.log | head -40
