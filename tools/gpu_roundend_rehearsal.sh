# rehearsal of the driver's round-end GPU tiers: full GPU suite, smoke(), default bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/re_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/re_tests.log; exit 1; }
tail -2 gpurun_out/re_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/re_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/re_smoke.log; exit 1; }
tail -1 gpurun_out/re_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/re_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/re_bench.log; exit 1; }
tail -1 gpurun_out/re_bench.log
