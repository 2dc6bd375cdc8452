# Round-2 state check after a container restore: GPU suite, smoke(), the driver's bench, kernel profile
export TMPDIR=/tmp
O=gpurun_out/r2chk
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
bash tools/gpu_prof_bench.sh r2chk
