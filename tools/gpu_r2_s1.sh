# round-2 first GPU session: GPU test tier, 1-GPU headline bench, kernel-time profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2s1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  && echo "pytest ok" \
  && timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 \
  && tail -1 $O/bench.log \
  && cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof_bench.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
tail -3 $O/pytest.log
echo "rc=$rc"
exit $rc
