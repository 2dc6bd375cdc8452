# round-6 end state on one box: full GPU suite + smoke, headline bench x2, rocprofv3 step table
O=gpurun_out/r6final8; mkdir -p $O
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py > $O/bench$i.json 2> $O/bench$i.err || exit 1
  cat $O/bench$i.json
done
bash scripts/gpu_prof.sh $O/prof --steps 6 --warmup 3 || exit 1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/prof_steps.py $f 9 > $O/steps.md 2>&1; head -40 $O/steps.md
find $O/prof -name "*.csv" -size +20M -delete
