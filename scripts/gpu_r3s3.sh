#!/bin/bash
# Session-3 state check on one MI355X, most important first: headline bench, padding-free step cost
# by token count (tools/varlen_probe.py), GPU suite + smoke, LoRA bench, headline kernel profile.
set -o pipefail
O=gpurun_out/${1:-r3s3}
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_head.log 2>&1 || { tail -20 $O/bench_head.log; exit 1; }
echo "bench: $(tail -1 $O/bench_head.log | cut -c1-200)"
timeout -k 10 400 python -u tools/varlen_probe.py > $O/varlen_probe.jsonl 2> $O/varlen_probe.err || { tail -20 $O/varlen_probe.err; exit 1; }
cat $O/varlen_probe.jsonl
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --peft lora > $O/bench_lora.log 2>&1 || { tail -20 $O/bench_lora.log; exit 1; }
echo "bench lora: $(tail -1 $O/bench_lora.log | cut -c1-200)"
