#!/bin/bash
# Session-3 end state on one MI355X: full GPU suite, smoke, headline + LoRA bench, headline kernel
# profile, the reference SFT job end to end (padded default).
set -o pipefail
O=gpurun_out/${1:-r3s3f}
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_head.log 2>&1 || { tail -20 $O/bench_head.log; exit 1; }
echo "bench: $(tail -1 $O/bench_head.log | cut -c1-200)"
timeout -k 10 300 python bench.py --peft lora > $O/bench_lora.log 2>&1 || { tail -20 $O/bench_lora.log; exit 1; }
echo "bench lora: $(tail -1 $O/bench_lora.log | cut -c1-200)"
bash scripts/gpu_sft_job_trace.sh ${1:-r3s3f}/sft || exit $?
bash scripts/gpu_prof.sh $O/prof_headline --steps 6 --warmup 3 || exit $?
