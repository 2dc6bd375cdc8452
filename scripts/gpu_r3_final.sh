#!/bin/bash
# Round-end state check on one MI355X: full GPU suite, smoke, headline + LoRA bench, rocprofv3
# kernel tables of both bench steps, and the reference SFT job end to end.
set -o pipefail
O=gpurun_out/${1:-r3final}
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for mode in "" "--peft lora"; do
  timeout -k 10 300 python bench.py $mode > $O/bench_${mode:7:4}.log 2>&1 || exit $?
  echo "bench $mode: $(tail -1 $O/bench_${mode:7:4}.log | cut -c1-170)"
done
bash scripts/gpu_prof.sh $O/prof_headline --steps 6 --warmup 3 || exit $?
bash scripts/gpu_prof.sh $O/prof_lora --peft lora --steps 6 --warmup 3 || exit $?
bash scripts/gpu_sft_job_trace.sh ${1:-r3final}/sft ${SFT_JOB_ENV:-GRT_X=0} || exit $?
