#!/bin/bash
# Attention workgroup schedule A/B: correctness tests (default schedule), kernel timings of both
# schedules interleaved in one process (bitwise-equality check), then the headline and LoRA
# bench under each schedule (GRT_ATTN_SCHED), interleaved.
set -o pipefail
O=gpurun_out/${1:-attnsched}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "attn or attention or varlen or flash" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/attn_ab.py --scheds 0,1 --rounds 7 > $O/attn_ab.jsonl 2>&1 || { cat $O/attn_ab.jsonl; exit 1; }
cat $O/attn_ab.jsonl
for mode in "" "--peft lora"; do
  for s in 0 1; do
    GRT_ATTN_SCHED=$s timeout -k 10 300 python bench.py $mode > $O/bench_s${s}_${mode:7:4}.log 2>&1 || exit $?
    echo "sched $s $mode: $(tail -1 $O/bench_s${s}_${mode:7:4}.log | cut -c1-160)"
  done
done
