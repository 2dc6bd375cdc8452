#!/bin/bash
# Round-3 batch 2: attention adaptive pairing + dK/dV interleave A/B, headline and LoRA bench on the
# new defaults, then the padding-free SFT GEMM shapes recorded / tuned / A/B'd.
set -o pipefail
O=gpurun_out/${1:-r3batch2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "attn or attention or varlen or flash" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/attn_ab.py --scheds 0,7,15 --rounds 7 > $O/attn_ab.jsonl 2>&1 || { cat $O/attn_ab.jsonl; exit 1; }
grep -v max_err $O/attn_ab.jsonl
for mode in "" "--peft lora"; do
  timeout -k 10 300 python bench.py $mode > $O/bench_${mode:7:4}.log 2>&1 || exit $?
  echo "bench $mode: $(tail -1 $O/bench_${mode:7:4}.log | cut -c1-150)"
done
SFT_ENV=GRT_SFT_PADDING_FREE=1 TUNE_S=600 bash scripts/gpu_sft_tune.sh ${1:-r3batch2}/pfree_tune || exit $?
