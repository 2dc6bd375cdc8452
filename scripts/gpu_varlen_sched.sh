#!/bin/bash
# padding-free attention: causal-pair schedule on (7) vs off (0), varlen 6144 vs padded 8 x 768
set -o pipefail
O=gpurun_out/${1:-r3vs}
mkdir -p $O
for s in 7 0 7 0; do
  GRT_ATTN_SCHED=$s timeout -k 10 300 python -u tools/varlen_probe.py --cfgs 6144,6656 --padded 8x768 --steps 6 \
    > $O/s$s.jsonl 2> $O/s$s.err || { tail $O/s$s.err; exit 1; }
  echo "sched $s"; cat $O/s$s.jsonl
done
