#!/bin/bash
# headline bench A/B: grid cap of the overlapped AdamW chunks (0 = full grid)
set -o pipefail
mkdir -p gpurun_out
for b in 0 64 128 32 256 0; do
  GRT_OVERLAP_OPT_BLOCKS=$b timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/optblocks_$b.log 2>&1 || exit $?
  echo "blocks=$b $(tail -1 gpurun_out/optblocks_$b.log | cut -c100-250)"
done
