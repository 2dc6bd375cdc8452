#!/bin/bash
# rocprofv3 kernel tables of one LoRA step: padding-free 6144 tokens vs padded 8 x 768
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3vvp}
mkdir -p $O
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/v6144 -o run \
  -- python3 $R/tools/varlen_probe.py --cfgs 6144 --padded "" --steps 4 --warmup 2 > $R/$O/v6144.log 2>&1) || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p8x768 -o run \
  -- python3 $R/tools/varlen_probe.py --cfgs "" --padded 8x768 --steps 4 --warmup 2 > $R/$O/p8x768.log 2>&1) || exit 1
grep cfg $O/v6144.log $O/p8x768.log
