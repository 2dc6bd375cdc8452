#!/bin/bash
# rocprofv3 kernel tables of one padding-free LoRA step at an odd vs even multiple of 512 tokens
# (tools/varlen_probe.py), then the LoRA bench step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3vp}
mkdir -p $O
R=$GRAFT_REPO_ROOT
for T in 5632 6144; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p$T -o run \
    -- python3 $R/tools/varlen_probe.py --cfgs $T --padded "" --steps 4 --warmup 2 > $R/$O/p$T.log 2>&1) || exit 1
  tail -1 $O/p$T.log
done
bash scripts/gpu_prof.sh $O/prof_lora --peft lora --steps 6 --warmup 3 || exit $?
