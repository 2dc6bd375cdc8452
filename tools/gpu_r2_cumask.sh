#!/bin/bash
# Overlapped optimizer on a CU-masked side stream: sweep of the CU count / pattern on the headline bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2cum
mkdir -p $O
timeout -k 10 120 python -c "
import torch
from gke_ray_train_amd.ops.streams import cu_masked_stream
from gke_ray_train_amd import _native
s = cu_masked_stream(32, 0)
print('mask', [hex(w) for w in _native.kernels().stream_cu_mask(s.cuda_stream, 8)])
x = torch.randn(1 << 20, device='cuda')
with torch.cuda.stream(s):
    y = x * 2
torch.cuda.current_stream().wait_stream(s)
assert torch.equal(y, x * 2)
print('masked stream ok')
" > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log
rm -f $O/ab.txt
for r in 1 ${ROUNDS:-}; do
  for v in "GRT_OPT_CUS=0" ${CFGS:-"GRT_OPT_CUS=32" "GRT_OPT_CUS=64" "GRT_OPT_CUS=32 GRT_OPT_CU_PATTERN=low" "GRT_OPT_CUS=16" "GRT_OPT_CUS=96"}; do
    env $v timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/run.log 2>&1 || { echo "[$v] failed"; tail -20 $O/run.log; exit 1; }
    echo "$v round $r: $(tail -1 $O/run.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["loss"])')" | tee -a $O/ab.txt
  done
done
