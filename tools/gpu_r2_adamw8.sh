#!/bin/bash
# 8-wide AdamW: optimizer GPU tests, standalone kernel time (zoo, both variants), headline bench A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2aw8
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_parallel_gpu.py tests/test_parallel_gpu_multiproc.py -k "adam or overlap or optim or zero or fsdp or ddp" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0; do
  cd /tmp && GRT_ADAMW_V4=$v ZOO_REP=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/zoo$v -o z -- python3 $GRAFT_REPO_ROOT/tools/kernel_zoo.py > $GRAFT_REPO_ROOT/$O/zoo$v.log 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT
  echo "GRT_ADAMW_V4=$v: $(grep -h adamw_kernel $O/zoo$v/*kernel_stats.csv | cut -d, -f1-8)"
done
bash tools/gpu_ab_env.sh r2aw8 "GRT_ADAMW_V4=1" "GRT_ADAMW_V4=0" 2
