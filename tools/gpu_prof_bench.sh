#!/bin/bash
# Kernel-time profile of the 1-GPU bench: bash tools/gpu_prof_bench.sh <outdir> [bench args...]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run \
  -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 3 "$@" > $GRAFT_REPO_ROOT/$O/prof_bench.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
tail -2 $O/prof_bench.log
exit $rc
