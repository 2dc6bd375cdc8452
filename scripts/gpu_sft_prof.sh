#!/bin/bash
# kernel profile of the SFT job's worker loop in one process (320 samples = 40 optimizer steps)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r2sftprof}
mkdir -p $O
export GRT_STORAGE_PATH=/tmp/grt_sftp
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run \
  -- python3 $GRAFT_REPO_ROOT/tools/sft_inproc.py --set NUM_TRAIN_SAMPLES=320 --set OUTPUT_DIR_BASE=/tmp/grt_sftp/out > $GRAFT_REPO_ROOT/$O/log.txt 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
grep -E "train_samples_per_second" $O/log.txt | tail -1 | cut -c1-250
exit $rc
