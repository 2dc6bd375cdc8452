#!/bin/bash
# kernel trace (no API trace: low host overhead) of the QLoRA reference SFT worker loop, 320 samples
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sftkt}
rm -rf $O; mkdir -p $O
export GRT_STORAGE_PATH=/tmp/grt_sftk
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O -o run \
  -- python3 $GRAFT_REPO_ROOT/tools/sft_inproc.py --set NUM_TRAIN_SAMPLES=320 --set EVAL_STEPS_SFT=1000 --set SAVE_STEPS_SFT=1000 --set OUTPUT_DIR_BASE=/tmp/grt_sftk/out > $O/log.txt 2>&1
rc=$?
cd $GRAFT_REPO_ROOT; grep "train_samples_per_second" $O/log.txt | tail -1 | cut -c1-200
find $O -name "*.csv" -size +20M -exec gzip {} \;
exit $rc
