#!/bin/bash
# Interleaved A/B of the reference SFT job (unchanged config): ab_base/ (a git worktree of an earlier
# commit, built in place) vs this tree, two runs each on one box.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-sftab}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
for i in 1 2; do
  for arm in base new; do
    root=$PWD; [ $arm = base ] && root=$PWD/ab_base
    export GRT_STORAGE_PATH=/tmp/grt_ab_$arm$i
    timeout -k 10 300 python3 $root/jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_ab_$arm$i/out > $OUT/$arm$i.log 2>&1; rc=$?
    echo "$arm $i: $(grep -h 'training finished' $OUT/$arm$i.log | grep -o "'train_runtime': [0-9.]*, 'train_samples_per_second': [0-9.]*")"; fatal $rc
    rm -rf /tmp/grt_ab_$arm$i
  done
done
