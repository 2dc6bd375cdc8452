#!/bin/bash
# Round 4 batch 7: no host-device sync inside a training step (pinned hyper-parameter uploads,
# index_fill_ label shift) + sync-free logs: tests, reference SFT job twice, HIP API trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r4b7; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_jobs.py tests/test_parallel_gpu.py tests/test_varlen.py > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; fatal $rc; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  export GRT_STORAGE_PATH=/tmp/grt_sftj$i
  timeout -k 10 300 python3 jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sftj$i/out > $OUT/sft$i.log 2>&1; rc=$?
  grep -h "train_samples_per_second\|eval_runtime" $OUT/sft$i.log | cut -c1-200; fatal $rc
  rm -rf /tmp/grt_sftj$i
done
bash scripts/gpu_sft_hiptrace.sh r4b7/hip; rc=$?; fatal $rc
echo done
