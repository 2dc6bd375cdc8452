#!/bin/bash
# Round 4 batch 4: LoRA W'-tail reuse in no-grad forwards (GPU tests), reference SFT job twice.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4b4; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "kcat" > $OUT/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error" $OUT/tests.log | tail -12; fatal $rc; [ $rc = 0 ] || exit $rc
for i in 1 2; do
  export GRT_STORAGE_PATH=/tmp/grt_sftj$i
  timeout -k 10 300 python3 jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sftj$i/out > $OUT/sft$i.log 2>&1; rc=$?
  grep -h "train_samples_per_second\|eval_runtime" $OUT/sft$i.log | cut -c1-200; fatal $rc
  rm -rf /tmp/grt_sftj$i
done
echo done
