#!/bin/bash
# Frozen-norm dX-only backward: GPU tests, reference SFT job x2, kernel trace of the SFT loop.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4norm}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "rmsnorm or layernorm or kcat or lora" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $OUT/test.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR" $OUT/test.log | head; tail -1 $OUT/test.log; fatal $rc; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  export GRT_STORAGE_PATH=/tmp/grt_n$i
  timeout -k 10 300 python3 jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_n$i/out > $OUT/sft$i.log 2>&1; rc=$?
  grep -h "training finished" $OUT/sft$i.log | grep -o "'train_runtime': [0-9.]*, 'train_samples_per_second': [0-9.]*"; fatal $rc
  rm -rf /tmp/grt_n$i
done
bash scripts/gpu_sft_ktrace.sh ${1:-r4norm}_kt; rc=$?; echo "ktrace rc $rc"
echo done
