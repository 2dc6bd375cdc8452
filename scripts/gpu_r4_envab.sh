#!/bin/bash
# Runtime env A/B on the headline: HIP_FORCE_DEV_KERNARG (kernel arguments in device memory).
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-envab}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
for r in 1 2; do
  for k in 0 1; do
    HIP_FORCE_DEV_KERNARG=$k timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/b_${k}_$r.log 2>&1; rc=$?
    echo "kernarg=$k r$r $(tail -1 $OUT/b_${k}_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"; fatal $rc
  done
done
for k in 0 1; do
  export GRT_STORAGE_PATH=/tmp/grt_e$k
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 300 python3 jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_e$k/out > $OUT/sft$k.log 2>&1; rc=$?
  echo "kernarg=$k sft $(grep -h 'training finished' $OUT/sft$k.log | grep -o "'train_samples_per_second': [0-9.]*")"; fatal $rc
  rm -rf /tmp/grt_e$k
done
echo done
