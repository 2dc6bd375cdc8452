#!/bin/bash
# The package's in-process HIP_FORCE_DEV_KERNARG default (unset in the shell) vs an explicit 0.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-envab2}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
unset HIP_FORCE_DEV_KERNARG
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/b_def_$r.log 2>&1; rc=$?
  echo "default r$r $(tail -1 $OUT/b_def_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"; fatal $rc
  HIP_FORCE_DEV_KERNARG=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/b_0_$r.log 2>&1; rc=$?
  echo "explicit0 r$r $(tail -1 $OUT/b_0_$r.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"; fatal $rc
done
export GRT_STORAGE_PATH=/tmp/grt_e2
timeout -k 10 300 python3 jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_e2/out > $OUT/sft.log 2>&1; rc=$?
echo "default sft $(grep -h 'training finished' $OUT/sft.log | grep -o "'train_samples_per_second': [0-9.]*")"; fatal $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log; fatal $rc
echo done
