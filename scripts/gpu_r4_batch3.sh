#!/bin/bash
# Round 4 batch 3: lean-DMA GEMM variants, reference SFT job
# twice (unchanged config), kernel traces of its evaluation pass and of its training steps.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r4b3; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 300 python -u tools/gemm_bench.py --set fwd --variants 3,4,7,8 --rounds 3 > $OUT/gemm.log 2>&1; rc=$?; grep '^{' $OUT/gemm.log; fatal $rc
for i in 1 2; do
  export GRT_STORAGE_PATH=/tmp/grt_sftj$i
  timeout -k 10 300 python3 jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sftj$i/out > $OUT/sft$i.log 2>&1; rc=$?
  grep -h "train_samples_per_second\|eval_runtime" $OUT/sft$i.log | cut -c1-260; fatal $rc
  rm -rf /tmp/grt_sftj$i
done
export GRT_STORAGE_PATH=/tmp/grt_sfte
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_eval -o run \
  -- python3 $GRAFT_REPO_ROOT/tools/sft_eval_inproc.py --evals 3 --set OUTPUT_DIR_BASE=/tmp/grt_sfte/out > $GRAFT_REPO_ROOT/$OUT/eval.log 2>&1; rc=$?
cd $GRAFT_REPO_ROOT; grep "eval wall" $OUT/eval.log | cut -c1-300; fatal $rc
export GRT_STORAGE_PATH=/tmp/grt_sftp
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_train -o run \
  -- python3 $GRAFT_REPO_ROOT/tools/sft_inproc.py --set NUM_TRAIN_SAMPLES=320 --set EVAL_STEPS_SFT=1000 --set OUTPUT_DIR_BASE=/tmp/grt_sftp/out > $GRAFT_REPO_ROOT/$OUT/train.log 2>&1; rc=$?
cd $GRAFT_REPO_ROOT; grep "train_samples_per_second" $OUT/train.log | tail -1 | cut -c1-250; fatal $rc
find $OUT -name "*.db" -delete; find $OUT -name "*kernel_trace.csv" -size +30M -exec gzip {} \;
echo done
