#!/bin/bash
# 70B QLoRA on one GPU with the streamed K-concatenated W' (cache off automatically), and the
# reference SFT job with the 4-bit-resident base (GRT_NF4_CACHE=0).
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-q70b}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 600 python -u bench.py --model llama3-70b --peft qlora --batch 8 --steps 3 --warmup 1 \
    --metrics-jsonl $OUT/m_b8.jsonl > $OUT/b8.log 2>&1; rc=$?
tail -1 $OUT/b8.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"mfu_bf16_dense": [0-9.]*\|"hbm_plan_gib": [0-9.]*\|"hbm_peak_gib": [0-9.]*' | tr '\n' ' '; echo; fatal $rc
[ $rc -eq 0 ] || exit $rc
export GRT_STORAGE_PATH=/tmp/grt_q4
GRT_NF4_CACHE=0 timeout -k 10 300 python3 jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_q4/out > $OUT/sft.log 2>&1; rc=$?
grep -h "training finished" $OUT/sft.log | grep -o "'train_runtime': [0-9.]*, 'train_samples_per_second': [0-9.]*"; fatal $rc
rm -rf /tmp/grt_q4
echo done
