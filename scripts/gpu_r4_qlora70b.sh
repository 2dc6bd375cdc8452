#!/bin/bash
# Llama-3-70B QLoRA on ONE MI355X: NF4 base without the dequant cache (set_dequant_cache auto = off
# at 70B), planner vs measured peak. Batch 2 then batch 8 (the planner's 237 GiB case).
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-q70}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
for b in 2 8; do
  timeout -k 10 600 python -u bench.py --model llama3-70b --peft qlora --batch $b --steps 3 --warmup 1 \
      --metrics-jsonl $OUT/m_b$b.jsonl > $OUT/b$b.log 2>&1; rc=$?
  grep -h "memory_plan\|hbm_total_gib" $OUT/b$b.log | tail -1 | cut -c1-200; tail -1 $OUT/b$b.log | cut -c1-300; fatal $rc
  [ $rc -eq 0 ] || exit $rc
done
echo done
