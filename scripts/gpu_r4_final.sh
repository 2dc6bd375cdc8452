#!/bin/bash
# Round-4 state check: full GPU suite, smoke, headline bench, LoRA / QLoRA bench, reference SFT job x2
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4final}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
grep -E "^FAILED|^ERROR" $OUT/tests.log | head -10; tail -1 $OUT/tests.log; fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log; fatal $rc
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1; rc=$?; tail -1 $OUT/bench.log | cut -c1-250; fatal $rc
for pe in lora qlora; do
  timeout -k 10 300 python bench.py --peft $pe > $OUT/bench_$pe.log 2>&1; rc=$?; tail -1 $OUT/bench_$pe.log | cut -c1-160; fatal $rc
done
for i in 1 2; do
  export GRT_STORAGE_PATH=/tmp/grt_sftj$i
  timeout -k 10 300 python3 jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sftj$i/out > $OUT/sft$i.log 2>&1; rc=$?
  grep -h "training finished" $OUT/sft$i.log | grep -o "'train_runtime': [0-9.]*, 'train_samples_per_second': [0-9.]*"; fatal $rc
  rm -rf /tmp/grt_sftj$i
done
echo done
