#!/bin/bash
# Round 4 batch 5: grouped LoRA adapter-gradient launches (lora_g / dB token reductions per module),
# sync-free training logs: GPU tests, LoRA / QLoRA bench, reference SFT job twice.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4b5; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lora_grad_gpu.py tests/test_gpu_jobs.py \
  "tests/test_kernels_gpu.py::test_kcat_lora_model_matches_epilogue_form" "tests/test_kernels_gpu.py::test_kcat_lora_matches_reference" > $OUT/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error" $OUT/tests.log | tail -8; tail -1 $OUT/tests.log; fatal $rc; [ $rc = 0 ] || exit $rc
for pe in lora qlora; do
  timeout -k 10 300 python bench.py --peft $pe --steps 10 --warmup 3 > $OUT/bench_$pe.log 2>&1; rc=$?; tail -1 $OUT/bench_$pe.log | cut -c1-160; fatal $rc
done
for i in 1 2; do
  export GRT_STORAGE_PATH=/tmp/grt_sftj$i
  timeout -k 10 300 python3 jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sftj$i/out > $OUT/sft$i.log 2>&1; rc=$?
  grep -h "train_samples_per_second\|eval_runtime" $OUT/sft$i.log | cut -c1-200; fatal $rc
  rm -rf /tmp/grt_sftj$i
done
echo done
