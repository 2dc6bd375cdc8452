#!/bin/bash
# Round 4 batch 1: GEMM + SFT-engine GPU tests, LoRA / QLoRA memory-plan check, proxy-world 8,
# full fine-tune through the reference SFT job at bench speed (llama2-7b), bench at its tokens/step.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4b1; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gemm_gpu.py \
  "tests/test_gpu_jobs.py::test_sft_full_ft_overlapped_engine_matches_plain_path" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for pe in lora qlora; do
  timeout -k 10 300 python bench.py --peft $pe --steps 5 --warmup 2 > $OUT/bench_$pe.log 2>&1 || { tail -20 $OUT/bench_$pe.log; exit 1; }
  tail -1 $OUT/bench_$pe.log
done
timeout -k 10 300 python bench.py --proxy-world 8 --steps 6 --warmup 3 > $OUT/bench_proxy8.log 2>&1 || { tail -20 $OUT/bench_proxy8.log; exit 1; }
tail -1 $OUT/bench_proxy8.log
timeout -k 10 600 python -u jobs/fine_tune_llama_ray.py --num-workers 1 --set USE_QLORA=false --set MODEL_ID=llama2-7b \
  --set OUTPUT_DIR_BASE=/tmp/sftfull --set SAVE_STRATEGY=no --set NUM_TRAIN_SAMPLES=400 --set REPORT_TO=none \
  --set LEARNING_RATE=2e-5 > $OUT/sft_full.log 2>&1 || { tail -30 $OUT/sft_full.log; exit 1; }
grep -E "tokens_per_sec|Results" $OUT/sft_full.log | tail -4
rm -rf /tmp/sftfull
timeout -k 10 300 python bench.py --batch 2 --seq 1024 --steps 20 --warmup 5 > $OUT/bench_b2.log 2>&1 || { tail -20 $OUT/bench_b2.log; exit 1; }
tail -1 $OUT/bench_b2.log
