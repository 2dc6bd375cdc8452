#!/bin/bash
# Round 2: every bench mode + the reference SFT job + BasicLLM job on one MI355X, then a 2-rank
# gloo rehearsal of the multi-GPU code paths (both ranks share the one GPU).
# Output: gpurun_out/r2modes/{bench_modes.jsonl,sft.log,basic.log,mp_*.log}
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2modes
mkdir -p $O
rm -f $O/bench_modes.jsonl
for mode in "" "--parallel fsdp" "--peft lora" "--peft qlora" "--peft lora --data pipeline"; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 $mode > $O/bench_mode.log 2>&1 || { echo "bench $mode failed"; tail -20 $O/bench_mode.log; exit 1; }
  tail -1 $O/bench_mode.log >> $O/bench_modes.jsonl
  echo "$mode: $(tail -1 $O/bench_mode.log | cut -c100-200)"
done
export GRT_STORAGE_PATH=/tmp/grt_sft
timeout -k 10 400 python -u jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sft/out > $O/sft.log 2>&1 || { echo "sft failed"; tail -30 $O/sft.log; exit 1; }
grep -E "train_samples_per_second|train_runtime" $O/sft.log | tail -3 | cut -c1-300
timeout -k 10 400 python -u jobs/pytorch_llm_ray.py --workers 1 > $O/basic.log 2>&1 || { echo "basicllm failed"; tail -30 $O/basic.log; exit 1; }
grep -iE "tokens/s|tok/s|throughput" $O/basic.log | tail -3 | cut -c1-300
for par in ddp fsdp; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --model llama-125m --batch 4 --seq 512 --steps 3 --warmup 1 --parallel $par > $O/mp_bench_$par.log 2>&1 || { echo "mp bench $par failed"; tail -30 $O/mp_bench_$par.log; exit 1; }
  grep metric $O/mp_bench_$par.log | cut -c1-220
done
