#!/bin/bash
# LoRA adapter-first forward: LoRA GPU tests, LoRA bench A/B (loss printed), SFT job, 2-rank gloo rehearsal
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2laf
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_jobs.py -k "lora or qlora or peft or fused_accumulation" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
rm -f $O/ab.txt
for r in 1 2; do
  for v in 0 1; do
    GRT_LORA_ADAPTER_FIRST=$v timeout -k 10 300 python bench.py --peft lora --steps 15 --warmup 4 > $O/run.log 2>&1 || { echo "bench [$v] failed"; tail -20 $O/run.log; exit 1; }
    echo "GRT_LORA_ADAPTER_FIRST=$v round $r: $(tail -1 $O/run.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["loss"])')" | tee -a $O/ab.txt
  done
done
export GRT_STORAGE_PATH=/tmp/grt_sft_af
timeout -k 10 400 python -u jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sft_af/out > $O/sft.log 2>&1 || { echo "sft failed"; tail -30 $O/sft.log; exit 1; }
echo "SFT: $(grep -E "train_samples_per_second" $O/sft.log | tail -1 | cut -c1-200)"
for par in ddp fsdp; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --model llama-125m --batch 4 --seq 512 --steps 3 --warmup 1 --parallel $par > $O/mp_bench_$par.log 2>&1 || { echo "mp bench $par failed"; tail -30 $O/mp_bench_$par.log; exit 1; }
  grep metric $O/mp_bench_$par.log | cut -c1-400
done
