# the reference SFT job (unchanged fine_tune_config.json: Llama-3.1-8B QLoRA r=64, 1000 samples) x2 on the
# final tree, plus the full-FT variant once
O=gpurun_out/r6sft; mkdir -p $O
for i in 1 2; do
  export GRT_STORAGE_PATH=/tmp/grt_sftj$i
  timeout -k 10 400 python3 -u jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sftj$i/out > $O/sft$i.log 2>&1 || { tail -20 $O/sft$i.log; exit 1; }
  grep -h "training finished" $O/sft$i.log | grep -o "'train_runtime': [0-9.]*, 'train_samples_per_second': [0-9.]*"
  rm -rf /tmp/grt_sftj$i
done
