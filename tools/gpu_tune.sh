export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1500 python tools/tune_gemms.py --out gpurun_out/tunableop_mi355x.csv > gpurun_out/tune.log 2>&1 || { echo "tuning failed"; tail -20 gpurun_out/tune.log; exit 1; }
tail -3 gpurun_out/tune.log
mkdir -p gke_ray_train_amd/tuning && cp gpurun_out/tunableop_mi355x.csv gke_ray_train_amd/tuning/
for flag in --no-tuned-gemm "" --no-tuned-gemm ""; do
  timeout -k 10 400 python bench.py --steps 6 --warmup 2 $flag > gpurun_out/tune_b.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/tune_b.log; exit 1; }
  tail -1 gpurun_out/tune_b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['library_gemms'], d['value'], d['ms_per_step'])"
done
