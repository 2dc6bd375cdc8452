# re-tune forward/dX GEMMs with a 1 GiB rotating buffer (cold operands) and A/B the headline bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/tune_gemms.py --rotating-mb 1024 --out gpurun_out/tunableop_cold.csv > gpurun_out/tune_cold.log 2>&1 || { echo "tune failed"; tail -20 gpurun_out/tune_cold.log; exit 1; }
cat gpurun_out/tunableop_cold.csv
rm -f gpurun_out/tune_ab.txt
for i in 1 2; do
for f in gke_ray_train_amd/tuning/tunableop_mi355x.csv gpurun_out/tunableop_cold.csv; do
  GRT_TUNED_GEMM_FILE=$f timeout -k 10 400 python bench.py --steps 8 --warmup 3 > gpurun_out/tune_b.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/tune_b.log; exit 1; }
  echo "$f $(tail -1 gpurun_out/tune_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/tune_ab.txt
done
done
