#!/bin/bash
# tune the TN weight-gradient GEMMs, gate the merged table, A/B it on the headline bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2tunetn
mkdir -p $O
timeout -k 10 400 python -u tools/tune_wgrad_tn.py --out $O/tn.csv > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -2 $O/tune.log
timeout -k 10 300 python -u tools/gemm_overread_probe.py --table $O/tn.csv --prune $O/tn_pruned.csv --out $O/probe.jsonl > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v '"ok": true' $O/probe.log | tail -5
bash tools/gpu_ab_env.sh r2tunetn/ab "GRT_TUNED_GEMM_FILE=gke_ray_train_amd/tuning/tunableop_mi355x.csv" "GRT_TUNED_GEMM_FILE=$O/tn_pruned.csv" 2
