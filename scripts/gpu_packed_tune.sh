#!/bin/bash
# Tune the library GEMM shapes of the padding-free SFT steps: record the shapes the shipped table
# misses during the reference SFT job (packed steps on), tune them with TunableOp on top of the
# table, poison-check every row (tools/tune_untuned.py).
set -o pipefail
O=gpurun_out/${1:-r3pt}
mkdir -p $O
export GRT_STORAGE_PATH=/tmp/grt_sftj
rm -rf /tmp/grt_sftj
env GRT_SFT_PADDING_FREE=1 GRT_TUNED_GEMM_RECORD_UNTUNED=$GRAFT_REPO_ROOT/$O/untuned.csv timeout -k 10 300 \
  python3 jobs/fine_tune_llama_ray.py --num-workers 1 --set OUTPUT_DIR_BASE=/tmp/grt_sftj/out > $O/job_record.log 2>&1 \
  || { tail -20 $O/job_record.log; exit 1; }
grep -h "train_samples_per_second" $O/job_record.log | tail -1 | cut -c1-200
ls $O; wc -l $O/untuned*.csv
timeout -k 10 780 python3 -u tools/tune_untuned.py "$O/untuned*.csv" --out $O/tuned.csv --duration 20 > $O/tune.log 2>&1
rc=$?; tail -5 $O/tune.log; exit $rc
