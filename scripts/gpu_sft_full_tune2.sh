#!/bin/bash
# continue scripts/gpu_sft_full_tune.sh: tune the logged shapes not yet in gpurun_out/r4ft/tuned.csv
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4ft2; rm -rf $O; mkdir -p $O
timeout -k 10 ${TUNE_S:-1000} python3 tools/tune_untuned.py "tuning_work/ft_untuned*.csv" --base tuning_work/ft_tuned_partial.csv --out $O/tuned.csv > $O/tune.log 2>&1; rc=$?
tail -3 $O/tune.log
exit $rc
