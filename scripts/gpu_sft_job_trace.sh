#!/bin/bash
# The reference SFT job end to end (unchanged fine_tune_config.json, one worker) with the per-step
# trace on: where train_runtime goes (steps by token count, eval, checkpoint saves, first step).
# usage: scripts/gpu_sft_job_trace.sh <out-subdir> [extra env assignments for the job ...]
set -o pipefail
O=gpurun_out/${1:-sftjob}
shift
mkdir -p $O
export GRT_STORAGE_PATH=/tmp/grt_sftj
rm -rf /tmp/grt_sftj
env GRT_SFT_STEP_TRACE=1 "$@" timeout -k 10 400 python3 jobs/fine_tune_llama_ray.py --num-workers 1 \
  --set OUTPUT_DIR_BASE=/tmp/grt_sftj/out > $O/job.log 2>&1
rc=$?
find /tmp/grt_sftj -name step_trace.jsonl -exec cp {} $O/ \;
grep -h "train_samples_per_second" $O/job.log | tail -1 | cut -c1-300
exit $rc
