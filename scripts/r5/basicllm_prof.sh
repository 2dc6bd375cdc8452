#!/bin/bash
# Reference job #1 (BasicLLM, fp32, 16 x 256 tokens per step) on one GPU under rocprofv3
# --kernel-trace --stats: which kernels (fp32 GEMM solutions) the step runs and their time.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5basicllm}; rm -rf $OUT; mkdir -p $OUT
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bl -- python3 -u $GRAFT_REPO_ROOT/tools/basicllm_inproc.py --max-windows ${WINDOWS:-3200} > $OUT/job.log 2>&1; rc=$?
tail -5 $OUT/job.log; [ $rc = 0 ] || { echo "rc=$rc"; exit $rc; }
cd $GRAFT_REPO_ROOT && python3 tools/prof_steps.py --help > /dev/null 2>&1
find $OUT/prof -name "*kernel_stats.csv" | head -3
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv; head -25 "$f" | cut -c1-300
rm -rf $OUT/prof
