#!/bin/bash
# PMC passes (one counter group per pass) + a kernel trace over an arbitrary python command:
#   bash scripts/gpu_pmc_cmd.sh <outdir under gpurun_out> <script.py> [args...]
# then: python3 tools/pmc_summary.py gpurun_out/<outdir>
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
shift
S=$1
shift
[[ $S != /* ]] && S=$GRAFT_REPO_ROOT/$S
set -- "$S" "$@"
rm -rf $OUT; mkdir -p $OUT
cd /tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $OUT -o trace -- python3 "$@" > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT -o sq -- python3 "$@" > $OUT/sq.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT -o fetch -- python3 "$@" > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT -o write -- python3 "$@" > $OUT/write.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && python3 tools/pmc_summary.py gpurun_out/${OUT##*/gpurun_out/} > $OUT/summary.md 2>&1
cat $OUT/summary.md | head -30
