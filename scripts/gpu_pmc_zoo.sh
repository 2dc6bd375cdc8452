#!/bin/bash
# PMC passes over tools/kernel_zoo.py (one counter group per pass, kernel trace for durations)
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmczoo}
rm -rf $OUT; mkdir -p $OUT
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT -o trace -- python3 $GRAFT_REPO_ROOT/tools/kernel_zoo.py > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT -o sq -- python3 $GRAFT_REPO_ROOT/tools/kernel_zoo.py > $OUT/sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT -o fetch -- python3 $GRAFT_REPO_ROOT/tools/kernel_zoo.py > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT -o write -- python3 $GRAFT_REPO_ROOT/tools/kernel_zoo.py > $OUT/write.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && find gpurun_out/${1:-pmczoo} -name "*.csv" | sort && python3 tools/pmc_summary.py gpurun_out/${1:-pmczoo} > gpurun_out/${1:-pmczoo}/summary.md 2>&1
head -40 gpurun_out/${1:-pmczoo}/summary.md
