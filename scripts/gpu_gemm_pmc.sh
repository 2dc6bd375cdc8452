#!/bin/bash
# PMC passes (one counter group per pass) over tools/gemm_pmc_drv.py; summary via tools/pmc_summary.py
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-gemmpmc}
rm -rf $OUT; mkdir -p $OUT
cd /tmp
D=$GRAFT_REPO_ROOT/tools/gemm_pmc_drv.py
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT -o trace -- python3 $D > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT -o sq -- python3 $D > $OUT/sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA --output-format csv -d $OUT -o sq2 -- python3 $D > $OUT/sq2.log 2>&1 || echo "sq2 pass failed (counter names?)"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT -o fetch -- python3 $D > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT -o write -- python3 $D > $OUT/write.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && python3 tools/pmc_summary.py gpurun_out/${1:-gemmpmc} > gpurun_out/${1:-gemmpmc}/summary.md 2>&1
cat gpurun_out/${1:-gemmpmc}/summary.md
