# PMC passes over tools/attn_pmc_run.py (B8 S1024 H32 causal fwd+bwd x3) on the round-6 kernels,
# dead-tile skips on (default) and off
export TMPDIR=/tmp
for s in 1 0; do
  OUT=$GRAFT_REPO_ROOT/gpurun_out/r6attnpmc$s
  rm -rf $OUT; mkdir -p $OUT
  export GRT_ATTN_SKIP=$s
  D=$GRAFT_REPO_ROOT/tools/attn_pmc_run.py
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT -o sq -- python3 $D > $OUT/sq.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA --output-format csv -d $OUT -o sq2 -- python3 $D > $OUT/sq2.log 2>&1 || exit $?
  cd $GRAFT_REPO_ROOT && python3 tools/pmc_summary.py gpurun_out/r6attnpmc$s > gpurun_out/r6attnpmc$s/summary.md 2>&1
  grep -i "attn" gpurun_out/r6attnpmc$s/summary.md | head -8
done
