#!/bin/bash
# k64 GEMM (gemm_k64.hip) correctness (tools/gemm_diag.py) + A/B vs hipBLASLt on the Llama-2-7B step
# shapes. VARIANTS: 9 / 10 = SCHED 1 persistent / per-tile, 11 / 12 = SCHED 2 persistent / per-tile
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5gemm9}; rm -rf $OUT; mkdir -p $OUT
V=${VARIANTS:-9,10,11,12}
for v in ${V//,/ }; do
  timeout -k 10 120 python -u tools/gemm_diag.py --variant $v > $OUT/diag$v.log 2>&1; rc=$?
  echo "--- diag $v"; cat $OUT/diag$v.log | tail -20
  [ $rc = 0 ] || { echo "diag rc=$rc"; exit $rc; }
done
timeout -k 10 400 python -u tools/gemm_bench.py --set fwd,dgrad,wgrad --variants $V --rounds 5 --reps 10 > $OUT/gemm.log 2>&1; rc=$?
grep -E '^\{|check|wrong|Error|error' $OUT/gemm.log | head -80; echo "rc=$rc"; exit $rc
