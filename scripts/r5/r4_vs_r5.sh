#!/bin/bash
# headline A/B on one box: the round-4 tree (git worktree ab_base/ at the round-4 commit, its own
# _C.so) vs this tree, driver arguments (--steps 20 --warmup 5), interleaved
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5vs4}; rm -rf $OUT; mkdir -p $OUT
for r in 1 2; do
  (cd ab_base && timeout -k 10 300 python bench.py --steps 20 --warmup 5 > ../$OUT/r4_$r.log 2>&1); rc=$?
  echo "r4 run $r: $(tail -1 $OUT/r4_$r.log | cut -c100-190)"; [ $rc = 0 ] || exit $rc
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/r5_$r.log 2>&1; rc=$?
  echo "r5 run $r: $(tail -1 $OUT/r5_$r.log | cut -c100-190)"; [ $rc = 0 ] || exit $rc
done
