#!/bin/bash
# every bench mode on the round-5 tree (one box): FSDP, LoRA, QLoRA, Ray-Data pipeline, forced RCCL
# collectives at world 1, the per-rank step of an 8-GPU ZeRO job
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5modes}; rm -rf $OUT; mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name: $(tail -1 $OUT/$name.log | python3 -c 'import json,sys
try:
    d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["parallelism"], d.get("hbm_plan_gib"), d.get("hbm_peak_gib"))
except Exception as e: print("parse error", e)')"
  return $rc
}
run headline || exit $?
run fsdp --parallel fsdp || exit $?
run lora --peft lora || exit $?
run qlora --peft qlora || exit $?
run pipeline --data pipeline || exit $?
run forced --force-collectives || exit $?
run proxy8 --proxy-world 8 || exit $?
