#!/bin/bash
# Current-tree numbers for the other bench configurations: proxy-8 ZeRO rank step, FSDP, FSDP +
# offload (16-layer 70B slice), BasicLLM job shape.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r4modes}; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > $OUT/$n.log 2>&1; local rc=$?
  echo "$n: $(tail -1 $OUT/$n.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"hbm_peak_gib": [0-9.]*\|"parallelism": "[^"]*"' | tr '\n' ' ')"
  fatal $rc; return $rc
}
run headline --steps 10 --warmup 3 && \
run proxy8 --proxy-world 8 --steps 10 --warmup 3 && \
run fsdp --parallel fsdp --steps 10 --warmup 3 && \
run offload70b16 --model llama3-70b --layers 16 --parallel fsdp --offload --steps 3 --warmup 2
echo done
