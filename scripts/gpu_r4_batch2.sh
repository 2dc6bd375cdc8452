#!/bin/bash
# Round 4 batch 2: FSDP offload overlap (tests + 16-layer Llama-3-70B slice: no offload, serial
# offload, overlapped offload all-streamed, overlapped with the planner's HBM-resident share),
# reference SFT job vs bench at the job's tokens/step.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4b2; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 300 python -u tools/offload_debug.py > $OUT/dbg.log 2>&1; rc=$?; grep -v amdgpu $OUT/dbg.log | tail -20; fatal $rc
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_parallel_gpu.py > $OUT/tests.log 2>&1; rc=$?; grep -E "PASS|FAIL" $OUT/tests.log | tail -15; fatal $rc
tail -3 $OUT/tests.log
S="--model llama3-70b --layers 16 --parallel fsdp --steps 3 --warmup 2"
timeout -k 10 400 python bench.py $S > $OUT/b70_plain.log 2>&1 || { tail -20 $OUT/b70_plain.log; exit 1; }
tail -1 $OUT/b70_plain.log
timeout -k 10 400 python bench.py $S --offload --offload-resident 0 --offload-overlap off > $OUT/b70_serial.log 2>&1 || { tail -20 $OUT/b70_serial.log; exit 1; }
tail -1 $OUT/b70_serial.log
timeout -k 10 400 python bench.py $S --offload --offload-resident 0 > $OUT/b70_overlap.log 2>&1 || { tail -20 $OUT/b70_overlap.log; exit 1; }
tail -1 $OUT/b70_overlap.log
timeout -k 10 400 python bench.py $S --offload > $OUT/b70_auto.log 2>&1 || { tail -20 $OUT/b70_auto.log; exit 1; }
tail -1 $OUT/b70_auto.log
timeout -k 10 300 python bench.py --batch 6 --seq 1024 --steps 20 --warmup 5 > $OUT/bench_b6.log 2>&1 || { tail -20 $OUT/bench_b6.log; exit 1; }
tail -1 $OUT/bench_b6.log
