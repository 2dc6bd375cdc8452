#!/bin/bash
cd $GRAFT_REPO_ROOT
bash scripts/r5/gemm9.sh r5gemm9 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r5gemm9/bench.log 2>&1; rc=$?; tail -1 gpurun_out/r5gemm9/bench.log | cut -c1-300; exit $rc
