#!/bin/bash
# new GPU tests (stream_copy, transposed dqkv, offload resume, scheduler flag), host-link + fp32
# probes, headline A/B of the transposed-dqkv epilogue
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r5batch7; rm -rf $OUT; mkdir -p $OUT
fatal() { case $1 in 0) ;; *) echo "fatal rc $1"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_hostcopy_gpu.py \
  "tests/test_kernels_gpu.py::test_attn_bwd_writes_transposed_dqkv" tests/test_kernels_gpu.py -k "transposed_dqkv or rope_attention_fused or stream_copy" > $OUT/tests.log 2>&1; rc=$?
grep -E "passed|failed|Error" $OUT/tests.log | tail -5; fatal $rc
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_parallel_gpu.py -k "resume or scheduler or overlapped_offload" > $OUT/tests2.log 2>&1; rc=$?
grep -E "passed|failed|Error" $OUT/tests2.log | tail -5; fatal $rc
timeout -k 10 200 python3 tools/hostlink_bench.py > $OUT/hostlink.log 2>&1; rc=$?; tail -1 $OUT/hostlink.log; fatal $rc
timeout -k 10 120 python3 tools/fp32_gemm_probe.py > $OUT/fp32.log 2>&1; rc=$?; tail -1 $OUT/fp32.log; fatal $rc
for r in 1 2; do
  for v in 0 1; do
    GRT_ATTN_DQKV_T=$v timeout -k 10 300 python bench.py > $OUT/bench_t${v}_$r.log 2>&1; rc=$?
    echo "dqkv_t=$v run $r: $(tail -1 $OUT/bench_t${v}_$r.log | cut -c1-160)"; fatal $rc
  done
done
