#!/bin/bash
# Decode-path kernels (parallel split combine, fused RoPE + KV append, K-split / SwiGLU GEMV): GPU tests + decode bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2dec
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_jobs.py -k "gemv or rope or decode or generation or graph or sft or qlora" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/decode_bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep tokens_per_s $O/bench.log
