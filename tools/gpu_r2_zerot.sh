#!/bin/bash
# ZeRO forward-time W^T: 2-rank engine tests on one GPU (gloo) + 2-rank bench rehearsal
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2zt
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parallel_gpu_multiproc.py tests/test_parallel_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 0 1; do
  GRT_ZERO_FWD_TRANSPOSE=$v timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --model llama-125m --batch 4 --seq 512 --steps 3 --warmup 1 > $O/mp_$v.log 2>&1 || { echo "mp bench $v failed"; tail -30 $O/mp_$v.log; exit 1; }
  echo "GRT_ZERO_FWD_TRANSPOSE=$v: $(grep metric $O/mp_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["loss"], d["config"]["parallelism"])')"
done
