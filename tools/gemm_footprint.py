"""Does a large resident footprint (as in a 7B training step: ~110 GB of params, grads, Adam state
and activations) slow the projection GEMMs (TLB reach)? Same GEMMs timed before and after
allocating FILL_GB of filler tensors, with operands spread between the filler allocations."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms()
M, K, N = 8192, 4096, 12288


def run(tag, dy, w, x, wf):
    res = {}
    for kind, fn in (("fwd", lambda: F.linear(x, wf)), ("dgrad", lambda: dy @ w)):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(40):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[kind] = round(2 * M * N * K / (e0.elapsed_time(e1) / 40) / 1e9)
    print(json.dumps({"tag": tag, **res}), flush=True)


def mk(*shape):
    return torch.randn(*shape, device="cuda", dtype=torch.bfloat16)


run("small footprint", mk(M, N), mk(N, K), mk(M, K), mk(N, K))
fill = []
ops = []
for i in range(int(os.environ.get("FILL_GB", "120")) // 4):
    fill.append(torch.empty(2 * 1024 ** 3, device="cuda", dtype=torch.bfloat16))  # 4 GB
    if i % 7 == 3:
        ops.append((mk(M, N), mk(N, K), mk(M, K), mk(N, K)))
print("allocated GB", torch.cuda.memory_allocated() / 2 ** 30, flush=True)
for j, o in enumerate(ops[:3]):
    run(f"large footprint set {j}", *o)
