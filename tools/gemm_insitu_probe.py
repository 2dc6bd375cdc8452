"""Find why in-step forward GEMMs dispatch a different library kernel than a bare F.linear.
Each variant runs the qkv-shaped projection 3x, separated by a marker kernel (a 1-element fill)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms  # noqa: E402

print("tuned:", enable_tuned_gemms(), flush=True)
from gke_ray_train_amd.ops.linear import linear as ops_linear  # noqa: E402
from gke_ray_train_amd.models import build_llama  # noqa: E402
from gke_ray_train_amd.parallel import DistributedDataParallel  # noqa: E402

mark = torch.zeros(1, device="cuda")
M, K, N = 8192, 4096, 12288
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)


def sep(tag):
    torch.cuda.synchronize()
    mark.fill_(1.0)
    torch.cuda.synchronize()
    print("variant", tag, flush=True)


sep("A plain F.linear")
for _ in range(3):
    F.linear(x, w)
sep("B requires_grad weight via ops.linear (no slot)")
wp = torch.nn.Parameter(w.clone())
for _ in range(3):
    ops_linear(x, wp)
sep("C 3-D input")
for _ in range(3):
    F.linear(x.view(8, 1024, K), w)
sep("D model forward (1 layer llama2-7b, DDP)")
m = build_llama("llama2-7b", device="cuda", dtype=torch.bfloat16, seed=0, num_hidden_layers=1)
ddp = DistributedDataParallel(m)
ids = torch.randint(0, 32000, (8, 1024), device="cuda")
for _ in range(2):
    loss = ddp(ids, labels=ids)["loss"]
    loss.backward()
    ddp.zero_grad()
sep("E model forward no_grad")
with torch.no_grad():
    ddp(ids, labels=ids)
sep("end")
