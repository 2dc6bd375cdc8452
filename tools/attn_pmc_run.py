"""Llama-2-7B attention fwd+bwd (B8 S1024 H32 D128 causal, bf16) x3, for PMC collection."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import ops  # noqa: E402

q, k, v = (torch.randn(8, 1024, 32, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
do = torch.randn(8, 1024, 32, 128, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    o = ops.flash_attention(q, k, v, causal=True)
    torch.autograd.backward(o, do)
torch.cuda.synchronize()
