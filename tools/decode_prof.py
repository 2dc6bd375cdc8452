"""Llama-3.1-8B batch-1 decode (prompt 512, 64 new tokens, GEMV; HIP graph unless argv[1] == eager)
for kernel profiling: rocprofv3 --kernel-trace --stats -- python3 tools/decode_prof.py [graph|eager]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.models import build_llama  # noqa: E402

graph = (sys.argv[1] if len(sys.argv) > 1 else "graph") != "eager"
m = build_llama("llama3.1-8b", device="cuda", dtype=torch.bfloat16, seed=0)
ids = torch.randint(0, m.config.vocab_size, (1, 512), device="cuda")
m.generate(ids, max_new_tokens=8, use_graph=graph)
m.generate(ids, max_new_tokens=64, use_graph=graph)
torch.cuda.synchronize()
