"""Decode throughput on MI355X: eager cached decode vs the HIP-graph decoder (models/generation.py).
Llama-3.1-8B architecture, random init, bf16, batch 1, prompt 512, 128 new tokens (the
reference's inference comparison generates up to MAX_NEW_GENERATION_TOKENS_INFERENCE = 300
tokens per sample, ray-jobs/fine_tune_config.json:35). One JSON line per mode."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.models import build_llama  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "llama3.1-8b"
m = build_llama(model, device="cuda", dtype=torch.bfloat16, seed=0)
B = int(os.environ.get("DECODE_B", "1"))  # sequences decoded together (batch of requests)
ids = torch.randint(0, m.config.vocab_size, (B, 512), device="cuda")
from gke_ray_train_amd.ops import linear as _lin  # noqa: E402

runs = [(False, True), (True, False), (True, True)]  # (graph, gemv)
for mode, gemv in runs:
    _lin._GEMV = gemv
    m.generate(ids, max_new_tokens=8, use_graph=mode)  # warm-up (kernels, graph pools)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = m.generate(ids, max_new_tokens=128, use_graph=mode)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"model": model, "mode": ("hip_graph" if mode else "eager") + ("+gemv" if gemv else "+library_gemm"),
                      "batch": B, "new_tokens": out.shape[1] - 512,
                      "seconds": round(dt, 3), "tokens_per_s": round(B * (out.shape[1] - 512) / dt, 1)}), flush=True)
