#!/usr/bin/env python3
"""List the large tensor copies (aten::copy_ / clone / contiguous) of one training step with the
Python stack that issued them: python tools/find_copies.py [--peft lora] [--layers 2] [--min-mb 16]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.models import build_llama, get_config  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama2-7b")
ap.add_argument("--peft", default="none", choices=["none", "lora", "qlora"])
ap.add_argument("--layers", type=int, default=2)
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--seq", type=int, default=1024)
ap.add_argument("--min-mb", type=float, default=16.0)
a = ap.parse_args()
dev = torch.device("cuda", 0)
from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms  # noqa: E402
enable_tuned_gemms()
cfg = get_config(a.model, num_hidden_layers=a.layers)
model = build_llama(cfg, device=dev, dtype=torch.bfloat16, seed=1)
fwd = model
if a.peft != "none":
    from gke_ray_train_amd.peft import BitsAndBytesConfig, LoraConfig, get_peft_model, quantize_model_
    if a.peft == "qlora":
        quantize_model_(model, BitsAndBytesConfig(bnb_4bit_compute_dtype=torch.bfloat16))
    fwd = get_peft_model(model, LoraConfig(r=64, lora_alpha=16, lora_dropout=0.1))
ids = torch.randint(0, cfg.vocab_size, (a.batch, a.seq), device=dev)
for _ in range(2):
    fwd(ids, labels=ids)["loss"].backward()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
    fwd(ids, labels=ids)["loss"].backward()
    torch.cuda.synchronize()
seen = 0
for ev in prof.events():
    if ev.name in ("aten::reshape", "aten::view", "aten::t", "aten::transpose", "aten::slice", "aten::select",
                   "aten::as_strided", "aten::empty", "aten::empty_like", "aten::detach", "aten::alias",
                   "aten::expand", "aten::narrow", "aten::unsqueeze", "aten::_unsafe_view", "aten::permute") \
            or ev.name.startswith("aten::mm") or ev.name.startswith("aten::addmm") or ev.name == "aten::linear" \
            or ev.name == "aten::matmul":
        continue
    shapes = ev.input_shapes or []
    numel = 0
    for sh in shapes:
        if sh and all(isinstance(d, int) for d in sh):
            n = 1
            for d in sh:
                n *= d
            numel = max(numel, n)
    if numel * 2 / 2 ** 20 < a.min_mb:
        continue
    seen += 1
    stack = [f for f in (ev.stack or []) if "gke_ray_train_amd" in f or "tools/" in f][:6]
    print(f"{ev.name} shapes {shapes} thread {ev.thread}" + ("\n    " + "\n    ".join(stack) if stack else ""),
          flush=True)
print("large copies:", seen)
