#!/usr/bin/env python3
"""LoRA adapter kernels (lora.hip) at the Llama-2-7B bench shapes: direct kernel numerics vs fp32
torch, then a 2-layer LoRA model fwd/bwd with the kernels on vs off (same seeds), reporting NaNs
and the largest relative differences per gradient."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402
from gke_ray_train_amd.ops import _ref  # noqa: E402

C = _native.kernels()
dev = torch.device("cuda", 0)
M = int(os.environ.get("PROBE_M", "8192"))


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


for K, R in ((4096, 192), (4096, 128), (4096, 64), (11008, 64)):
    torch.manual_seed(0)
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    a = (torch.randn(R, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
    seed, p = 12345, 0.1
    h, xd = C.lora_down(x, a, p, seed, 0, True)
    keep = _ref.dropout_keep_mask(seed, 0, M * K, p).to(dev).view(M, K).float()
    xr = x.float() * keep / (1 - p)
    print(f"down K={K} R={R}: nan h {h.isnan().any().item()} xd {xd.isnan().any().item()} "
          f"rel h {rel(h, xr @ a.float().t()):.3e} rel xd {rel(xd, xr):.3e}", flush=True)
    g = torch.randn(M, R, device=dev, dtype=torch.bfloat16)
    dx = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    ref = (g.float() @ a.float()) * keep / (1 - p) + dx.float()
    ok = C.lora_dx(g, a.t().contiguous(), dx, p, seed, 0, True)
    print(f"dx   K={K} R={R}: ran {ok} nan {dx.isnan().any().item()} rel {rel(dx, ref):.3e}", flush=True)
    del x, xd, xr, keep, dx, ref

from gke_ray_train_amd.models import build_llama, get_config  # noqa: E402
from gke_ray_train_amd.peft import LoraConfig, get_peft_model  # noqa: E402
from gke_ray_train_amd.peft import lora as lora_mod  # noqa: E402

cfg = get_config("llama2-7b", num_hidden_layers=2)
res = {}
for on in (False, True):
    lora_mod._LORA_DOWN = lora_mod._LORA_DX = on
    model = build_llama(cfg, device=dev, dtype=torch.bfloat16, seed=1)
    torch.manual_seed(3)
    pm = get_peft_model(model, LoraConfig(r=64, lora_alpha=16, lora_dropout=0.1))
    with torch.no_grad():
        for n, prm in pm.named_parameters():
            if prm.requires_grad and "lora_B" in n:
                prm.normal_(0, 0.02)
    torch.manual_seed(7)
    ids = torch.randint(0, cfg.vocab_size, (M // 1024, 1024), device=dev)
    loss = pm(ids, labels=ids)["loss"]
    loss.backward()
    torch.cuda.synchronize()
    res[on] = (loss.item(), {n: prm.grad.detach().clone() for n, prm in pm.named_parameters() if prm.grad is not None})
    print(f"kernels={on}: loss {loss.item():.5f}, nan grads "
          f"{[n for n, g in res[on][1].items() if not torch.isfinite(g).all()][:6]}", flush=True)
    del model, pm, loss
worst = sorted(((rel(res[True][1][n], res[False][1][n]), n) for n in res[False][1]), reverse=True)[:8]
for r, n in worst:
    print(f"  grad rel diff {r:.3e} {n}")

# a few optimizer steps as bench.py runs them (DDP engine + fused AdamW, overlapped or not)
from gke_ray_train_amd.ops import FusedAdamW  # noqa: E402
from gke_ray_train_amd.parallel import DistributedDataParallel  # noqa: E402
from gke_ray_train_amd.parallel.overlap import OverlappedOptimizer  # noqa: E402
for on in (False, True):
    for overlap in (False, True):
        lora_mod._LORA_DOWN = lora_mod._LORA_DX = on
        model = build_llama(cfg, device=dev, dtype=torch.bfloat16, seed=1)
        torch.manual_seed(3)
        pm = get_peft_model(model, LoraConfig(r=64, lora_alpha=16, lora_dropout=0.1))
        eng = DistributedDataParallel(pm)
        opt = FusedAdamW(eng.optimizer_param_groups(weight_decay=0.0), lr=2e-5)
        if overlap:
            opt = OverlappedOptimizer(eng, opt)
        losses = []
        for it in range(5):
            ids = torch.randint(0, cfg.vocab_size, (M // 1024, 1024), device=dev)
            loss = pm(ids, labels=ids)["loss"]
            loss.backward()
            eng.finish_gradient_sync()
            st = eng.clip_grad_norm_(0.3)
            opt.step(grad_scale=st)
            eng.after_optimizer_step()
            eng.zero_grad()
            losses.append(round(loss.item(), 4))
        print(f"kernels={on} overlap={overlap}: losses {losses}", flush=True)
        del model, pm, eng, opt
