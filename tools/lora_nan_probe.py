#!/usr/bin/env python3
"""Find the first non-finite tensor of a Llama-2-7B LoRA forward/backward built exactly as bench.py
builds it (tuned library GEMMs on): every lora_down / lora_dx call is checked against its torch
equivalent, and every module's forward output is checked for NaN/Inf."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import _native  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(1234)
if os.environ.get("PROBE_TUNED", "1") == "1":
    from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms
    print("tuned gemms:", enable_tuned_gemms(), flush=True)
Creal = _native.kernels()
calls = {"down": 0, "dx": 0}
reported = [0]


class Proxy:
    def __getattr__(self, name):
        return getattr(Creal, name)

    def lora_down(self, x, a, p, seed, offset, want_xd):
        res = Creal.lora_down(x, a, p, seed, offset, want_xd)
        calls["down"] += 1
        if res and reported[0] < 5:
            h = res[0]
            xd = Creal.dropout_fwd_seeded(x, p, seed, offset) if p > 0 else x
            ht = xd @ a.t()
            bad = (not torch.isfinite(h).all().item()) or (not torch.isfinite(x).all().item())
            err = ((h.float() - ht.float()).norm() / ht.float().norm()).item()
            if bad or err > 1e-2:
                reported[0] += 1
                print(f"lora_down call {calls['down']}: x {tuple(x.shape)} stride {x.stride()} a {tuple(a.shape)} "
                      f"x finite {torch.isfinite(x).all().item()} h finite {torch.isfinite(h).all().item()} "
                      f"ht finite {torch.isfinite(ht).all().item()} rel err {err:.3e} "
                      f"x ptr {x.data_ptr() % 4096} a ptr {a.data_ptr() % 4096}", flush=True)
        return res

    def lora_dx(self, g, at, dx, p, seed, offset, acc):
        calls["dx"] += 1
        return Creal.lora_dx(g, at, dx, p, seed, offset, acc)


_native._C = Proxy()

from gke_ray_train_amd.models import build_llama, get_config  # noqa: E402
from gke_ray_train_amd.peft import LoraConfig, get_peft_model  # noqa: E402

cfg = get_config("llama2-7b", num_hidden_layers=int(os.environ.get("PROBE_LAYERS", "32")))
model = build_llama(cfg, device=dev, dtype=torch.bfloat16, seed=1234)
pm = get_peft_model(model, LoraConfig(r=64, lora_alpha=16, lora_dropout=0.1))
pm.train()
first = []


def hook(mod, inp, out):
    if first:
        return
    t = out if torch.is_tensor(out) else (out[0] if isinstance(out, (tuple, list)) else None)
    if torch.is_tensor(t) and t.is_floating_point() and not torch.isfinite(t).all().item():
        first.append(mod._probe_name)
        print("first non-finite module output:", mod._probe_name, flush=True)


for n, m in pm.named_modules():
    m._probe_name = n
    m.register_forward_hook(hook)
ids = torch.randint(0, cfg.vocab_size, (8, 1024), device=dev)
cap = {}
qkv = dict(pm.named_modules())["base_model.model.layers.0.self_attn.qkv_proj"]
qkv.register_forward_pre_hook(lambda m, inp: cap.setdefault("x", inp[0].detach().clone()))
loss = pm(ids, labels=ids)["loss"]
print("loss", loss.item(), "calls", calls, flush=True)
loss.backward()
torch.cuda.synchronize()
bad = [n for n, p in pm.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
print("non-finite grads:", len(bad), bad[:4], "calls", calls, flush=True)

# replay layer 0's fused qkv LoRA forward step by step
from gke_ray_train_amd.peft.lora import _base_weight  # noqa: E402
import torch.nn.functional as F  # noqa: E402
x2 = cap["x"].reshape(-1, cap["x"].shape[-1]).contiguous()
names = list(qkv.lora_A.keys())
As = [qkv.lora_A[n] for n in names]
Bs = [qkv.lora_B[n] for n in names]
acat = torch.cat(As, 0).detach()
fin = lambda t: torch.isfinite(t).all().item()  # noqa: E731
print("replay: x finite", fin(x2), "A finite", fin(acat), "B finite", all(fin(b) for b in Bs), "names", names,
      "spec", getattr(qkv, "spec", None), flush=True)
for mode in ("torch", "kernel"):
    y = F.linear(x2, _base_weight(qkv.base).detach())
    print(mode, "y after linear finite", fin(y), flush=True)
    if mode == "kernel":
        h, xd = Creal.lora_down(x2, acat, 0.1, 99, 0, True)
    else:
        xd = Creal.dropout_fwd_seeded(x2, 0.1, 99, 0)
        h = xd @ acat.t()
    print(mode, "h finite", fin(h), "h stride", h.stride(), "absmax", h.abs().max().item(), flush=True)
    r = qkv.r
    for i in range(len(names)):
        off = i * 4096
        y[:, off:off + 4096].addmm_(h[:, i * r:(i + 1) * r], Bs[i].detach().t(), alpha=qkv.scaling)
        print(mode, f"after addmm {i}: y finite", fin(y), flush=True)
    torch.cuda.synchronize()
