"""Reproduce an uninitialised read: fill the caching allocator's free blocks with NaN, then run the
early-norm DDP step of tests/test_parallel_gpu.py and report which gradients / activations are NaN."""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
from gke_ray_train_amd.models import build_llama
from gke_ray_train_amd.parallel import DistributedDataParallel
blocks = [torch.full((n,), float("nan"), device="cuda") for n in [1 << 20, 1 << 22, 1 << 24, 1 << 26] * 4]
blocks += [torch.full((n,), float("nan"), device="cuda") for n in [256, 1024, 4096, 16384, 65536, 131072, 200000] * 40]
del blocks  # cached, not returned: later empty() allocations see NaN
m = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=3)
ddp = DistributedDataParallel(m, bucket_cap_mb=0.25)
g = torch.Generator(device="cuda").manual_seed(5)
acts = {}
def hook(name):
    def f(mod, inp, out):
        o = out[0] if isinstance(out, (tuple, list)) else out
        if isinstance(o, dict):
            o = o.get("logits", o.get("loss"))
        if isinstance(o, torch.Tensor):
            acts.setdefault(name, []).append(bool(torch.isnan(o.float()).any()))
    return f
for n, mod in m.named_modules():
    if n.count(".") <= 3:
        mod.register_forward_hook(hook(n))
for step in range(2):
    ids = torch.randint(0, 512, (2, 128), device="cuda", generator=g)
    out = ddp(ids, labels=ids)
    print("step", step, "loss", float(out["loss"]), flush=True)
    bad_act = [k for k, v in acts.items() if v[-1]]
    print("NaN activations:", bad_act[:20], flush=True)
    out["loss"].backward()
    ddp.finish_gradient_sync()
    bad = [n for n, p in m.named_parameters() if p.grad is not None and torch.isnan(p.grad.float()).any()]
    none = [n for n, p in m.named_parameters() if p.grad is None]
    print("NaN grads:", bad[:30], "no grad:", none[:10], flush=True)
    for gi, gr in enumerate(ddp.grad_buffers()):
        nz = torch.isnan(gr.float()).nonzero().flatten()
        if nz.numel():
            print(f"group {gi}: {nz.numel()} NaN of {gr.numel()} first {nz[:8].tolist()}", flush=True)
    ddp.zero_grad()
