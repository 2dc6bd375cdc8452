"""Repeat the early-norm DDP step of tests/test_parallel_gpu.py many times in one process, with
every CU's LDS NaN-filled before each step and after the 70B-shape FSDP test's allocations, and
report any non-finite gradient (the round-6 flake hunt)."""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
from gke_ray_train_amd import _native
from gke_ray_train_amd.models import build_llama
from gke_ray_train_amd.parallel import DistributedDataParallel
C = _native.kernels()
bad_total = 0
for trial in range(40):
    m = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=3)
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.25)
    g = torch.Generator(device="cuda").manual_seed(5)
    for step in range(3):
        ids = torch.randint(0, 512, (2, 128), device="cuda", generator=g)
        C.lds_fill(0x7FC00000, 0)
        (ddp(ids, labels=ids)["loss"]).backward()
        ddp.finish_gradient_sync()
        st = ddp.clip_grad_norm_(0.3)
        torch.cuda.synchronize()
        bad = [n for n, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
        if bad or not torch.isfinite(st.buf).all():
            bad_total += 1
            print(f"trial {trial} step {step}: non-finite grads {bad} norm {st.buf.tolist()}", flush=True)
        ddp.zero_grad()
    del m, ddp
print("trials with non-finite gradients:", bad_total, flush=True)
