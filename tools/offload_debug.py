"""Diagnose serial vs overlapped offloaded AdamW on FSDP (world 1): determinism of each path and
where the first difference appears (after the first update, before any forward; or later)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.models.llama import LlamaForCausalLM, RMSNorm, get_config  # noqa: E402
from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel  # noqa: E402

cfg = get_config("llama-tiny-gqa")


def init(mod):
    with torch.no_grad():
        if isinstance(mod, (torch.nn.Linear, torch.nn.Embedding)):
            mod.weight.normal_(0, 0.02)
        elif isinstance(mod, RMSNorm):
            mod.weight.fill_(1.0)


def run(overlap, steps=3, sync=True):
    torch.manual_seed(0)
    m = LlamaForCausalLM(cfg, device="meta", dtype=torch.bfloat16)
    f = FullyShardedDataParallel(m, param_init_fn=init, device="cuda", cpu_offload=True, offload_chunk_elems=1 << 14)
    opt = f.build_optimizer(lr=1e-3, overlap=overlap, resident_fraction=0.0)
    g = torch.Generator(device="cuda").manual_seed(4)
    out = []
    for _ in range(steps):
        ids = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=g)
        loss = f(ids, labels=ids)["loss"]
        loss.backward()
        f.finish_gradient_sync()
        grads = (f.grad_store.clone(), f.rep_grad.clone())
        st = f.clip_grad_norm_(1.0)
        opt.step(grad_scale=st)
        f.zero_grad()
        if sync and hasattr(opt, "synchronize"):
            opt.synchronize()
            torch.cuda.synchronize()
        out.append((loss.item(), grads, f.shard_store.clone(), f.rep_flat.clone(), float(st.buf[0]), float(st.buf[1])))
    return out


a, a2, b, c = run(False), run(False), run(True), run(True, sync=False)
for name, x, y in (("serial vs serial", a, a2), ("serial vs overlap(sync)", a, b), ("serial vs overlap(nosync)", a, c)):
    for i, (u, v) in enumerate(zip(x, y)):
        print(name, "step", i, "loss", u[0], v[0], "grad_store eq", torch.equal(u[1][0], v[1][0]),
              "rep_grad eq", torch.equal(u[1][1], v[1][1]), "norm", u[4], v[4], "coef", u[5], v[5],
              "shard eq", torch.equal(u[2], v[2]), "rep eq", torch.equal(u[3], v[3]),
              "shard maxdiff", float((u[2].float() - v[2].float()).abs().max()), flush=True)
