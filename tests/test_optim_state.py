"""Optimizer checkpoint reload keeps fp32 moments (torch's load_state_dict casts state to
the parameter dtype/device, i.e. bf16 on the GPU for a bf16 model, and would put an offloaded
optimizer's host state in HBM). A reloaded optimizer must continue bit-identically."""
import pytest
import torch

from gke_ray_train_amd.ops.optim import FusedAdamW, OffloadedAdamW


def _params(dev, dtype, seed=0):
    g = torch.Generator().manual_seed(seed)
    ps = [torch.nn.Parameter(torch.randn(64, 32, generator=g).to(dev, dtype)),
          torch.nn.Parameter(torch.randn(128, generator=g).to(dev, dtype))]
    return ps


def _grads(ps, step):
    g = torch.Generator().manual_seed(100 + step)
    for p in ps:
        p.grad = torch.randn(p.shape, generator=g).to(p.device, p.dtype)


def _run(dev, dtype, opt_cls, steps_before=2, steps_after=2):
    ps = _params(dev, dtype)
    opt = opt_cls(ps, lr=1e-2, weight_decay=0.01)
    for s in range(steps_before):
        _grads(ps, s)
        opt.step()
    sd = opt.state_dict()
    # a fresh optimizer on an identical copy of the parameters, loaded from the checkpoint
    ps2 = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt2 = opt_cls(ps2, lr=1e-2, weight_decay=0.01)
    opt2.load_state_dict(sd)
    for p2 in ps2:
        st = opt2.state[p2]
        for k in ("exp_avg", "exp_avg_sq"):
            assert st[k].dtype == torch.float32, (k, st[k].dtype)
            if opt_cls._host_states:
                assert st[k].device.type == "cpu"
            else:
                assert st[k].device == p2.device
    for p, p2 in zip(ps, ps2):
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(opt.state[p][k].cpu(), opt2.state[p2][k].cpu())
    for s in range(steps_before, steps_before + steps_after):
        _grads(ps, s)
        _grads(ps2, s)
        opt.step()
        opt2.step()
    for p, p2 in zip(ps, ps2):
        assert torch.equal(p.detach().cpu(), p2.detach().cpu())
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(opt.state[p][k].cpu(), opt2.state[p2][k].cpu())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fused_adamw_reload_cpu(dtype):
    _run(torch.device("cpu"), dtype, FusedAdamW)


@pytest.mark.gpu
@pytest.mark.parametrize("opt_cls", [FusedAdamW, OffloadedAdamW])
def test_adamw_reload_gpu_bf16(opt_cls):
    _run(torch.device("cuda", 0), torch.bfloat16, opt_cls)
