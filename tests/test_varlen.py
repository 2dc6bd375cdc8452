"""Padding-free packing (``ops.Varlen``): sequences concatenated on one token axis with per-sequence
causal attention and RoPE positions. Must equal running the sequences one by one: logits, loss and
gradients (CPU reference path here; the packed HIP attention kernels on the GPU)."""
import pytest
import torch

from gke_ray_train_amd.models import build_llama
from gke_ray_train_amd.ops import Varlen

LENS = [37, 64, 20, 129]


def _seqs(vocab, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(0, vocab, (n,), generator=g).to(dev) for n in LENS]


def _check_model(dev, dtype, tol):
    torch.manual_seed(0)
    m = build_llama("llama-tiny-gqa", device=dev, dtype=dtype, seed=3)
    seqs = _seqs(m.config.vocab_size, dev)
    vl = Varlen(LENS, dev)
    packed = torch.cat(seqs).view(1, -1)
    out = m(packed, labels=packed, varlen=vl, return_logits=True)
    ref_logits = torch.cat([m(s.view(1, -1), return_logits=True)["logits"][0] for s in seqs])
    err = (out["logits"][0].float() - ref_logits.float()).abs().max().item()
    assert err < tol, f"packed logits differ by {err}"
    # the packed mean loss = token-weighted mean of the per-sequence losses
    losses = [m(s.view(1, -1), labels=s.view(1, -1))["loss"] for s in seqs]
    n = [len(s) - 1 for s in seqs]
    ref = sum(l * k for l, k in zip(losses, n)) / sum(n)
    assert abs(out["loss"].item() - ref.item()) < tol * 5
    # gradients: packed backward vs the per-sequence backward of the same objective
    m.zero_grad()
    out["loss"].backward()
    g_packed = {k: p.grad.float().clone() for k, p in m.named_parameters()}
    m.zero_grad()
    ref2 = sum(m(s.view(1, -1), labels=s.view(1, -1))["loss"] * k for s, k in zip(seqs, n)) / sum(n)
    ref2.backward()
    for k, p in m.named_parameters():
        d = (g_packed[k] - p.grad.float()).norm() / p.grad.float().norm().clamp_min(1e-12)
        assert d < tol * 10, f"grad {k}: rel err {d.item():.3g}"


def test_varlen_model_matches_per_sequence_cpu():
    _check_model(torch.device("cpu"), torch.float32, 1e-4)


@pytest.mark.gpu
def test_varlen_model_matches_per_sequence_gpu():
    _check_model(torch.device("cuda", 0), torch.bfloat16, 3e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("hq,hkv", [(4, 4), (8, 2)])
def test_packed_attention_kernel_matches_fp32_per_sequence(hq, hkv):
    """The packed HIP kernels (fwd, dK/dV, dQ with the RoPE epilogue) against the fp32 math path
    run sequence by sequence, every element."""
    from gke_ray_train_amd import ops
    from gke_ray_train_amd.ops import _ref
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    lens = [300, 17, 128, 1, 255]
    vl = Varlen(lens, dev)
    T, D = vl.total, 128
    qkv = torch.randn(T, (hq + 2 * hkv) * D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    cos, sin = _ref.rope_tables(vl.max_len, D, device=dev)
    o = ops.rope_attention(qkv, cos, sin, 1, T, hq, hkv, D, causal=True, varlen=vl)
    do = torch.randn_like(o)
    (o.float() * do.float()).sum().backward()
    x = qkv.detach().float().requires_grad_()
    xr = x.view(T, hq + 2 * hkv, D)
    q = _ref.apply_rope(xr[:, :hq], cos, sin, vl.pos)
    k = _ref.apply_rope(xr[:, hq:hq + hkv], cos, sin, vl.pos)
    v = xr[:, hq + hkv:]
    outs = []
    for a, b in zip(vl.cu_host[:-1], vl.cu_host[1:]):
        outs.append(_ref.attention(q[a:b].unsqueeze(0), k[a:b].unsqueeze(0), v[a:b].unsqueeze(0), causal=True)[0])
    ref = torch.cat(outs).reshape(T, hq * D)
    (ref * do.float()).sum().backward()
    for got, want, what, tol in ((o, ref, "o", 2e-2), (qkv.grad, x.grad, "dqkv", 3e-2)):
        err = (got.float() - want).abs()
        bound = tol + tol * want.abs()
        assert (err <= 10 * bound).all(), f"{what}: worst {(err / bound).max().item():.1f}x tolerance"
        assert (err > bound).float().mean() < 1e-3, f"{what}: {(err > bound).float().mean().item():.2e} out of tol"
