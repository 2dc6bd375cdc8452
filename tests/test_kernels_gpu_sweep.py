"""Hypothesis-driven shape sweeps of the HIP kernels against fp32 PyTorch references (SURVEY §4
tier 4: edge shapes — rows not a multiple of the tile, odd sequence lengths, GQA ratios, padding,
row widths at the vector granularity). Derandomized with a fixed example budget so a GPU run is
bounded and reproducible."""
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

pytestmark = pytest.mark.gpu
DEV = "cuda"
SETTINGS = settings(max_examples=12, deadline=None, derandomize=True,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


@SETTINGS
@given(rows=st.integers(1, 300), d8=st.integers(1, 96), dtype=st.sampled_from([torch.bfloat16, torch.float32]))
def test_rmsnorm_sweep(rows, d8, dtype):
    from gke_ray_train_amd import ops
    d = 8 * d8
    g = torch.Generator(device=DEV).manual_seed(rows * 131 + d)
    x = torch.randn(rows, d, device=DEV, dtype=dtype, generator=g).requires_grad_()
    w = (1 + 0.1 * torch.randn(d, device=DEV, dtype=dtype, generator=g)).requires_grad_()
    y = ops.rms_norm(x, w, 1e-5)
    gy = torch.randn(y.shape, device=DEV, dtype=dtype, generator=g)
    (y.float() * gy.float()).sum().backward()
    xr, wr = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    (yr * gy.float()).sum().backward()
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    assert _rel(y, yr) < tol and _rel(x.grad, xr.grad) < 2 * tol and _rel(w.grad, wr.grad) < 4 * tol


@SETTINGS
@given(rows=st.integers(1, 200), f8=st.integers(1, 200), dtype=st.sampled_from([torch.bfloat16, torch.float32]))
def test_swiglu_sweep(rows, f8, dtype):
    from gke_ray_train_amd import ops
    f = 8 * f8
    g = torch.Generator(device=DEV).manual_seed(rows * 7 + f)
    gu = torch.randn(rows, 2 * f, device=DEV, dtype=dtype, generator=g).requires_grad_()
    y = ops.swiglu(gu)
    gy = torch.randn(y.shape, device=DEV, dtype=dtype, generator=g)
    (y.float() * gy.float()).sum().backward()
    gr = gu.detach().float().requires_grad_()
    a, u = gr.chunk(2, -1)
    yr = torch.nn.functional.silu(a) * u
    (yr * gy.float()).sum().backward()
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    assert _rel(y, yr) < tol and _rel(gu.grad, gr.grad) < tol


@SETTINGS
@given(B=st.integers(1, 3), S=st.integers(1, 300), hkv=st.sampled_from([1, 2, 4]), grp=st.sampled_from([1, 2, 4]),
       causal=st.booleans(), pad=st.booleans(), dtype=st.sampled_from([torch.bfloat16, torch.float32]))
def test_flash_attention_sweep(B, S, hkv, grp, causal, pad, dtype):
    from gke_ray_train_amd import ops
    from gke_ray_train_amd.ops import _ref
    hq, D = hkv * grp, 128
    g = torch.Generator(device=DEV).manual_seed(B * 1000 + S * 10 + hq)
    q = torch.randn(B, S, hq, D, device=DEV, dtype=dtype, generator=g).requires_grad_()
    k = torch.randn(B, S, hkv, D, device=DEV, dtype=dtype, generator=g).requires_grad_()
    v = torch.randn(B, S, hkv, D, device=DEV, dtype=dtype, generator=g).requires_grad_()
    sl = None
    if pad:
        sl = torch.randint(1, S + 1, (B,), device=DEV, generator=g).to(torch.int32)
    o = ops.flash_attention(q, k, v, causal=causal, seqlens_k=sl)
    do = torch.randn(o.shape, device=DEV, dtype=dtype, generator=g)
    (o.float() * do.float()).sum().backward()
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = _ref.attention(qr, kr, vr, causal=causal, seqlens_k=sl)
    (orf * do.float()).sum().backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 2e-4
    assert _rel(o, orf) < tol
    for a, b, n in ((q.grad, qr.grad, "dq"), (k.grad, kr.grad, "dk"), (v.grad, vr.grad, "dv")):
        if b.norm() > 0:
            assert _rel(a, b) < 2 * tol, n


@SETTINGS
@given(rows=st.integers(1, 257), V=st.sampled_from([512, 1000, 32000, 50257]), ignore=st.floats(0.0, 0.5))
def test_cross_entropy_sweep(rows, V, ignore):
    from gke_ray_train_amd import ops
    g = torch.Generator(device=DEV).manual_seed(rows + V)
    h = torch.randn(rows, 64, device=DEV, dtype=torch.bfloat16, generator=g).requires_grad_()
    w = (0.05 * torch.randn(V, 64, device=DEV, dtype=torch.bfloat16, generator=g)).requires_grad_()
    lab = torch.randint(0, V, (rows,), device=DEV, generator=g)
    lab[torch.rand(rows, device=DEV, generator=g) < ignore] = -100
    loss = ops.lm_head_cross_entropy(h, w, lab)
    loss.backward()
    hr, wr = h.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    lr = torch.nn.functional.cross_entropy(hr @ wr.t(), lab, ignore_index=-100)
    lr.backward()
    if (lab != -100).any():
        assert abs(float(loss.detach()) - float(lr.detach())) < 2e-2 * max(1.0, abs(float(lr.detach())))
        assert _rel(h.grad, hr.grad) < 3e-2 and _rel(w.grad, wr.grad) < 3e-2
