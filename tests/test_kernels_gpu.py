"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 reference of the same op."""
import contextlib
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _C():
    from gke_ray_train_amd import _native
    return _native.kernels()


def _close(a, b, atol, rtol, what=""):
    a, b = a.float(), b.float()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol)
    assert not torch.isnan(a).any(), f"{what}: NaN in kernel output"
    assert bad.float().mean().item() < 1e-3, f"{what}: max err {err.max().item():.4g} (mean {err.mean().item():.3g})"
    # no element may be far off: a wrong row / tile edge fails even if it is < 0.1 % of the tensor
    worst = (err / tol).max().item()
    assert worst <= 10.0, f"{what}: an element is {worst:.1f}x its tolerance (max err {err.max().item():.4g})"


def test_native_loaded():
    C = _C()
    assert hasattr(C, "attn_fwd")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("d", [256, 4096, 2048 + 512])
def test_rmsnorm(dtype, d):
    from gke_ray_train_amd import ops
    torch.manual_seed(0)
    x = torch.randn(37, d, device=DEV, dtype=dtype, requires_grad=True)
    r = torch.randn(37, d, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(d, device=DEV, dtype=dtype)).requires_grad_()
    y, h = ops.add_rms_norm(x, r, w, 1e-5)
    gy = torch.randn_like(y)
    gh = torch.randn_like(h)
    (y.float() * gy.float()).sum().add((h.float() * gh.float()).sum()).backward()
    xr, rr, wr = (t.detach().float().requires_grad_() for t in (x, r, w))
    hr = xr + rr
    yr = hr * torch.rsqrt(hr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    (yr * gy.float()).sum().add((hr * gh.float()).sum()).backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    _close(y, yr, tol, tol, "rms y")
    _close(h, hr, tol, tol, "rms h")
    _close(x.grad, xr.grad, tol * 5, tol, "rms dx")
    _close(w.grad, wr.grad, tol * 20, tol * 2, "rms dw")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("fused_add", [False, True])
def test_rmsnorm_frozen_weight_dx_only(dtype, fused_add):
    """Frozen norm weight (LoRA / QLoRA): the dX-only backward gives the same dX bits as the full
    backward and no weight gradient."""
    from gke_ray_train_amd import ops
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(300, 4096, device=DEV, dtype=dtype, generator=g)
    r = torch.randn(300, 4096, device=DEV, dtype=dtype, generator=g)
    dy = torch.randn(300, 4096, device=DEV, dtype=dtype, generator=g)
    grads = {}
    for trainable in (True, False):
        w = (1 + 0.1 * torch.randn(4096, device=DEV, dtype=dtype, generator=torch.Generator(device=DEV).manual_seed(4)))
        w.requires_grad_(trainable)
        xi = x.clone().requires_grad_()
        if fused_add:
            y, h = ops.add_rms_norm(xi, r, w, 1e-5)
            (y.float() * dy.float()).sum().add(h.float().sum()).backward()
        else:
            (ops.rms_norm(xi, w, 1e-5).float() * dy.float()).sum().backward()
        grads[trainable] = (xi.grad, w.grad)
    assert torch.equal(grads[True][0], grads[False][0])
    assert grads[False][1] is None and grads[True][1] is not None


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_layernorm(dtype):
    from gke_ray_train_amd import ops
    torch.manual_seed(1)
    d = 2048
    x = torch.randn(64, d, device=DEV, dtype=dtype, requires_grad=True)
    r = torch.randn(64, d, device=DEV, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(d, device=DEV, dtype=dtype)).requires_grad_()
    b = (0.1 * torch.randn(d, device=DEV, dtype=dtype)).requires_grad_()
    y = ops.layer_norm(x, w, b, 1e-5, residual=r)
    gy = torch.randn_like(y)
    (y.float() * gy.float()).sum().backward()
    xr, rr, wr, br = (t.detach().float().requires_grad_() for t in (x, r, w, b))
    yr = torch.nn.functional.layer_norm(xr + rr, (d,), wr, br, 1e-5)
    (yr * gy.float()).sum().backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    _close(y, yr, tol, tol, "ln y")
    _close(x.grad, xr.grad, tol * 5, tol, "ln dx")
    _close(r.grad, rr.grad, tol * 5, tol, "ln dres")
    _close(w.grad, wr.grad, tol * 30, tol * 2, "ln dw")
    _close(b.grad, br.grad, tol * 30, tol * 2, "ln db")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,f,pad", [(6656, 14336, 0), (33, 688, 0), (257, 1024, 64)])
def test_swiglu_single_pass_kernels_match_grid_stride(dtype, rows, f, pad):
    """The single-pass SwiGLU kernels (32-bit indexing, one vector per thread) give the grid-stride
    kernels' forward (incl. a padded LoRA-tail row buffer) and backward bit for bit."""
    C = _C()
    g = torch.Generator(device=DEV).manual_seed(rows + f)
    gu = torch.randn(rows, 2 * f, device=DEV, dtype=dtype, generator=g)
    dout = torch.randn(rows, f, device=DEV, dtype=dtype, generator=g)
    out = []
    try:
        for fast in (1, 0):
            C.ew_set_fast(fast)
            y = C.swiglu_fwd(gu, pad)
            dgu = C.swiglu_bwd(gu, dout)
            torch.cuda.synchronize()
            out.append((y[:, :f].clone(), dgu))
    finally:
        C.ew_set_fast(1)
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_swiglu_gelu(dtype):
    from gke_ray_train_amd import ops
    torch.manual_seed(2)
    gu = torch.randn(33, 2 * 688, device=DEV, dtype=dtype, requires_grad=True)
    y = ops.swiglu(gu)
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    gr = gu.detach().float().requires_grad_()
    a, u = gr.chunk(2, -1)
    yr = torch.nn.functional.silu(a) * u
    (yr * g.float()).sum().backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    _close(y, yr, tol, tol, "swiglu")
    _close(gu.grad, gr.grad, tol, tol, "swiglu bwd")
    x = torch.randn(1024, 64, device=DEV, dtype=dtype, requires_grad=True)
    y = ops.gelu(x)
    (y.float() * x.detach().float()).sum().backward()
    xr = x.detach().float().requires_grad_()
    yr = torch.nn.functional.gelu(xr)
    (yr * xr.detach()).sum().backward()
    _close(y, yr, tol, tol, "gelu")
    _close(x.grad, xr.grad, tol, tol, "gelu bwd")


def test_dropout():
    from gke_ray_train_amd import ops
    x = torch.ones(1 << 16, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = ops.dropout(x, 0.1, True, seed=7)
    keep = (y != 0).float().mean().item()
    assert abs(keep - 0.9) < 0.01
    assert torch.allclose(y[y != 0].float(), torch.full_like(y[y != 0].float(), 1 / 0.9), atol=1e-2)
    y.float().sum().backward()
    assert torch.equal((x.grad != 0), (y != 0))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("offset", [0, 1, 3, 6, (1 << 40) + 5])
@pytest.mark.parametrize("n", [12345, 4096, 7])
def test_dropout_masks_match_host_hash(dtype, offset, n):
    """Every dropout entry point (mask-storing fwd, mask-free fwd, seeded bwd with and without
    accumulation) produces the keep pattern of the independent host reimplementation of the hash
    (ops/_ref.py::dropout_keep_mask) — including unaligned offsets (offset % 4 != 0, the per-element
    path of drop_keep_vec), the scalar tail (n % vector width != 0) and seeds above bit 40."""
    from gke_ray_train_amd.ops import _ref
    C = _C()
    p, seed = 0.3, (0x5DEECE66D << 20) | 0xABC
    ref = _ref.dropout_keep_mask(seed, offset, n, p).to(DEV)
    ones = torch.ones(n, device=DEV, dtype=dtype)
    y, mask = C.dropout_fwd(ones, p, seed, offset)
    assert torch.equal(mask.bool(), ref), "stored mask"
    assert torch.equal(y != 0, ref)
    assert torch.allclose(y[ref].float(), torch.full_like(y[ref].float(), 1 / (1 - p)), rtol=1e-2)
    assert torch.equal(C.dropout_fwd_seeded(ones, p, seed, offset) != 0, ref), "mask-free fwd"
    dx = torch.empty_like(ones)
    C.dropout_bwd_seeded(ones, dx, p, seed, offset, False)
    assert torch.equal(dx != 0, ref), "seeded bwd"
    acc = torch.full_like(ones, 2.0)
    C.dropout_bwd_seeded(ones, acc, p, seed, offset, True)
    expect = 2.0 + ref.to(dtype) / (1 - p)
    assert torch.allclose(acc.float(), expect.float(), rtol=1e-2), "seeded bwd accumulate"
    assert torch.equal(C.dropout_bwd(ones, mask, p) != 0, ref), "mask bwd"
    if n >= 4096:
        assert abs(ref.float().mean().item() - (1 - p)) < 0.03
    # a different seed gives a different mask; seeds differing only above bit 40 too
    assert not torch.equal(_ref.dropout_keep_mask(seed ^ (1 << 50), offset, n, p), ref.cpu()) or n < 64


def test_dropout_rejects_bad_p():
    C = _C()
    x = torch.ones(64, device=DEV, dtype=torch.bfloat16)
    for bad in (-0.1, 1.0, 1.5):
        with pytest.raises(RuntimeError):
            C.dropout_fwd(x, bad, 1, 0)
        with pytest.raises(RuntimeError):
            C.dropout_fwd_seeded(x, bad, 1, 0)
        with pytest.raises(RuntimeError):
            C.dropout_bwd_seeded(x, torch.empty_like(x), bad, 1, 0, False)


def test_lora_dropout_under_gradient_checkpointing():
    """LoRA input dropout inside a non-reentrant checkpoint: the recompute draws the same
    (seed, offset) (torch's CPU RNG state is restored by checkpoint), so the gradients equal
    those of the same step without checkpointing."""
    import torch.utils.checkpoint as ckpt
    from gke_ray_train_amd.ops.linear import Linear
    from gke_ray_train_amd.peft.lora import LoraConfig, LoraLinear
    torch.manual_seed(0)
    lin = Linear(256, 512, bias=False, device=DEV, dtype=torch.bfloat16)
    lin.weight.requires_grad_(False)
    mod = LoraLinear(lin, [("q_proj", 0, 512)], LoraConfig(r=16, lora_alpha=32, lora_dropout=0.3)).train()
    with torch.no_grad():
        mod.lora_B["q_proj"].normal_(0, 0.05)
    x0 = torch.randn(4, 64, 256, device=DEV, dtype=torch.bfloat16)
    dy = torch.randn(4, 64, 512, device=DEV, dtype=torch.bfloat16)
    grads = []
    for use_ckpt in (False, True):
        mod.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        torch.manual_seed(123)
        y = ckpt.checkpoint(mod, x, use_reentrant=False) if use_ckpt else mod(x)
        torch.manual_seed(999)  # the RNG moves on between forward and backward
        (y.float() * dy.float()).sum().backward()
        grads.append((x.grad.clone(), mod.lora_A["q_proj"].grad.clone(), mod.lora_B["q_proj"].grad.clone()))
    for a, b, what in zip(grads[0], grads[1], ("dx", "dA", "dB")):
        assert torch.equal(a, b), what


def test_rope():
    from gke_ray_train_amd.ops import _ref
    C = _C()
    torch.manual_seed(3)
    B, S, hq, hkv, D = 2, 40, 4, 2, 128
    T = B * S
    qkv = torch.randn(T, (hq + 2 * hkv) * D, device=DEV, dtype=torch.bfloat16)
    cos, sin = _ref.rope_tables(S, D, 10000.0, device=DEV)
    q, k = C.rope_fwd(qkv, cos, sin, None, hq, hkv, D, S)
    x = qkv.view(T, hq + 2 * hkv, D)
    qr = _ref.apply_rope(x[:, :hq].float(), cos, sin)
    kr = _ref.apply_rope(x[:, hq:hq + hkv].float(), cos, sin)
    _close(q, qr, 2e-2, 2e-2, "rope q")
    _close(k, kr, 2e-2, 2e-2, "rope k")
    dq = torch.randn_like(q)
    dk = torch.randn_like(k)
    dqkv = torch.zeros_like(qkv)
    C.rope_bwd(dq, dk, dqkv, cos, sin, None, hq, hkv, D, S)
    # inverse rotation == rotation by -theta
    qi = _ref.apply_rope(dq.float(), cos, -sin)
    _close(dqkv.view(T, -1, D)[:, :hq], qi, 2e-2, 2e-2, "rope bwd")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("T,S,hq,hkv,packed", [(8192, 1024, 32, 32, False), (600, 300, 32, 8, True), (37, 37, 4, 2, False)])
def test_rope_d128_kernel_matches_generic(dtype, T, S, hq, hkv, packed):
    """The D = 128 RoPE kernel (32-bit indexing, one 8-pair group per thread) gives the generic
    kernel's q / k and backward dqkv bit for bit, with and without per-token positions."""
    from gke_ray_train_amd.ops import _ref
    C = _C()
    D = 128
    g = torch.Generator(device=DEV).manual_seed(T + hq)
    qkv = torch.randn(T, (hq + 2 * hkv) * D, device=DEV, dtype=dtype, generator=g)
    cos, sin = _ref.rope_tables(S, D, 10000.0, device=DEV)
    cos, sin = cos.float().contiguous(), sin.float().contiguous()
    pos = torch.cat([torch.arange(S, device=DEV), torch.arange(T - S, device=DEV)]).int() if packed else None
    dq = torch.randn(T, hq * D, device=DEV, dtype=dtype, generator=g)
    dk = torch.randn(T, hkv * D, device=DEV, dtype=dtype, generator=g)
    out = []
    try:
        for fast in (1, 0):
            C.ew_set_fast(fast)
            q, k = C.rope_fwd(qkv, cos, sin, pos, hq, hkv, D, S)
            dqkv = torch.full_like(qkv, float("nan"))
            C.rope_bwd(dq, dk, dqkv, cos, sin, pos, hq, hkv, D, S)
            torch.cuda.synchronize()
            out.append((q, k, dqkv[:, :(hq + hkv) * D].clone()))
    finally:
        C.ew_set_fast(1)
    for name, a, b in zip(("q", "k", "dqk"), *out):
        assert torch.equal(a, b), name


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("V", [32000, 283])
def test_cross_entropy(dtype, V):
    from gke_ray_train_amd import ops
    torch.manual_seed(4)
    N = 67
    logits = (3 * torch.randn(N, V, device=DEV, dtype=torch.float32)).to(dtype).requires_grad_()
    labels = torch.randint(0, V, (N,), device=DEV)
    labels[::7] = -100
    loss = ops.cross_entropy(logits, labels)
    loss.backward()
    lr = logits.detach().float().requires_grad_()
    ref = torch.nn.functional.cross_entropy(lr, labels, ignore_index=-100)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-3 * max(1.0, abs(ref.item()))
    _close(logits.grad, lr.grad, 1e-4 if dtype == torch.float32 else 3e-3, 2e-2, "ce grad")


def test_cross_entropy_llama3_vocab():
    """V = 128256 (Llama-3.1 vocabulary of the SFT job), M = 2048 tokens, bf16 logits vs fp32."""
    from gke_ray_train_amd import ops
    torch.manual_seed(6)
    N, V = 2048, 128256
    logits = (2 * torch.randn(N, V, device=DEV)).to(torch.bfloat16).requires_grad_()
    labels = torch.randint(0, V, (N,), device=DEV)
    labels[::5] = -100
    labels[-3:] = V - 1
    loss = ops.cross_entropy(logits, labels)
    loss.backward()
    lr = logits.detach().float().requires_grad_()
    ref = torch.nn.functional.cross_entropy(lr, labels, ignore_index=-100)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-3 * max(1.0, abs(ref.item()))
    _close(logits.grad, lr.grad, 1e-8, 2e-2, "ce V=128256 grad")
    assert torch.all(logits.grad[labels == -100] == 0), "ignored rows must get zero gradient"


def test_lm_head_ce():
    from gke_ray_train_amd import ops
    torch.manual_seed(5)
    N, d, V = 64, 256, 1000
    h = torch.randn(N, d, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    W = (0.05 * torch.randn(V, d, device=DEV, dtype=torch.bfloat16)).requires_grad_()
    lab = torch.randint(0, V, (N,), device=DEV)
    loss = ops.lm_head_cross_entropy(h, W, lab)
    loss.backward()
    hr, Wr = h.detach().float().requires_grad_(), W.detach().float().requires_grad_()
    ref = torch.nn.functional.cross_entropy(hr @ Wr.t(), lab)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 2e-2
    _close(h.grad, hr.grad, 2e-3, 5e-2, "lmce dh")
    _close(W.grad, Wr.grad, 2e-3, 5e-2, "lmce dW")


def test_lm_head_ce_row_weights():
    """Weighted-sum loss (fused grad accumulation): per-row scale goes through the CE backward."""
    from gke_ray_train_amd import ops
    torch.manual_seed(15)
    N, d, V = 96, 256, 1000
    h = torch.randn(N, d, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    W = (0.05 * torch.randn(V, d, device=DEV, dtype=torch.bfloat16)).requires_grad_()
    lab = torch.randint(0, V, (N,), device=DEV)
    lab[::7] = -100
    rw = torch.rand(N, device=DEV) / 8
    loss = ops.lm_head_cross_entropy(h, W, lab, row_weights=rw)
    loss.backward()
    hr, Wr = h.detach().float().requires_grad_(), W.detach().float().requires_grad_()
    rows = torch.nn.functional.cross_entropy(hr @ Wr.t(), lab, reduction="none")
    ref = (rows * rw * (lab != -100)).sum()
    ref.backward()
    assert abs(loss.item() - ref.item()) < 2e-2 * max(1.0, abs(ref.item()))
    _close(h.grad, hr.grad, 2e-3, 5e-2, "lmce-w dh")
    _close(W.grad, Wr.grad, 2e-3, 5e-2, "lmce-w dW")


@pytest.mark.parametrize("pdt", [torch.bfloat16, torch.float32])
def test_adamw_and_clip(pdt):
    from gke_ray_train_amd.ops import FusedAdamW, clip_grad_norm_, _ref
    torch.manual_seed(6)
    n = 10007
    p = torch.randn(n, device=DEV, dtype=pdt)
    g = torch.randn(n, device=DEV, dtype=pdt) * 3
    P = torch.nn.Parameter(p.clone())
    P.grad = g.clone()
    opt = FusedAdamW([P], lr=1e-2, weight_decay=0.01)
    st = clip_grad_norm_([P], 1.0)
    norm = g.float().norm()
    assert abs(st.norm.item() - norm.item()) < 1e-3 * norm.item()
    opt.step(grad_scale=st)
    pr = p.float().clone()
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    _ref.adamw_(pr, g.float(), m, v, 1, 1e-2, 0.9, 0.999, 1e-8, 0.01, grad_scale=min(1.0, 1.0 / (norm.item() + 1e-6)))
    _close(P.data, pr, 1e-2 if pdt == torch.bfloat16 else 1e-6, 1e-2 if pdt == torch.bfloat16 else 1e-5, "adamw")
    _close(opt.state[P]["exp_avg"], m, 1e-6, 1e-4, "adamw m")


@pytest.mark.parametrize("sr", [False, True])
def test_adamw_bf16_stochastic_rounding(sr):
    """bf16 params without a master copy: an update of 1/4 of the bf16 spacing below 1.0 (lr 2^-10
    on p = 1, first Adam step |update| = lr) rounds away under round-to-nearest but is kept in
    expectation under stochastic rounding (mean within a few sigma, values only the two neighbours)."""
    from gke_ray_train_amd.ops import FusedAdamW
    n = 1 << 20
    P = torch.nn.Parameter(torch.ones(n, device=DEV, dtype=torch.bfloat16))
    P.grad = torch.ones(n, device=DEV, dtype=torch.bfloat16)
    opt = FusedAdamW([P], lr=2.0 ** -10, weight_decay=0.0, stochastic_rounding=sr)
    opt.step()
    x = P.data.float()
    if not sr:
        assert torch.equal(x, torch.ones_like(x))
        return
    lo = 1.0 - 2.0 ** -8
    assert bool(((x == 1.0) | (x == lo)).all())
    mean = x.mean().item()
    sigma = 2.0 ** -8 * (0.25 * 0.75) ** 0.5 / n ** 0.5
    assert abs(mean - (1.0 - 2.0 ** -10)) < 6 * sigma, (mean, 1.0 - 2.0 ** -10)


@pytest.mark.parametrize("sr", [0.0, 1.0])
def test_adamw_slices_and_alignment_bit_identical(sr):
    """The 8-wide AdamW path (16-byte aligned operands), the 4-wide fallback (a slice starting 4
    elements in: 8-byte aligned bf16) and chunked launches with index offsets all produce the same
    bits as one launch over the whole buffer (the stochastic-rounding stream is keyed by the flat
    index), including a scalar tail (n % 8 != 0)."""
    C = _C()
    n = (1 << 16) + 13
    g0 = torch.Generator(device=DEV).manual_seed(5)
    p0 = torch.randn(n, device=DEV, generator=g0).to(torch.bfloat16)
    gr = torch.randn(n, device=DEV, generator=g0).to(torch.bfloat16)
    m0 = torch.randn(n, device=DEV, generator=g0) * 0.01
    v0 = torch.rand(n, device=DEV, generator=g0) * 0.01
    hyper = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.01, 0.1, 0.001, 1.0, sr, 3.0], device=DEV)

    def run(cuts):
        p, m, v = p0.clone(), m0.clone(), v0.clone()
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            C.adamw(p[lo:hi], gr[lo:hi], m[lo:hi], v[lo:hi], None, hyper, None, 0, lo)
        return p, m, v

    whole = run([0, n])
    for cuts in ([0, 4, n], [0, 64, 1028, n], [0, 8, 12, n]):
        got = run(cuts)
        for a, b, what in zip(got, whole, ("p", "m", "v")):
            assert torch.equal(a, b), f"cuts {cuts}: {what} differs"


@pytest.mark.parametrize("rows", [192, 512])
@pytest.mark.parametrize("sr", [0.0, 1.0])
def test_adamw_t_matches_flat_update_and_transposes(sr, rows):
    """adamw_t (update of a [rows, cols] weight that also writes W^T) == the flat AdamW kernel on
    the same data (same rounding stream for a matching index offset), and pt == p^T exactly."""
    C = _C()
    torch.manual_seed(8)
    cols, off = 384, 128
    p0 = torch.randn(rows, cols, device=DEV).bfloat16()
    g = torch.randn(rows, cols, device=DEV).bfloat16()
    m0 = torch.randn(rows, cols, device=DEV).abs() * 0.01
    v0 = torch.rand(rows, cols, device=DEV) * 1e-3
    hyper = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.01, 0.1, 0.001, 1.0, sr, 3.0], device=DEV)
    gsc = torch.tensor([1.0, 0.5], device=DEV)
    pa, ma, va = p0.clone(), m0.clone(), v0.clone()
    C.adamw(pa.view(-1), g.view(-1), ma.view(-1), va.view(-1), None, hyper, gsc, 0, off)
    pb, mb, vb = p0.clone(), m0.clone(), v0.clone()
    pt = torch.empty(cols, rows, device=DEV, dtype=torch.bfloat16)
    C.adamw_t(pb, g, mb, vb, hyper, gsc, pt, off)
    torch.cuda.synchronize()
    assert torch.equal(pt, pb.t()), "transpose"
    _close(mb, ma, 1e-7, 1e-6, "adamw_t m")
    _close(vb, va, 1e-9, 1e-6, "adamw_t v")
    ulp = (pa.float() - pb.float()).abs() / pa.float().abs().clamp_min(1e-3)
    assert (ulp > 1e-2).float().mean().item() < 1e-3, "adamw_t params"


def test_nf4_roundtrip():
    from gke_ray_train_amd import ops
    from gke_ray_train_amd.ops import _ref
    torch.manual_seed(7)
    w = torch.randn(4096 * 64, device=DEV, dtype=torch.bfloat16)
    q, a = ops.nf4_quantize(w, 64)
    qr, ar = _ref.nf4_quantize(w.cpu(), 64)
    assert torch.allclose(a.cpu(), ar, rtol=1e-6)
    assert (q.cpu() != qr).float().mean().item() < 1e-3
    wd = ops.nf4_dequantize(q, a, w.numel(), 64, torch.bfloat16)
    wr = _ref.nf4_dequantize(qr, ar, w.numel(), 64, torch.bfloat16)
    _close(wd.cpu(), wr, 1e-2, 1e-2, "nf4 dequant")
    rel = (wd.float() - w.float()).norm() / w.float().norm()
    assert rel < 0.15


def _attn_case(B, Sq, Sk, Hq, Hkv, causal, seqlens=None, strided=False, dropout_p=0.0, dtype=torch.bfloat16,
               D=128):
    from gke_ray_train_amd import ops
    from gke_ray_train_amd.ops import _ref
    torch.manual_seed(8)
    if strided:
        qkv = torch.randn(B, Sq, Hq + 2 * Hkv, D, device=DEV, dtype=dtype)
        q = qkv[:, :, :Hq].detach().requires_grad_()
        base = torch.randn(B, Sk, 2 * Hkv, D, device=DEV, dtype=dtype)
        k = base[:, :, :Hkv]
        v = base[:, :, Hkv:]
        k = k.detach().requires_grad_()
        v = v.detach().requires_grad_()
    else:
        q = torch.randn(B, Sq, Hq, D, device=DEV, dtype=dtype, requires_grad=True)
        k = torch.randn(B, Sk, Hkv, D, device=DEV, dtype=dtype, requires_grad=True)
        v = torch.randn(B, Sk, Hkv, D, device=DEV, dtype=dtype, requires_grad=True)
    sl = None if seqlens is None else torch.tensor(seqlens, device=DEV, dtype=torch.int32)
    o = ops.flash_attention(q, k, v, causal=causal, seqlens_k=sl, dropout_p=dropout_p, seed=1234)
    do = torch.randn_like(o)
    (o.float() * do.float()).sum().backward()
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = _ref.attention(qr, kr, vr, causal=causal, seqlens_k=sl, dropout_p=dropout_p, seed=1234)
    (orf * do.float()).sum().backward()
    valid = torch.ones(B, Sq, dtype=torch.bool, device=DEV)
    tol = (2e-2, 3e-2) if dtype == torch.bfloat16 else (2e-4, 5e-4)  # fp32: exact-f32 MFMA vs fp32 math
    _close(o, orf, tol[0], tol[0], "attn o")
    _close(q.grad, qr.grad, tol[1], tol[1], "attn dq")
    _close(k.grad, kr.grad, tol[1], tol[1], "attn dk")
    _close(v.grad, vr.grad, tol[1], tol[1], "attn dv")


@pytest.mark.parametrize("case", [
    dict(B=2, Sq=256, Sk=256, Hq=4, Hkv=4, causal=True),
    dict(B=1, Sq=200, Sk=200, Hq=4, Hkv=2, causal=True),
    dict(B=2, Sq=130, Sk=130, Hq=2, Hkv=2, causal=False),
    dict(B=1, Sq=64, Sk=192, Hq=2, Hkv=1, causal=True),
    dict(B=2, Sq=256, Sk=256, Hq=4, Hkv=2, causal=True, strided=True),
    dict(B=2, Sq=160, Sk=160, Hq=2, Hkv=2, causal=False, seqlens=[160, 77]),
    dict(B=2, Sq=256, Sk=256, Hq=4, Hkv=2, causal=True, dropout_p=0.1),
    dict(B=1, Sq=200, Sk=200, Hq=2, Hkv=2, causal=True, dropout_p=0.3),
])
def test_flash_attention(case):
    _attn_case(**case)


@pytest.mark.parametrize("case", [
    dict(B=8, Sq=1024, Sk=1024, Hq=32, Hkv=32, causal=True),                      # Llama-2-7B bench step
    dict(B=2, Sq=2048, Sk=2048, Hq=32, Hkv=8, causal=True),                       # Llama-3.1 GQA 32:8
    dict(B=2, Sq=1024, Sk=1024, Hq=32, Hkv=8, causal=True, seqlens=[1024, 611]),  # SFT right padding
], ids=["llama2_7b_b8_s1024", "gqa_s2048", "gqa_padded"])
def test_flash_attention_production_shapes(case):
    """The production shapes against the fp32 math path, every element."""
    _attn_case(**case)


@pytest.mark.parametrize("case", [
    dict(B=2, Sq=256, Sk=256, Hq=4, Hkv=4, causal=True),
    dict(B=1, Sq=200, Sk=200, Hq=4, Hkv=2, causal=True, D=64),
    dict(B=2, Sq=130, Sk=130, Hq=2, Hkv=2, causal=False),
    dict(B=1, Sq=64, Sk=192, Hq=2, Hkv=1, causal=True, D=64),
    dict(B=2, Sq=256, Sk=256, Hq=4, Hkv=2, causal=True, strided=True),
    dict(B=2, Sq=160, Sk=160, Hq=2, Hkv=2, causal=False, seqlens=[160, 77]),
    dict(B=2, Sq=256, Sk=256, Hq=4, Hkv=4, causal=True, dropout_p=0.1),
    dict(B=1, Sq=200, Sk=200, Hq=2, Hkv=2, causal=True, dropout_p=0.3, D=64),
])
def test_flash_attention_fp32(case):
    """exact-fp32 kernels (attention_f32.hip, BasicLLM's reference dtype) vs the fp32 math path"""
    _attn_case(dtype=torch.float32, **case)


@pytest.mark.parametrize("fused_bwd", [True, False])
@pytest.mark.parametrize("B,S,hq,hkv", [(2, 192, 4, 2), (1, 1024, 4, 4)])
def test_rope_attention_fused(fused_bwd, B, S, hq, hkv, monkeypatch):
    """RoPE + flash attention vs fp32 math; fused_bwd: the backward kernels' epilogues undo the
    RoPE and write dQ / dK straight into dqkv (no rope_bwd pass)."""
    from gke_ray_train_amd import ops
    from gke_ray_train_amd.ops import _ref
    from gke_ray_train_amd.ops import fused as F_
    monkeypatch.setattr(F_, "_ROPE_BWD_FUSED", fused_bwd)
    torch.manual_seed(9)
    D = 128
    qkv = torch.randn(B * S, (hq + 2 * hkv) * D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    cos, sin = _ref.rope_tables(S, D, 10000.0, device=DEV)
    o = ops.rope_attention(qkv, cos, sin, B, S, hq, hkv, D)
    g = torch.randn_like(o)
    (o.float() * g.float()).sum().backward()
    xr = qkv.detach().float().requires_grad_()
    x = xr.view(B * S, hq + 2 * hkv, D)
    q = _ref.apply_rope(x[:, :hq], cos, sin).view(B, S, hq, D)
    k = _ref.apply_rope(x[:, hq:hq + hkv], cos, sin).view(B, S, hkv, D)
    v = x[:, hq + hkv:].reshape(B, S, hkv, D)
    orf = _ref.attention(q, k, v, causal=True).reshape(B * S, hq * D)
    (orf * g.float()).sum().backward()
    _close(o, orf, 2e-2, 2e-2, "rope-attn o")
    _close(qkv.grad, xr.grad, 3e-2, 3e-2, "rope-attn dqkv")


def test_llama_tiny_matches_reference_math():
    """Whole-model parity: native kernels vs the CPU reference path on the same weights."""
    from gke_ray_train_amd.models import build_llama
    torch.manual_seed(10)
    m = build_llama("llama-tiny-gqa", device=DEV, dtype=torch.bfloat16, seed=1)
    ids = torch.randint(0, m.config.vocab_size, (2, 128), device=DEV)
    loss = m(ids, labels=ids)["loss"]
    loss.backward()
    g_native = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    mc = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32, seed=None)
    mc.load_state_dict({k: v.float().cpu() for k, v in m.state_dict().items()})
    lc = mc(ids.cpu(), labels=ids.cpu())["loss"]
    lc.backward()
    assert abs(loss.item() - lc.item()) < 2e-2 * max(1.0, lc.item())
    for n, p in mc.named_parameters():
        a, b = g_native[n].cpu(), p.grad
        rel = (a - b).norm() / (b.norm() + 1e-8)
        assert rel < 0.08, f"{n}: rel grad err {rel:.3f}"


@pytest.mark.parametrize("R,P,Q,strided", [(64, 256, 256, False), (1024, 768, 512, False), (2048, 512, 1280, True),
                                          (8192, 256, 256, False), (96, 512, 256, False)])
def test_gemm_wgrad(R, P, Q, strided):
    mode = 0
    """Hand-written MFMA wgrad GEMM vs an fp32 reference, overwrite and accumulate (beta=1)."""
    C = _C()
    g = torch.Generator(device="cuda").manual_seed(R + P + Q)
    xs = torch.randn(R, P + (64 if strided else 0), device="cuda", generator=g).bfloat16()
    ys = torch.randn(R, Q + (128 if strided else 0), device="cuda", generator=g).bfloat16()
    x, y = xs[:, :P], ys[:, :Q]
    ref = x.float().t() @ y.float()
    out = torch.full((P, Q), float("nan"), device="cuda", dtype=torch.bfloat16)
    if R % 64:
        assert not C.gemm_wgrad(x, y, out, False, mode)
        return
    assert C.gemm_wgrad(x, y, out, False, mode)
    tol = 2e-2 * ref.abs().max().item() + 1e-2
    assert (out.float() - ref).abs().max().item() < tol
    base = torch.randn(P, Q, device="cuda", generator=g).bfloat16()
    out2 = base.clone()
    assert C.gemm_wgrad(x, y, out2, True, mode)
    assert (out2.float() - (ref + base.float())).abs().max().item() < tol
    # tiles that do not divide are refused (the caller falls back to hipBLASLt)
    assert not C.gemm_wgrad(x[:, : P - 8], y, torch.empty(P - 8, Q, device="cuda", dtype=torch.bfloat16), False)


def test_wgrad_helper_fallback_and_native():
    from gke_ray_train_amd.ops.linear import wgrad
    dy = torch.randn(512, 384, device="cuda").bfloat16()   # 384 is not a multiple of 256 -> hipBLASLt
    x = torch.randn(512, 512, device="cuda").bfloat16()
    ref = dy.float().t() @ x.float()
    assert (wgrad(dy, x).float() - ref).abs().max().item() < 0.05 * ref.abs().max().item()
    dy = torch.randn(512, 512, device="cuda").bfloat16()
    ref = dy.float().t() @ x.float()
    assert (wgrad(dy, x).float() - ref).abs().max().item() < 0.05 * ref.abs().max().item()


def test_direct_grad_linear_transpose_placements_agree(monkeypatch):
    """X^T taken in the forward (saved instead of X) and dY^T at the top of the backward give the
    same dX / dW bits as the transposes inside wgrad, into a gradient slot over two accumulating
    micro-steps, and match the fp32 math."""
    from gke_ray_train_amd.ops import linear as L
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(2, 192, 512, device=DEV, generator=g).bfloat16()
    w = (torch.randn(384, 512, device=DEV, generator=g) * 0.05).bfloat16()
    dys = [torch.randn(2, 192, 384, device=DEV, generator=g).bfloat16() for _ in range(2)]
    res = {}
    for xt_fwd, dyt_first in ((False, False), (True, False), (True, True)):
        monkeypatch.setattr(L, "_WGRAD_XT_FWD", xt_fwd)
        monkeypatch.setattr(L, "_WGRAD_DYT_FIRST", dyt_first)
        wp = torch.nn.Parameter(w.clone())
        wp._grt_slot = L.GradSlot(torch.empty_like(w), lambda p: None)
        dxs = []
        for dy in dys:
            xi = x.clone().requires_grad_()
            y = L.linear(xi, wp)
            y.backward(dy)
            dxs.append(xi.grad)
        res[(xt_fwd, dyt_first)] = (dxs, wp._grt_slot.view.clone())
    base = res[(False, False)]
    for k, (dxs, dw) in res.items():
        assert all(torch.equal(a, b) for a, b in zip(dxs, base[0])), k
        assert torch.equal(dw, base[1]), k
    ref = sum(dy.reshape(-1, 384).float().t() @ x.reshape(-1, 512).float() for dy in dys)
    assert (base[1].float() - ref).abs().max().item() < 0.02 * ref.abs().max().item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_embedding_fwd_bwd(dtype):
    """Gather forward and the one-pass segmented backward (zero-fill of unhit rows, duplicates,
    accumulate mode) against torch's embedding / index_add in fp32."""
    C = _C()
    V, d, n = 1000, 256, 4096
    g = torch.Generator(device=DEV).manual_seed(5)
    w = torch.randn(V, d, device=DEV, generator=g).to(dtype)
    ids = torch.randint(0, 300, (n,), device=DEV, generator=g)  # rows 300..999 never hit
    out = C.embedding_fwd(ids, w)
    assert torch.equal(out, torch.nn.functional.embedding(ids, w))
    dy = torch.randn(n, d, device=DEV, generator=g).to(dtype)
    ref = torch.zeros(V, d, device=DEV).index_add_(0, ids, dy.float())
    dw = torch.full((V, d), float("nan"), device=DEV, dtype=dtype)
    C.embedding_bwd(dy, ids, dw, False)
    _close(dw, ref, 2e-2, 2e-2, "embedding dW")
    base = torch.randn(V, d, device=DEV, generator=g).to(dtype)
    dw2 = base.clone()
    C.embedding_bwd(dy, ids, dw2, True)
    _close(dw2, ref + base.float(), 3e-2, 2e-2, "embedding dW accumulate")


def test_embedding_module_autograd(monkeypatch):
    from gke_ray_train_amd.ops import linear as L
    monkeypatch.setattr(L, "_NATIVE_EMBEDDING", True)
    e = L.Embedding(512, 128, device=DEV, dtype=torch.bfloat16)
    ids = torch.randint(0, 512, (4, 64), device=DEV)
    y = e(ids)
    y.float().pow(2).sum().backward()
    ref = torch.zeros(512, 128, device=DEV).index_add_(0, ids.view(-1), 2 * y.detach().float().view(-1, 128))
    _close(e.weight.grad, ref, 2e-2, 2e-2, "Embedding module grad")


@pytest.mark.parametrize("engine", ["none", "ddp", "ddp_accum"])
@pytest.mark.parametrize("targets", ["qv", "qkv"])
@pytest.mark.parametrize("nf4", [False, True])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_fused_lora_matches_reference(nf4, p, targets, engine):
    """The fused LoRA op (epilogue accumulation, seeded dropout regenerated in backward, in-place
    dX accumulation) equals the unfused formula y = W x + s * B_i A_i drop(x) per target slice.
    engine=ddp: the adapters sit in the DDP flat buffers, so A_cat is a view of them and dA / dB are
    written by the GEMMs straight into the gradient slots; ddp_accum: two micro-steps (the first
    under no_sync) accumulate into the slots."""
    from gke_ray_train_amd.ops.linear import Linear
    from gke_ray_train_amd.peft.lora import LoraConfig, LoraLinear
    from gke_ray_train_amd.peft.quant import BitsAndBytesConfig, NF4Linear
    torch.manual_seed(0)
    lin = Linear(256, 768, bias=False, device=DEV, dtype=torch.bfloat16)
    lin.slices = [("q_proj", 256), ("k_proj", 256), ("v_proj", 256)]
    base = NF4Linear.from_linear(lin, BitsAndBytesConfig()) if nf4 else lin
    for q in base.parameters():
        q.requires_grad_(False)
    cfg = LoraConfig(r=16, lora_alpha=32, lora_dropout=p)
    tg = [("q_proj", 0), ("v_proj", 512)] if targets == "qv" else [("q_proj", 0), ("k_proj", 256), ("v_proj", 512)]
    mod = LoraLinear(base, [(n, off, 256) for n, off in tg], cfg).train()
    names = [n for n, _ in tg]
    with torch.no_grad():
        for n in names:
            mod.lora_B[n].normal_(0, 0.05)
    x = torch.randn(4, 64, 256, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    from gke_ray_train_amd.ops import _ref
    fwd, eng, reps = mod, None, 1
    if engine != "none":
        from gke_ray_train_amd.parallel import DistributedDataParallel
        fwd = eng = DistributedDataParallel(mod)
        reps = 2 if engine == "ddp_accum" else 1
    rng = torch.get_rng_state()
    dy = None
    for rep in range(reps):
        ctx = eng.no_sync(rep < reps - 1) if eng is not None else contextlib.nullcontext()
        with ctx:
            y = fwd(x)
            dy = torch.randn_like(y) if dy is None else dy
            (y.float() * dy.float()).sum().backward()
    if eng is not None:
        eng.finish_gradient_sync()
        assert all(getattr(q, "_grt_slot", None) is not None for q in mod.direct_grad_params())
        from gke_ray_train_amd.peft.lora import _packed
        assert _packed([mod.lora_A[n] for n in names]) is not None  # the no-copy A_cat view path ran
    # reference in fp32; the mask from the host reimplementation of the hash with the seed the op
    # drew from torch's CPU generator (ops/fused.py::dropout_seed_offset)
    # (one seed per micro-step: each forward draws its own, so the reference regenerates every mask)
    torch.set_rng_state(rng)
    x2 = x.detach().view(-1, 256).float().requires_grad_()
    w = (base.dequantize() if nf4 else lin.weight).detach().float()
    A = {n: mod.lora_A[n].detach().float().requires_grad_() for n in names}
    B = {n: mod.lora_B[n].detach().float().requires_grad_() for n in names}
    for rep in range(reps):
        seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
        if p > 0:
            keep = _ref.dropout_keep_mask(seed, 0, x2.numel(), p).to(DEV).view_as(x2).float()
            xd = x2 * keep / (1 - p)
        else:
            xd = x2
        yr = x2 @ w.t()
        yr = yr.clone()
        for n, off in tg:
            yr[:, off:off + 256] = yr[:, off:off + 256] + cfg.scaling * (xd @ A[n].t()) @ B[n].t()
        (yr * dy.view(-1, 768).float()).sum().backward()
    _close(y.view(-1, 768), yr, 3e-2, 3e-2, "lora y")
    _close(x.grad.view(-1, 256), x2.grad, 3e-2, 3e-2, "lora dx")
    for n in names:
        # adapter grads are reductions over all tokens of bf16 intermediates (as in PEFT under bf16):
        # compare by relative Frobenius error
        for got, ref, what in ((mod.lora_A[n].grad, A[n].grad, "dA"), (mod.lora_B[n].grad, B[n].grad, "dB")):
            rel = (got.float() - ref).norm() / ref.norm().clamp_min(1e-6)
            assert rel < 2e-2, f"lora {what} {n}: rel err {rel.item():.3g}"


def test_lora_fp32_adapters_take_the_gemm_path():
    """fp32 base + adapters with >= 256 tokens: the bf16-only HIP adapter kernels must be bypassed
    (ADVICE r2), and the result equals the fp32 formula."""
    from gke_ray_train_amd.ops.linear import Linear
    from gke_ray_train_amd.peft.lora import LoraConfig, LoraLinear
    torch.manual_seed(0)
    lin = Linear(256, 256, bias=False, device=DEV, dtype=torch.float32)
    lin.weight.requires_grad_(False)
    cfg = LoraConfig(r=16, lora_alpha=32, lora_dropout=0.0)
    mod = LoraLinear(lin, [("q_proj", 0, 256)], cfg).train()
    with torch.no_grad():
        mod.lora_B["q_proj"].normal_(0, 0.05)
    x = torch.randn(512, 256, device=DEV, requires_grad=True)
    y = mod(x)
    y.sum().backward()
    A, B = mod.lora_A["q_proj"].detach(), mod.lora_B["q_proj"].detach()
    yr = x.detach() @ lin.weight.t() + cfg.scaling * (x.detach() @ A.t()) @ B.t()
    _close(y, yr, 1e-4, 1e-4, "lora fp32 y")
    assert mod.lora_A["q_proj"].grad is not None and mod.lora_A["q_proj"].grad.dtype == torch.float32


@pytest.mark.parametrize("M,K,R,p,offset,strided", [
    (256, 256, 32, 0.0, 0, False), (200, 512, 64, 0.1, 0, False), (77, 1024, 192, 0.1, 8, True),
    (1024, 4096, 128, 0.1, 0, False), (33, 128, 256, 0.5, 4, False), (6144, 14336, 64, 0.1, 0, True),
    (300, 4096, 192, 0.0, 0, True), (130, 256, 64, 0.1, 4, False)])
def test_lora_down_kernel(M, K, R, p, offset, strided):
    """lora.hip lora_down: h = drop(x) A^T (mask = the host hash, ops/_ref.py) and the x_d side output."""
    from gke_ray_train_amd.ops import _ref
    C = _C()
    torch.manual_seed(1)
    xs = torch.randn(M, K + (64 if strided else 0), device=DEV, dtype=torch.bfloat16)
    x = xs[:, :K]
    a = (torch.randn(R, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16)
    seed = 0x1234_5678_9abc
    res = C.lora_down(x, a, p, seed, offset, True)
    assert len(res) == 2, "kernel path not taken"
    h, xd = res
    keep = _ref.dropout_keep_mask(seed, offset, M * K, p).to(DEV).view(M, K).float() if p > 0 else 1.0
    xr = x.float() * keep / (1 - p)
    _close(xd, xr, 1e-2, 1e-2, "lora_down xd")
    _close(h, xr @ a.float().t(), 2e-2, 2e-2, "lora_down h")
    assert len(C.lora_down(x, a, p, seed, offset, False)) == 1
    assert C.lora_down(x[:, :K - 32], a[:, :K - 32].contiguous(), p, seed, offset, True) == []  # K % 64


@pytest.mark.parametrize("M,K,R,p,offset,acc", [
    (256, 256, 32, 0.0, 0, True), (200, 512, 48, 0.1, 0, True), (77, 1024, 192, 0.1, 8, False),
    (1024, 4096, 128, 0.1, 0, True), (65, 128, 256, 0.5, 4, True), (100, 384, 16, 0.1, 0, True)])
def test_lora_dx_kernel(M, K, R, p, offset, acc):
    """lora.hip lora_dx: dx (+)= keep/(1-p) * (g A), A^T given as [K, R]."""
    from gke_ray_train_amd.ops import _ref
    C = _C()
    torch.manual_seed(2)
    g = torch.randn(M, R, device=DEV, dtype=torch.bfloat16)
    a = (torch.randn(R, K, device=DEV) / math.sqrt(R)).to(torch.bfloat16)
    dx = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    dx0 = dx.float().clone()
    seed = 987654321
    assert C.lora_dx(g, a.t().contiguous(), dx, p, seed, offset, acc), "kernel path not taken"
    keep = _ref.dropout_keep_mask(seed, offset, M * K, p).to(DEV).view(M, K).float() if p > 0 else 1.0
    ref = (g.float() @ a.float()) * keep / (1 - p) + (dx0 if acc else 0)
    _close(dx, ref, 2e-2, 2e-2, "lora_dx")
    assert not C.lora_dx(g, a.t().contiguous()[:64].contiguous(), dx[:, :64].contiguous(), p, seed, offset, acc)


def test_transpose_and_nf4_dequant_t():
    """HIP transpose and transposing NF4 dequant match torch exactly."""
    from gke_ray_train_amd import ops
    C = _C()
    w = torch.randn(384, 640, device=DEV, dtype=torch.bfloat16)
    wt = torch.empty(640, 384, device=DEV, dtype=torch.bfloat16)
    C.transpose_into(w, wt)
    assert torch.equal(wt, w.t())
    q, absmax = ops.nf4_quantize(w.reshape(-1), 64)
    deq = ops.nf4_dequantize(q, absmax, w.numel(), 64, torch.bfloat16).view(384, 640)
    assert torch.equal(C.nf4_dequantize_t(q, absmax, 384, 640, 64), deq.t())


@pytest.mark.parametrize("rows,cols", [(384, 640), (4096, 1024), (200, 256), (64, 4224)])
def test_nf4_dequant_v2_exact(rows, cols):
    """v2 dequantisation (byte-indexed LDS table): flat, into a row-strided [W | tail] buffer, and
    transposed, all bit-equal to the fp32 math (level x absmax, one rounding to bf16)."""
    from gke_ray_train_amd import ops
    from gke_ray_train_amd.ops import _ref
    C = _C()
    g = torch.Generator(device=DEV).manual_seed(rows + cols)
    w = torch.randn(rows, cols, device=DEV, generator=g).bfloat16()
    q, absmax = ops.nf4_quantize(w.reshape(-1), 64)
    ref = _ref.nf4_dequantize(q.cpu(), absmax.cpu(), w.numel(), 64, torch.bfloat16).view(rows, cols)
    flat = ops.nf4_dequantize(q, absmax, w.numel(), 64, torch.bfloat16).view(rows, cols)
    assert torch.equal(flat.cpu(), ref)
    buf = torch.full((rows, cols + 192), float("nan"), device=DEV, dtype=torch.bfloat16)
    assert C.nf4_dequantize_into(q, absmax, buf[:, :cols], 64)
    assert torch.equal(buf[:, :cols].cpu(), ref) and bool(torch.isnan(buf[:, cols:]).all())
    assert torch.equal(C.nf4_dequantize_t(q, absmax, rows, cols, 64).cpu(), ref.t())


def test_swiglu_transposing_kernels_exact():
    """swiglu_fwd_t / swiglu_bwd_t: the row-major results are bit-equal to the plain kernels and the
    second outputs are exactly their transposes; unhandled shapes return nothing."""
    C = _C()
    g = torch.Generator(device=DEV).manual_seed(9)
    gu = torch.randn(256, 2 * 384, device=DEV, generator=g).bfloat16()
    dout = torch.randn(256, 384, device=DEV, generator=g).bfloat16()
    out = C.swiglu_fwd(gu, 0)
    o, ot = C.swiglu_fwd_t(gu, 0)
    assert torch.equal(o, out) and torch.equal(ot, out.t())
    o64, ot64 = C.swiglu_fwd_t(gu, 64)  # the [rows, f + 64] LoRA-tail row buffer
    assert o64.stride(0) == 384 + 64 and torch.equal(o64, out) and torch.equal(ot64, out.t())
    dgu = C.swiglu_bwd(gu, dout)
    d, dt = C.swiglu_bwd_t(gu, dout)
    assert torch.equal(d, dgu) and torch.equal(dt, dgu.t())
    assert not C.swiglu_fwd_t(gu[:100].contiguous(), 0) and not C.swiglu_bwd_t(gu[:100].contiguous(), dout[:100].contiguous())


@pytest.mark.parametrize("producer", ["swiglu", "attention"])
def test_swiglu_transposed_wgrad_path_matches(producer, monkeypatch):
    """Llama layers under the DDP engine: with the transposing producers the weight gradients take
    their transposed operand from the producing kernel (SwiGLU: h^T for down, dgu^T for gate_up;
    attention: o^T from the forward for o_proj, dqkv^T from the backward for qkv_proj), two fewer
    transposes per layer each, and every gradient is bit-identical to the separate-transpose path."""
    from gke_ray_train_amd.models import build_llama, get_config
    from gke_ray_train_amd.ops import fused as Fu
    from gke_ray_train_amd.ops import linear as L
    from gke_ray_train_amd.parallel import DistributedDataParallel
    cfg = get_config("llama-tiny-gqa", intermediate_size=1536)
    ids = torch.randint(0, 512, (2, 256), device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
    calls = {"n": 0}
    real = L.wgrad_tn

    def counting(*a):
        calls["n"] += 1
        return real(*a)
    monkeypatch.setattr(L, "wgrad_tn", counting)
    out, ncalls = [], []
    for flag in (False, True):
        monkeypatch.setattr(Fu, "_SWIGLU_T", flag and producer == "swiglu")
        monkeypatch.setattr(Fu, "_ATTN_DQKV_T", flag and producer == "attention")
        calls["n"] = 0
        m = build_llama(cfg, device=DEV, dtype=torch.bfloat16, seed=2)
        ddp = DistributedDataParallel(m)
        m(ids, labels=ids)["loss"].backward()
        ddp.finish_gradient_sync()
        torch.cuda.synchronize()
        out.append({n: p.grad.clone() for n, p in m.named_parameters()})
        ncalls.append(calls["n"])
    for n in out[0]:
        assert torch.equal(out[0][n], out[1][n]), n
    # with the flag: two weight gradients per layer ran on the provided copies
    assert ncalls == [0, 2 * cfg.num_hidden_layers], ncalls


def test_transposed_dgrad_linear_matches_nn():
    """Trainable DDP weight: forward writes W^T on a side stream, backward runs the TN GEMM;
    gradients equal the NN path (GRT_TRANSPOSED_DGRAD=0) to bf16 rounding."""
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.ops import linear as L
    from gke_ray_train_amd.parallel import DistributedDataParallel
    ids = torch.randint(0, 512, (2, 256), device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
    out = []
    L._TRANSPOSED_DGRAD_TRAINABLE = True
    for flag in (False, True):
        L._TRANSPOSED_DGRAD = flag
        m = build_llama("llama-tiny-gqa", device=DEV, dtype=torch.bfloat16, seed=2)
        ddp = DistributedDataParallel(m)
        m(ids, labels=ids)["loss"].backward()
        ddp.finish_gradient_sync()
        out.append({n: p.grad.float().clone() for n, p in m.named_parameters()})
        if flag:
            assert any(getattr(p, "_grt_wt_buf", None) is not None for p in m.parameters())
    L._TRANSPOSED_DGRAD = True
    L._TRANSPOSED_DGRAD_TRAINABLE = False
    for n in out[0]:
        rel = (out[0][n] - out[1][n]).norm() / out[0][n].norm().clamp_min(1e-12)
        assert rel < 1e-2, (n, float(rel))


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,K", [(4096, 4096), (6144, 4096), (1000, 11008), (37, 264)])
def test_gemv_decode(M, N, K):
    """Decode GEMV (gemv.hip) vs the fp32 product; routed automatically by ops.linear under no_grad."""
    from gke_ray_train_amd.ops.linear import linear
    g = torch.Generator(device=DEV).manual_seed(M * N + K)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16, generator=g) * 0.02
    y = _C().gemv(x, w)
    ref = x.float() @ w.float().t()
    _close(y, ref, 2e-2, 2e-2, "gemv")
    from gke_ray_train_amd.ops.linear import _gemv_rows_ok
    with torch.no_grad():
        y2 = linear(x.view(M, 1, K), w)
    assert y2.shape == (M, 1, N)
    if _gemv_rows_ok(M, K):  # routed to the GEMV (FMA for 1-2 rows, MFMA for 3-16)
        assert torch.equal(y2.view(M, N), y)
    else:  # the library GEMM
        _close(y2.view(M, N), ref, 2e-2, 2e-2, "linear (library) at M rows")


@pytest.mark.parametrize("M", [3, 5, 8, 16])
@pytest.mark.parametrize("N,K", [(4096, 4096), (1000, 11008), (37, 512), (20000, 256)])
def test_gemv_mfma_rows(M, N, K):
    """Skinny MFMA GEMM for 3-16 decode rows (gemv.hip gemv_mfma_kernel, both wave counts, ragged N)
    vs the fp32 product."""
    g = torch.Generator(device=DEV).manual_seed(M * N + K)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16, generator=g) * 0.02
    y = _C().gemv(x, w)
    _close(y, x.float() @ w.float().t(), 2e-2, 2e-2, "gemv_mfma")


@pytest.mark.parametrize("M", [1, 3])
@pytest.mark.parametrize("N,K", [(4096, 14336), (12288, 1024), (37, 264)])
def test_gemv_swiglu_decode(M, N, K):
    """Down-projection GEMV with the SwiGLU of the fused gate/up output folded in (both the
    K-split (N <= 8192) and the one-wave-per-row variants) == swiglu kernel + GEMV == fp32 math."""
    from gke_ray_train_amd import ops
    g = torch.Generator(device=DEV).manual_seed(M * N + K)
    gu = torch.randn(M, 2 * K, device=DEV, dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16, generator=g) * 0.02
    y = _C().gemv(gu, w, swiglu=True)
    with torch.no_grad():
        a = ops.swiglu(gu)
    _close(y, _C().gemv(a, w), 1e-2, 1e-2, "gemv_swiglu vs swiglu + gemv")
    gf = gu.float()
    ref = (torch.nn.functional.silu(gf[:, :K]) * gf[:, K:]) @ w.float().t()
    _close(y, ref, 2e-2, 2e-2, "gemv_swiglu vs fp32")


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("swiglu", [False, True])
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 14336), (37, 264)])
def test_gemv_resnorm_epilogue(M, N, K, swiglu):
    """Producer GEMV with the residual add and the next RMSNorm's statistics in its epilogue:
    h == bf16(gemv(x, w)) + res bitwise (torch rounding); the fixed-point sum of squares (slot) ==
    sum(h^2) and is bitwise reproducible; the other slot is zeroed for the next producer; a consumer
    reading the slot normalises like rsqrt(mean(h^2) + eps)."""
    C = _C()
    g = torch.Generator(device=DEV).manual_seed(M * N + K + swiglu)
    x = torch.randn(M, (2 if swiglu else 1) * K, device=DEV, dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16, generator=g) * 0.02
    res = torch.randn(M, N, device=DEV, dtype=torch.bfloat16, generator=g)
    sums = []
    for slot in (0, 1, 0):
        acc = torch.full((2, M, 64), 12345, dtype=torch.int64, device=DEV)
        acc[slot] = 0
        h = C.gemv_fused(x, w, acc, slot, swiglu=swiglu, res=res)
        assert torch.equal(h, (C.gemv(x, w, swiglu).float() + res.float()).to(torch.bfloat16))
        assert int(acc[1 - slot].abs().sum()) == 0
        ref = h.double().pow(2).sum(-1)
        torch.testing.assert_close(acc[slot].sum(-1).double() / 2 ** 20, ref, rtol=1e-5, atol=1e-5)
        sums.append(acc[slot].clone())
    assert torch.equal(sums[0], sums[1]) and torch.equal(sums[0], sums[2])
    if N % 8:
        return
    # a consumer of h (normalise on the fly) against the norm math with the exact rstd
    w2 = torch.randn(64, N, device=DEV, dtype=torch.bfloat16, generator=g) * 0.02
    nw = (1 + 0.1 * torch.randn(N, device=DEV, generator=g)).to(torch.bfloat16)
    y = C.gemv_fused(h, w2, torch.stack([torch.zeros_like(sums[0]), sums[0]]), 1, g=nw, eps=1e-5)
    rstd = torch.rsqrt(h.float().pow(2).mean(-1) + 1e-5)
    _close(y, (h.float() * rstd[:, None] * nw.float()) @ w2.float().t(), 2e-2, 2e-2, "normx after resnorm")


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("N,K", [(6144, 4096), (1000, 8192), (37, 264)])
def test_gemv_normx_prologue(M, N, K):
    """Consumer GEMV normalising its input on the fly from the fixed-point sum of squares: ==
    rms_norm-rounded input + GEMV, and == fp32 math."""
    C = _C()
    g = torch.Generator(device=DEV).manual_seed(M * N + K)
    h = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=g)
    nw = (1 + 0.1 * torch.randn(K, device=DEV, generator=g)).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16, generator=g) * 0.02
    acc = torch.zeros(2, M, 64, dtype=torch.int64, device=DEV)
    acc[0, :, 5] = torch.round(h.double().pow(2).sum(-1) * 2 ** 20).long()
    y = C.gemv_fused(h, w, acc, 0, g=nw, eps=1e-5)
    rstd = torch.rsqrt(h.float().pow(2).mean(-1) + 1e-5)
    xn = (h.float() * rstd[:, None] * nw.float()).to(torch.bfloat16)
    _close(y, C.gemv(xn, w), 1e-2, 1e-2, "gemv normx vs normalised input + gemv")
    ref = (h.float() * rstd[:, None] * nw.float()) @ w.float().t()
    _close(y, ref, 2e-2, 2e-2, "gemv normx vs fp32")


@pytest.mark.parametrize("M,hq,hkv,normx", [(1, 32, 8, True), (2, 8, 8, False), (2, 4, 1, True)])
def test_gemv_rope_epilogue(M, hq, hkv, normx):
    """qkv GEMV with the RoPE + KV-cache append epilogue == GEMV + rope_append (q bitwise, cache
    slots bitwise, untouched slots unchanged); an out-of-range position writes nothing."""
    C, D, L = _C(), 128, 16
    g = torch.Generator(device=DEV).manual_seed(M * hq + hkv)
    K = 512
    N = (hq + 2 * hkv) * D
    h = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16, generator=g) * 0.05
    nw = (1 + 0.1 * torch.randn(K, device=DEV, generator=g)).to(torch.bfloat16)
    acc = torch.zeros(2, M, 64, dtype=torch.int64, device=DEV)
    acc[1, :, 0] = torch.round(h.double().pow(2).sum(-1) * 2 ** 20).long()
    ang = torch.arange(L, device=DEV, dtype=torch.float32)[:, None] * torch.rand(64, device=DEV, generator=g)
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    pos = torch.tensor([3, 11][:M], device=DEV, dtype=torch.int32)
    if M == 2 and hq == 8:
        pos[1] = L + 5  # past the cache / rope table: no write for that row
    kc0 = torch.randn(M, L, hkv, D, device=DEV, dtype=torch.bfloat16, generator=g)
    vc0 = torch.randn(M, L, hkv, D, device=DEV, dtype=torch.bfloat16, generator=g)
    kc, vc, kr, vr = kc0.clone(), vc0.clone(), kc0.clone(), vc0.clone()
    if normx:
        q = C.gemv_fused(h, w, acc, 1, g=nw, eps=1e-5, cos=cos, sin=sin, pos=pos, kc=kc, vc=vc, hq=hq, hkv=hkv)
        qkv = C.gemv_fused(h, w, acc, 1, g=nw, eps=1e-5)
    else:
        q = C.gemv_fused(h, w, acc, 1, cos=cos, sin=sin, pos=pos, kc=kc, vc=vc, hq=hq, hkv=hkv)
        qkv = C.gemv(h, w)
    qr = C.rope_append(qkv, cos, sin, pos, hq, hkv, D, L, kr, vr, 1)
    ok = (pos < L).tolist()
    for m in range(M):  # same bf16 qkv; the rotation's fp32 contraction may differ by an ulp
        if ok[m]:
            _close(q[m], qr[m].view(hq, D), 1e-2, 1e-2, "rope epilogue q")
    _close(kc, kr, 1e-2, 1e-2, "rope epilogue k cache")
    assert torch.equal(vc, vr)
    assert not torch.equal(kc, kc0) and not torch.equal(vc, vc0)
    for m in range(M):  # only the slot at pos[m] changed
        keep = torch.ones(L, dtype=torch.bool)
        if ok[m]:
            keep[int(pos[m])] = False
        assert torch.equal(kc[m, keep], kc0[m, keep]) and torch.equal(vc[m, keep], vc0[m, keep])


@pytest.mark.parametrize("B", [1, 2])
def test_decode_fused_norm_matches_unfused(B):
    """GraphDecoder with the residual adds / norms / RoPE inside the GEMVs == the unfused decode
    (GRT_GEMV_NORM=0 path): same greedy tokens, logits within bf16 rounding (1 and 2 rows)."""
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.models import generation as G
    torch.manual_seed(0)
    m = build_llama("llama-tiny-gqa", device=DEV, dtype=torch.bfloat16, seed=0).eval()
    ids = torch.randint(0, m.config.vocab_size, (B, 12), device=DEV)
    outs = []
    for fused in (True, False):
        G._GEMV_NORM = fused
        try:
            dec = G.GraphDecoder(m, B, 32)
            assert (dec.norm_ws is not None) == fused
            lg = [dec.prefill(ids)]
            nxt = lg[-1].argmax(-1)
            for _ in range(6):
                lg.append(dec.step(nxt).clone())
                nxt = lg[-1].argmax(-1)
            outs.append(torch.stack(lg))
        finally:
            G._GEMV_NORM = True
    assert torch.equal(outs[0].argmax(-1), outs[1].argmax(-1))
    _close(outs[0], outs[1], 2e-2, 2e-2, "fused vs unfused decode logits")


@pytest.mark.parametrize("B,S,hq,hkv,L,start", [(1, 1, 32, 8, 64, 17), (2, 5, 8, 8, 40, 3), (3, 4, 4, 1, 10, 8)])
def test_rope_append(B, S, hq, hkv, L, start):
    """Decode RoPE + KV-cache append (rope_append, elementwise.hip) == rope_fwd + cache slice writes;
    positions past the cache are skipped, every other slot is untouched."""
    from gke_ray_train_amd.ops import _ref
    C, D = _C(), 128
    g = torch.Generator(device=DEV).manual_seed(B * S + hq)
    qkv = torch.randn(B * S, (hq + 2 * hkv) * D, device=DEV, dtype=torch.bfloat16, generator=g)
    # rope table longer than the cache: positions past the cache are valid rope positions (q is
    # still rotated) whose k / v writes the kernel must skip
    St = start + S + 4
    cos, sin = _ref.rope_tables(St, D, 10000.0, device=DEV)
    pos = torch.arange(start, start + S, device=DEV, dtype=torch.int32).repeat(B)
    kc = torch.randn(B, L, hkv, D, device=DEV, dtype=torch.bfloat16, generator=g)
    vc = torch.randn(B, L, hkv, D, device=DEV, dtype=torch.bfloat16, generator=g)
    kc0, vc0 = kc.clone(), vc.clone()
    q = C.rope_append(qkv, cos, sin, pos, hq, hkv, D, St, kc, vc, S)
    x3 = qkv.view(B * S, hq + 2 * hkv, D)
    qr = _ref.apply_rope(x3[:, :hq], cos, sin, pos)
    kr = _ref.apply_rope(x3[:, hq:hq + hkv], cos, sin, pos)
    n = max(0, min(S, L - start))  # slots written
    qv = q.view(B, S, hq, D)[:, :n]  # q rows of skipped positions are not written
    _close(qv, qr.view(B, S, hq, D)[:, :n], 1e-2, 1e-2, "rope_append q")
    ke, ve = kc0.clone(), vc0.clone()
    ke[:, start:start + n] = kr.view(B, S, hkv, D)[:, :n]
    ve[:, start:start + n] = x3[:, hq + hkv:].reshape(B, S, hkv, D)[:, :n]
    _close(kc, ke, 1e-2, 1e-2, "rope_append k cache")
    assert torch.equal(vc, ve), "rope_append v cache"


@pytest.mark.parametrize("B,Sk,hq,hkv,pad", [(1, 1, 4, 4, False), (1, 600, 32, 8, False), (3, 77, 8, 1, True),
                                             (2, 1300, 16, 8, True), (2, 33, 8, 4, False)])
def test_decode_attention(B, Sk, hq, hkv, pad):
    """Split-K decode kernel (decode_attention.hip) vs the fp32 math path: one query per sequence
    at the last position (causal) or under a valid-length mask (seqlens_k)."""
    from gke_ray_train_amd import ops
    from gke_ray_train_amd.ops import _ref
    g = torch.Generator(device=DEV).manual_seed(B * Sk + hq)
    q = torch.randn(B, 1, hq, 128, device=DEV, dtype=torch.bfloat16, generator=g)
    k = torch.randn(B, Sk, hkv, 128, device=DEV, dtype=torch.bfloat16, generator=g)
    v = torch.randn(B, Sk, hkv, 128, device=DEV, dtype=torch.bfloat16, generator=g)
    sl = torch.randint(1, Sk + 1, (B,), device=DEV, generator=g).to(torch.int32) if pad else None
    with torch.no_grad():
        o = ops.flash_attention(q, k, v, causal=not pad, seqlens_k=sl)
    ref = _ref.attention(q.float(), k.float(), v.float(), causal=not pad, seqlens_k=sl)
    _close(o, ref, 1e-2, 1e-2, "decode attention")


@pytest.mark.parametrize("nf4", [False, True, "stream"])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("engine", ["none", "ddp"])
def test_kcat_lora_matches_reference(nf4, p, engine):
    """K-concatenated LoRA (peft/lora.py _LoraKcatFn): the input is the head of a [M, in + R] row
    buffer, h' lands in its tail, y = [x | h'] W'^T and [dX | g] = dY W' are single GEMMs. Same
    y / dX / dA / dB as the fp32 formula (masks regenerated from the seed the op drew).
    nf4="stream": NF4 base without the dequant cache, W' rebuilt per forward (_kcat_weight_streamed)."""
    stream = nf4 == "stream"
    nf4 = bool(nf4)
    from gke_ray_train_amd.ops import _ref
    from gke_ray_train_amd.ops.linear import Linear
    from gke_ray_train_amd.peft.lora import LoraConfig, LoraLinear
    from gke_ray_train_amd.peft.quant import BitsAndBytesConfig, NF4Linear
    torch.manual_seed(0)
    lin = Linear(256, 768, bias=False, device=DEV, dtype=torch.bfloat16)
    lin.slices = [("q_proj", 256), ("k_proj", 256), ("v_proj", 256)]
    base = NF4Linear.from_linear(lin, BitsAndBytesConfig()) if nf4 else lin
    if nf4:
        base.set_dequant_cache(not stream)
    for q in base.parameters():
        q.requires_grad_(False)
    cfg = LoraConfig(r=64, lora_alpha=32, lora_dropout=p)
    tg = [("q_proj", 0), ("k_proj", 256), ("v_proj", 512)]
    mod = LoraLinear(base, [(n, off, 256) for n, off in tg], cfg).train()
    names = [n for n, _ in tg]
    R = 64 * 3
    assert mod.kcat_pad == R
    with torch.no_grad():
        for n in names:
            mod.lora_B[n].normal_(0, 0.05)
    M = 384
    xw = torch.randn(M, 256 + R, device=DEV, dtype=torch.bfloat16)
    xw[:, 256:] = float("nan")  # the op must write every tail element before the GEMM reads it
    x = xw[:, :256].detach().requires_grad_()
    x._grt_tail = R
    fwd = mod
    if engine == "ddp":
        from gke_ray_train_amd.parallel import DistributedDataParallel
        fwd = DistributedDataParallel(mod)
        x._grt_tail = R
    rng = torch.get_rng_state()
    y = fwd(x)
    dy = torch.randn_like(y)
    (y.float() * dy.float()).sum().backward()
    if engine == "ddp":
        fwd.finish_gradient_sync()
    torch.set_rng_state(rng)
    seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
    x2 = x.detach().float().requires_grad_()
    w = (base.dequantize() if nf4 else lin.weight).detach().float()
    A = {n: mod.lora_A[n].detach().float().requires_grad_() for n in names}
    B = {n: mod.lora_B[n].detach().float().requires_grad_() for n in names}
    if p > 0:
        keep = _ref.dropout_keep_mask(seed, 0, x2.numel(), p).to(DEV).view_as(x2).float()
        xd = x2 * keep / (1 - p)
    else:
        xd = x2
    yr = (x2 @ w.t()).clone()
    for n, off in tg:
        yr[:, off:off + 256] = yr[:, off:off + 256] + cfg.scaling * (xd @ A[n].t()) @ B[n].t()
    (yr * dy.float()).sum().backward()
    _close(y, yr, 3e-2, 3e-2, "kcat y")
    _close(x.grad, x2.grad, 3e-2, 3e-2, "kcat dx")
    if stream:
        assert mod._wk is None and getattr(base, "_w_cache", None) is None  # nothing bf16 stays resident
    for n in names:
        for got, ref, what in ((mod.lora_A[n].grad, A[n].grad, "dA"), (mod.lora_B[n].grad, B[n].grad, "dB")):
            rel = (got.float() - ref).norm() / ref.norm().clamp_min(1e-6)
            assert rel < 2e-2, f"kcat {what} {n}: rel err {rel.item():.3g}"


def test_kcat_lora_model_matches_epilogue_form(monkeypatch):
    """A LoRA Llama whose q/k/v/o/gate/up run K-concatenated (down stays on the epilogue form: its
    input width is not a multiple of 128 here) trains like the epilogue form: same loss, same
    adapter gradients within bf16 tolerance."""
    import gke_ray_train_amd.peft.lora as L
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.peft import LoraConfig, get_peft_model
    res = {}
    for kcat in (True, False):
        monkeypatch.setattr(L, "_LORA_KCAT", kcat)
        torch.manual_seed(0)
        m = build_llama("llama-tiny-gqa", device=DEV, dtype=torch.bfloat16, seed=2)
        pm = get_peft_model(m, LoraConfig(r=64, lora_alpha=16, lora_dropout=0.0))
        for lm in pm.lora_modules.values():
            for b in lm.lora_B.values():
                torch.nn.init.normal_(b, 0, 0.02, generator=torch.Generator(device=DEV).manual_seed(9))
        ids = torch.randint(0, m.config.vocab_size, (2, 256), device=DEV, generator=torch.Generator(device=DEV).manual_seed(4))
        loss = pm(ids, labels=ids)["loss"]
        loss.backward()
        res[kcat] = (float(loss.detach()), {n: p.grad.float().clone() for n, p in pm.named_parameters() if p.grad is not None})
        if kcat:
            assert any(lm.kcat_pad for lm in pm.lora_modules.values())
    (l1, g1), (l0, g0) = res[True], res[False]
    assert abs(l1 - l0) < 2e-2 * max(1.0, abs(l0))
    assert g1.keys() == g0.keys() and g1
    for n in g0:
        rel = (g1[n] - g0[n]).norm() / g0[n].norm().clamp_min(1e-8)
        assert rel < 5e-2, f"{n}: rel {rel.item():.3g}"


def test_kcat_lora_no_grad_forwards_reuse_tail_until_b_changes():
    """Evaluation forwards (no autograd) of a K-concatenated LoRA projection skip the W' tail refresh
    while B is unchanged, and pick up every change: an in-place torch edit (version counter), a
    framework optimizer step (raw-pointer writes: ops.optim.param_generation) and a training
    forward in between. Each result equals the grad-enabled forward of the same weights."""
    from gke_ray_train_amd.ops.linear import Linear
    from gke_ray_train_amd.ops.optim import FusedAdamW
    from gke_ray_train_amd.peft.lora import LoraConfig, LoraLinear
    torch.manual_seed(0)
    lin = Linear(256, 512, bias=False, device=DEV, dtype=torch.bfloat16)
    lin.slices = [("gate_proj", 256), ("up_proj", 256)]
    lin.weight.requires_grad_(False)
    mod = LoraLinear(lin, [("gate_proj", 0, 256), ("up_proj", 256, 256)], LoraConfig(r=64, lora_alpha=16,
                                                                                    lora_dropout=0.0))
    R = 128
    assert mod.kcat_pad == R
    xw = torch.randn(256, 256 + R, device=DEV, dtype=torch.bfloat16)

    def fwd(grad):
        x = xw[:, :256]
        x._grt_tail = R
        with torch.set_grad_enabled(grad):
            return mod(x).detach().float()

    def ref():
        y = xw[:, :256].float() @ lin.weight.float().t()
        for n, off in (("gate_proj", 0), ("up_proj", 256)):
            y[:, off:off + 256] += mod.scaling * (xw[:, :256].float() @ mod.lora_A[n].float().t()) @ mod.lora_B[n].float().t()
        return y

    with torch.no_grad():
        for b in mod.lora_B.values():
            b.normal_(0, 0.05)
    y0 = fwd(False)
    _close(y0, ref(), 3e-2, 3e-2, "first no-grad forward")
    key = mod._wk_key
    assert key is not None
    assert torch.equal(fwd(False), y0) and mod._wk_key == key  # reused
    with torch.no_grad():
        mod.lora_B["up_proj"].mul_(-2.0)  # version counter
    _close(fwd(False), ref(), 3e-2, 3e-2, "after an in-place edit")
    # an optimizer step through the fused kernel (no version bump)
    opt = FusedAdamW([p for p in mod.parameters() if p.requires_grad], lr=1e-2)
    xt = xw[:, :256].detach().requires_grad_()
    xt._grt_tail = R
    y = mod(xt)
    y.float().square().mean().backward()
    assert mod._wk_key is None  # a training forward refreshed and dropped the key
    v = mod.lora_B["gate_proj"]._version
    opt.step()
    assert mod.lora_B["gate_proj"]._version == v
    _close(fwd(False), ref(), 3e-2, 3e-2, "after a fused optimizer step")
    _close(fwd(True), ref(), 3e-2, 3e-2, "grad-enabled forward")


@pytest.mark.parametrize("B,S,hq,hkv,causal,pad,p,rope", [
    (2, 256, 4, 4, True, None, 0.0, False),
    (1, 200, 4, 2, True, None, 0.0, True),        # partial tail block, GQA, RoPE epilogue
    (2, 160, 2, 2, False, [160, 77], 0.0, False),  # key padding
    (2, 256, 4, 2, True, None, 0.1, False),        # probability dropout
    (8, 1024, 32, 32, True, None, 0.0, False),     # Llama-2-7B bench shape (causal pairs)
    (2, 2048, 32, 8, True, None, 0.0, True),       # Llama-3 GQA 32:8
])
def test_dkdv_wave_pair_matches_four_wave_kernel(B, S, hq, hkv, causal, pad, p, rope):
    """The wave-pair dK / dV kernel (attention.hip attn_bwd_dkdv2_kernel, S-wave + dP-wave per 32
    keys) does the 4-wave kernel's arithmetic in the same order: dQ / dK / dV bitwise equal."""
    from gke_ray_train_amd import _native
    from gke_ray_train_amd.ops import _ref
    C = _native.kernels()
    D = 128
    g = torch.Generator(device=DEV).manual_seed(B * S + hq)
    q, do = (torch.randn(B, S, hq, D, device=DEV, dtype=torch.bfloat16, generator=g) for _ in range(2))
    k, v = (torch.randn(B, S, hkv, D, device=DEV, dtype=torch.bfloat16, generator=g) for _ in range(2))
    sl = None if pad is None else torch.tensor(pad, device=DEV, dtype=torch.int32)
    cos = sin = None
    if rope:
        cos, sin = _ref.rope_tables(S, D, 10000.0, device=DEV)
        cos, sin = cos.float().contiguous(), sin.float().contiguous()
    o, lse = C.attn_fwd(q, k, v, None, D ** -0.5, causal, sl, p, 11)
    out = {}
    try:
        for form in (1, 2):
            C.attn_set_dkdv_form(form)
            out[form] = C.attn_bwd(do, q, k, v, o, lse, None, None, None, D ** -0.5, causal, sl, p, 11, cos, sin)
        torch.cuda.synchronize()
    finally:
        C.attn_set_dkdv_form(2)
    for name, a, b in zip(("dq", "dk", "dv"), out[1], out[2]):
        assert torch.equal(a, b), f"{name}: max diff {(a.float() - b.float()).abs().max().item():.3g}"


@pytest.mark.parametrize("B,S,hq,hkv,rope,form,varlen", [
    (2, 256, 4, 4, True, 2, False),       # wave-pair dK / dV kernel, RoPE epilogue
    (2, 256, 4, 2, False, 2, False),      # GQA, plain epilogue
    (1, 192, 4, 2, True, 1, False),       # 4-wave dK / dV kernel, partial tail block
    (1, 384, 4, 4, True, 2, True),        # padding-free packed sequences (cu_seqlens)
    (8, 1024, 32, 32, True, 2, False),    # Llama-2-7B step shape
])
def test_attn_bwd_writes_transposed_dqkv(B, S, hq, hkv, rope, form, varlen):
    """The epilogues' transposed copies — the forward's o^T (attn_fwd o_t, the o projection's TN
    weight-gradient operand) and the backward's dqkv^T (attn_bwd dqkv_t, the QKV projection's) —
    equal o^T / dqkv^T bit for bit, and the row-major outputs are unchanged by them."""
    from gke_ray_train_amd import _native
    from gke_ray_train_amd.ops import _ref
    C = _native.kernels()
    D = 128
    g = torch.Generator(device=DEV).manual_seed(B * S + hq + form)
    W = (hq + 2 * hkv) * D
    qkv = torch.randn(B * S, W, device=DEV, dtype=torch.bfloat16, generator=g)
    do = torch.randn(B, S, hq, D, device=DEV, dtype=torch.bfloat16, generator=g)
    cu, ml, pos = None, 0, None
    if varlen:
        cu = torch.tensor([0, 100, 228, 384], device=DEV, dtype=torch.int32)
        ml = 156
        pos = torch.cat([torch.arange(b - a, device=DEV) for a, b in ((0, 100), (100, 228), (228, 384))]).int()
    cos, sin = _ref.rope_tables(S, D, 10000.0, device=DEV)
    cos, sin = cos.float().contiguous(), sin.float().contiguous()
    q, k = C.rope_fwd(qkv, cos, sin, pos, hq, hkv, D, ml if varlen else S)
    q4, k4 = q.view(B, S, hq, D), k.view(B, S, hkv, D)
    v4 = qkv.view(B, S, hq + 2 * hkv, D)[:, :, hq + hkv:, :]
    o = torch.empty(B, S, hq, D, device=DEV, dtype=torch.bfloat16)
    o_t = torch.full((hq * D, B * S), float("nan"), device=DEV, dtype=torch.bfloat16)
    _, lse = C.attn_fwd(q4, k4, v4, o, D ** -0.5, True, None, cu_seqlens=cu, max_seqlen=ml, o_t=o_t)
    o2 = torch.empty_like(o)
    C.attn_fwd(q4, k4, v4, o2, D ** -0.5, True, None, cu_seqlens=cu, max_seqlen=ml)
    torch.cuda.synchronize()
    assert torch.equal(o, o2)  # the transposed copy changes nothing in o
    assert torch.equal(o_t, o.view(B * S, hq * D).t().contiguous())  # forward epilogue's o^T
    outs = []
    try:
        C.attn_set_dkdv_form(form)
        for with_t in (False, True):
            dqkv = torch.full_like(qkv, float("nan"))
            d4 = dqkv.view(B, S, hq + 2 * hkv, D)
            dqkv_t = torch.full((W, B * S), float("nan"), device=DEV, dtype=torch.bfloat16) if with_t else None
            C.attn_bwd(do, q4, k4, v4, o, lse, d4[:, :, :hq], d4[:, :, hq:hq + hkv], d4[:, :, hq + hkv:], D ** -0.5,
                       True, None, rope_cos=cos if rope else None, rope_sin=sin if rope else None, cu_seqlens=cu,
                       max_seqlen=ml, dqkv_t=dqkv_t)
            outs.append((dqkv, dqkv_t))
        torch.cuda.synchronize()
    finally:
        C.attn_set_dkdv_form(2)
    assert torch.equal(outs[0][0], outs[1][0])
    assert not torch.isnan(outs[1][0].float()).any()
    assert torch.equal(outs[1][1], outs[1][0].t().contiguous())


@pytest.mark.parametrize("dt,n", [(torch.bfloat16, 40_000_013), (torch.bfloat16, 3 * 1024 * 256 * 8 + 5),
                                  (torch.float32, 9_000_011)])
def test_sumsq_unrolled_matches_float64(dt, n):
    """Grad-norm partial sums over sizes that run the 4-load unrolled loop on every lane, on some
    lanes only (3 grid strides + a tail) and through the scalar remainder."""
    from gke_ray_train_amd import _native
    K = _native.kernels()
    torch.manual_seed(11)
    x = torch.randn(n, device=DEV, dtype=dt)
    ws = torch.zeros(2 * K.sumsq_blocks(), device=DEV, dtype=torch.float32)
    K.sumsq(x, ws, 1)
    got = ws[K.sumsq_blocks():].double().sum().item()
    ref = x.double().square().sum().item()
    assert abs(got - ref) < 1e-5 * ref, (got, ref)
    assert float(ws[:K.sumsq_blocks()].abs().sum()) == 0.0
