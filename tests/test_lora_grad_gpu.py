"""The LoRA adapter-gradient kernels (csrc/kernels/lora_grad.hip) against a plain fp32 PyTorch
reference: lora_g (C = alpha A B from B^T) and lora_tred (C = alpha A^T H, plain and transposed
output), on row-strided views like the ones the LoRA backward passes (column blocks of dY, of the
g / h' buffers and of the B^T buffer), assigning and accumulating; then a LoRA Llama's adapter
gradients with the kernels on vs the library GEMMs."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _C():
    from gke_ray_train_amd import _native
    return _native.kernels()


def _check(got, ref, what, tol=1e-2):
    got, ref = got.float(), ref.float()
    assert torch.isfinite(got).all(), f"{what}: non-finite output"
    err = (got - ref).abs()
    scale = ref.abs().max().clamp_min(1e-6)
    # every element: bf16 output rounding (2^-8 relative) of values up to the tensor's max
    assert (err / scale).max().item() < tol, f"{what}: max err {err.max().item():.4g} vs scale {scale.item():.4g}"


@pytest.mark.parametrize("M,K", [(256, 1024), (200, 4096), (8192, 1024), (96, 11008)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_lora_g(M, K, accumulate):
    torch.manual_seed(0)
    C = _C()
    wide = torch.randn(M, K + 256, device=DEV, dtype=torch.bfloat16)
    a = wide[:, 128:128 + K]                                   # column block of dY (row stride K + 256)
    btbuf = torch.randn(192, K + 512, device=DEV, dtype=torch.bfloat16) * 0.05
    bt = btbuf[64:128, 256:256 + K]                           # block of the B^T buffer
    gbuf = torch.randn(M, 192, device=DEV, dtype=torch.bfloat16)
    c = gbuf[:, 64:128]
    before = gbuf.clone()
    alpha = 0.25
    ref = alpha * (a.float() @ bt.float().t()) + (before[:, 64:128].float() if accumulate else 0)
    assert C.lora_g(a, bt, c, alpha, accumulate)
    _check(c, ref, f"lora_g M{M} K{K} acc{accumulate}")
    assert torch.equal(gbuf[:, :64], before[:, :64]) and torch.equal(gbuf[:, 128:], before[:, 128:])


@pytest.mark.parametrize("M", [200, 6016, 8192])
@pytest.mark.parametrize("accumulate", [False, True])
def test_lora_g_group(M, accumulate):
    """One launch for the targets of a fused module (q / k / v column blocks of one dY, their B^T
    rows, their g column blocks); equals the per-target products, incl. the k-split path (small M)."""
    torch.manual_seed(3)
    C = _C()
    ns = [(0, 1024), (1024, 256), (1280, 256)]  # (offset, width) of q / k / v in the fused dY
    dy = torch.randn(M, 1536, device=DEV, dtype=torch.bfloat16)
    btbuf = torch.randn(192, 1536, device=DEV, dtype=torch.bfloat16) * 0.05
    g = torch.randn(M, 192, device=DEV, dtype=torch.bfloat16)
    before = g.clone()
    a = [dy[:, o:o + n] for o, n in ns]
    bt = [btbuf[64 * j:64 * (j + 1), o:o + n] for j, (o, n) in enumerate(ns)]
    c = [g[:, 64 * j:64 * (j + 1)] for j in range(3)]
    assert C.lora_g_group(a, bt, c, 0.5, accumulate)
    for j in range(3):
        ref = 0.5 * (a[j].float() @ bt[j].float().t()) + (before[:, 64 * j:64 * (j + 1)].float() if accumulate else 0)
        _check(c[j], ref, f"lora_g_group M{M} product {j}")
    assert not C.lora_g_group(a + a[:2], bt + bt[:2], c + c[:2], 0.5, False)  # more than 4 products


@pytest.mark.parametrize("M", [384, 6016])
def test_lora_tred_group(M):
    """dB_i = dY_i^T h'_i of a fused module's targets in one launch: column blocks of one dY against
    their own h' column blocks, each product assigning or accumulating into its own output."""
    torch.manual_seed(4)
    C = _C()
    ns = [(0, 1024), (1024, 256), (1280, 256)]
    dy = torch.randn(M, 1536, device=DEV, dtype=torch.bfloat16)
    hc = torch.randn(M, 192, device=DEV, dtype=torch.bfloat16)
    outs = [torch.randn(n, 64, device=DEV, dtype=torch.bfloat16) for _, n in ns]
    before = [o.clone() for o in outs]
    acc = [False, True, False]
    a = [dy[:, o:o + n] for o, n in ns]
    h = [hc[:, 64 * j:64 * (j + 1)] for j in range(3)]
    assert C.lora_tred_group(a, h, outs, 1.0, acc)
    for j in range(3):
        ref = a[j].float().t() @ h[j].float() + (before[j].float() if acc[j] else 0)
        _check(outs[j], ref, f"lora_tred_group M{M} product {j}")
    assert not C.lora_tred_group(a, [hc[:, :128]] + h[1:], outs, 1.0, acc)  # R differs


@pytest.mark.parametrize("M,N,R", [(384, 256, 64), (8192, 4096, 64), (2048, 1024, 128), (1024, 11008, 64),
                                   (4096, 4096, 192)])
@pytest.mark.parametrize("transpose", [False, True])
@pytest.mark.parametrize("accumulate", [False, True])
def test_lora_tred(M, N, R, transpose, accumulate):
    torch.manual_seed(1)
    C = _C()
    wide = torch.randn(M, N + 128, device=DEV, dtype=torch.bfloat16)
    a = wide[:, 128:]
    hbuf = torch.randn(M, R + 64, device=DEV, dtype=torch.bfloat16)
    h = hbuf[:, :R]
    out = torch.randn((R, N) if transpose else (N, R), device=DEV, dtype=torch.bfloat16)
    old = out.clone()
    ref = a.float().t() @ h.float()
    if transpose:
        ref = ref.t()
    ref = ref + (old.float() if accumulate else 0)
    assert C.lora_tred(a, h, out, 1.0, accumulate, transpose)
    _check(out, ref, f"lora_tred M{M} N{N} R{R} T{transpose} acc{accumulate}")


def test_lora_tred_refuses_unsupported():
    C = _C()
    a = torch.randn(100, 256, device=DEV, dtype=torch.bfloat16)  # M % 32 != 0
    h = torch.randn(100, 64, device=DEV, dtype=torch.bfloat16)
    assert not C.lora_tred(a, h, torch.empty(256, 64, device=DEV, dtype=torch.bfloat16), 1.0, False, False)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_lora_model_grads_kernels_vs_library(monkeypatch, p):
    """Adapter gradients of a LoRA Llama (K-concatenated forward, direct-to-slot gradients through
    DDP) with the one-pass gradient kernels vs hipBLASLt's GEMMs: same loss, gradients within bf16."""
    import gke_ray_train_amd.peft.lora as L
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.parallel import DistributedDataParallel
    from gke_ray_train_amd.peft import LoraConfig, get_peft_model
    res = {}
    for on in (True, False):
        monkeypatch.setattr(L, "_LORA_GRAD_KERNELS", on)
        torch.manual_seed(0)
        m = build_llama("llama-tiny-gqa", device=DEV, dtype=torch.bfloat16, seed=2)
        pm = get_peft_model(m, LoraConfig(r=64, lora_alpha=16, lora_dropout=p))
        for lm in pm.lora_modules.values():
            for b in lm.lora_B.values():
                torch.nn.init.normal_(b, 0, 0.02, generator=torch.Generator(device=DEV).manual_seed(9))
        ddp = DistributedDataParallel(pm)
        ids = torch.randint(0, m.config.vocab_size, (2, 256), device=DEV, generator=torch.Generator(device=DEV).manual_seed(4))
        torch.manual_seed(5)  # same dropout seeds both runs
        loss = pm(ids, labels=ids)["loss"]
        loss.backward()
        ddp.finish_gradient_sync()
        grads = {i: b.float().clone() for i, b in enumerate(ddp.grad_buffers())}
        res[on] = (float(loss.detach()), grads)
        if on:
            assert any(getattr(lm, "_bt", None) is not None for lm in pm.lora_modules.values())
    (l1, g1), (l0, g0) = res[True], res[False]
    assert abs(l1 - l0) < 1e-3 * max(1.0, abs(l0))
    assert g1.keys() == g0.keys() and g1
    for n in g0:
        rel = (g1[n] - g0[n]).norm() / g0[n].norm().clamp_min(1e-8)
        assert rel < 2e-2, f"{n}: rel {rel.item():.3g}"
