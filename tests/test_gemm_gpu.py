"""Hand-written gfx950 GEMM family (csrc/kernels/gemm_mfma.hip) against an fp32 reference of the same
product, every output element checked: the forward / input-gradient form C = A B^T (pipeline
variants), the token-major weight-gradient form C = X^T Y and the NN form C = A B, overwrite and
accumulate (beta = 1), at tile-edge shapes (one 256 x 256 tile, the shortest reductions each
pipeline accepts, non-power-of-two tile counts, padded row strides)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from gke_ray_train_amd import _native
    return _native.kernels()


def _check(out, ref, what):
    err = (out.float() - ref).abs()
    # bf16 output rounding (2^-8 relative) plus fp32-accumulation-order noise
    bound = ref.abs() * 2.0 ** -7 + 2e-2
    bad = int((err > bound).sum())
    assert bad == 0, f"{what}: {bad} elements out of bound, max err {float(err.max()):.4g}"


def _rand(*shape, ld=None):
    if ld is None:
        return torch.randn(*shape, device="cuda").to(torch.bfloat16)
    buf = torch.randn(shape[0], ld, device="cuda").to(torch.bfloat16)
    return buf[:, :shape[1]]


@pytest.mark.parametrize("variant", [0, 1, 3, 4, 5])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 192), (768, 256, 4096), (256, 1280, 320)])
def test_gemm_nt_matches_fp32(variant, M, N, K):
    C = _C()
    if variant == 3 and K % 64:
        pytest.skip("half-tile variant needs K % 64 == 0")
    torch.manual_seed(M + N + K)
    a, b = _rand(M, K), _rand(N, K)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    assert C.gemm_nt(a, b, out, False, variant)
    ref = a.float() @ b.float().t()
    _check(out, ref, f"v{variant} {M}x{N}x{K}")
    acc = out.clone()
    assert C.gemm_nt(a, b, acc, True, variant)
    _check(acc, out.float() + ref, f"v{variant} accumulate")


def test_gemm_nt_strided_operands_and_unsupported_shapes():
    C = _C()
    a, b = _rand(512, 256, ld=264), _rand(256, 256, ld=320)
    out = torch.empty(512, 384, device="cuda", dtype=torch.bfloat16)[:, :256]
    assert C.gemm_nt(a, b, out, False, 0)
    _check(out, a.float() @ b.float().t(), "strided")
    bad = torch.empty(300, 256, device="cuda", dtype=torch.bfloat16)
    assert not C.gemm_supported(_rand(300, 256), b, bad)  # M not a tile multiple: caller falls back
    assert not C.gemm_nt(_rand(300, 256), b, bad, False, 0)


@pytest.mark.parametrize("variant", [9, 10, 11, 12])
@pytest.mark.parametrize("M,N,K,lda", [(256, 256, 128, None), (512, 768, 256, None), (768, 256, 4096, None),
                                       (256, 1280, 384, 392), (4096, 4352, 256, None)])
def test_gemm_k64_matches_fp32(variant, M, N, K, lda):
    """gemm_k64.hip: one tile, the shortest reduction (two K-tiles), a long reduction, a padded row
    stride, and 272 tiles (> 256 CUs: the persistent grid's second, partial round of tiles and
    the cross-tile K pipeline into a tile that another workgroup's round ends on)."""
    C = _C()
    torch.manual_seed(M + N + K + variant)
    a, b = _rand(M, K, ld=lda), _rand(N, K)
    out = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    assert C.gemm_nt(a, b, out, False, variant)
    ref = a.float() @ b.float().t()
    _check(out, ref, f"k64 v{variant} {M}x{N}x{K}")
    out2 = torch.empty_like(out)
    assert C.gemm_nt(a, b, out2, False, variant)
    assert torch.equal(out, out2), "run-to-run difference (race)"
    acc = out.clone()
    assert C.gemm_nt(a, b, acc, True, variant)
    _check(acc, out.float() + ref, f"k64 v{variant} accumulate")


@pytest.mark.parametrize("P,Q,R", [(256, 256, 64), (512, 768, 192), (256, 1280, 1024)])
def test_gemm_wgrad_token_major_matches_fp32(P, Q, R):
    C = _C()
    torch.manual_seed(P * 7 + Q + R)
    x, y = _rand(R, P), _rand(R, Q)
    out = torch.empty(P, Q, device="cuda", dtype=torch.bfloat16)
    assert C.gemm_wgrad2(x, y, out, False)
    ref = x.float().t() @ y.float()
    _check(out, ref, f"tt {P}x{Q}x{R}")
    acc = out.clone()
    assert C.gemm_wgrad2(x, y, acc, True)
    _check(acc, out.float() + ref, "tt accumulate")


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 192), (768, 256, 1024)])
def test_gemm_nn_matches_fp32(M, N, K):
    C = _C()
    torch.manual_seed(M + 3 * N + K)
    a, b = _rand(M, K), _rand(K, N)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    assert C.gemm_nn(a, b, out, False)
    _check(out, a.float() @ b.float(), f"nn {M}x{N}x{K}")
