"""Device-driven HBM <-> pinned-host copy (csrc/kernels/optim.hip ``stream_copy``), the offloaded
optimizer's moment write-back: exact in both directions for sizes that do not divide the grid
(tails), with plain and non-temporal stores; unaligned / unpinned operands are refused."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from gke_ray_train_amd import _native
    return _native.kernels()


@pytest.mark.parametrize("n", [4, 1024 + 4, (1 << 20) + 36, 3 * (1 << 22)])
@pytest.mark.parametrize("nt", [False, True])
@pytest.mark.parametrize("nblocks", [1, 7, 128])
def test_stream_copy_round_trip(n, nt, nblocks):
    C = _C()
    g = torch.Generator().manual_seed(n)
    src_h = torch.randn(n, generator=g).pin_memory()
    dev = torch.empty(n, device="cuda")
    C.stream_copy(src_h, dev, nblocks, nt)  # host -> device (the kernel reads mapped host memory)
    back = torch.full((n,), float("nan")).pin_memory()
    C.stream_copy(dev, back, nblocks, nt)  # device -> host
    torch.cuda.synchronize()
    assert torch.equal(dev.cpu(), src_h)
    assert torch.equal(back, src_h)


def test_stream_copy_refuses_bad_operands():
    C = _C()
    d = torch.zeros(64, device="cuda")
    with pytest.raises(RuntimeError):
        C.stream_copy(d, torch.zeros(64), 8, True)  # not pinned
    with pytest.raises(RuntimeError):
        C.stream_copy(d[1:], torch.zeros(64).pin_memory()[1:], 8, True)  # 4-byte offset, 252 bytes
    with pytest.raises(RuntimeError):
        C.stream_copy(d, torch.zeros(32).pin_memory(), 8, True)  # size mismatch
