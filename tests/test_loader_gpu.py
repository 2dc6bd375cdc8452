"""``train.torch.prepare_data_loader`` on the GPU: batches copied on a side stream are recorded on the
compute stream, so every batch a slow consumer reads is intact even while the
loader keeps dropping and re-allocating batch memory one step ahead."""
import pytest
import torch
from torch.utils.data import DataLoader, TensorDataset

pytestmark = pytest.mark.gpu


def test_device_loader_batches_survive_slow_consumer():
    from gke_ray_train_amd.train.torch import _DeviceLoader
    dev = torch.device("cuda", 0)
    n, d = 64, 1 << 16
    data = torch.arange(n, dtype=torch.float32).view(n, 1).expand(n, d).contiguous()
    loader = _DeviceLoader(DataLoader(TensorDataset(data), batch_size=2, shuffle=False), dev)
    w = torch.randn(512, 512, device=dev)
    sums = []
    for (b,) in loader:
        x = w
        for _ in range(20):  # keep the compute stream busy so the copy stream runs ahead
            x = x @ w
        sums.append(b.sum(dim=1) + 0 * x[0, 0])
        del b  # the loader's reference is the last one: memory goes back to the allocator
    got = torch.stack(sums).cpu()
    want = data.sum(dim=1).view(-1, 2)
    assert torch.equal(got, want)
