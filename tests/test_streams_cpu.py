"""CU-mask construction for side streams (ops/streams.py) — host-side logic only."""
import pytest

from gke_ray_train_amd.ops.streams import cu_mask_words


@pytest.mark.parametrize("n", [1, 16, 32, 64, 96, 256])
def test_cu_mask_spread_selects_n_distinct_cus(n):
    w = cu_mask_words(n, 256, "spread")
    assert len(w) == 8 and all(0 <= x < 2 ** 32 for x in w)
    bits = [i for i in range(256) if w[i // 32] >> (i % 32) & 1]
    assert len(bits) == n
    if n > 1:  # evenly spaced over the whole CU range
        gaps = {b - a for a, b in zip(bits, bits[1:])}
        assert max(gaps) - min(gaps) <= 1


def test_cu_mask_low_and_bounds():
    w = cu_mask_words(40, 256, "low")
    assert w[0] == 0xFFFFFFFF and w[1] == 0xFF and not any(w[2:])
    with pytest.raises(ValueError):
        cu_mask_words(0, 256)
    with pytest.raises(ValueError):
        cu_mask_words(300, 256)
    with pytest.raises(ValueError):
        cu_mask_words(8, 256, "diagonal")
