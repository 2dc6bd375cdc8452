"""CPU checks of the weight-gradient operand hand-off in ops/linear.py: a producer kernel may attach
the transposed copy of its output (``_grt_T``, ops.fused.swiglu); the consuming projection takes it
exactly once and only when it is the [C, M] transpose of the 2-D view it needs."""
import torch

from gke_ray_train_amd.models.llama import _direct_wgrad
from gke_ray_train_amd.ops import linear as L


def test_provided_transposed_is_taken_once_and_shape_checked():
    t = torch.randn(2, 64, 128).bfloat16()
    t2 = t.reshape(-1, 128)
    t._grt_T = t2.t().contiguous()
    got = L.provided_transposed(t2, t)
    assert got is not None and torch.equal(got, t2.t())
    assert not hasattr(t, "_grt_T") and L.provided_transposed(t2, t) is None  # consumed
    t._grt_T = torch.empty(64, 128, dtype=torch.bfloat16)  # not [C, M]
    assert L.provided_transposed(t2, t) is None and not hasattr(t, "_grt_T")
    u = torch.randn(100, 128).bfloat16()  # M not a multiple of 64: the TN path does not apply
    u._grt_T = u.t().contiguous()
    assert L.provided_transposed(u, u) is None
    v = torch.randn(128, 128)  # fp32
    v._grt_T = v.t().contiguous()
    assert L.provided_transposed(v, v) is None


def test_direct_wgrad_needs_a_trainable_slotted_device_weight():
    lin = L.Linear(128, 64, bias=False)
    assert not _direct_wgrad(lin)  # CPU weight, no gradient slot
    lin.weight._grt_slot = L.GradSlot(torch.empty(64, 128), lambda p: None)
    assert not _direct_wgrad(lin)  # still a CPU weight
    lin.weight.requires_grad_(False)
    assert not _direct_wgrad(lin)
