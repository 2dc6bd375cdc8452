"""Node-wide GPU leases (runtime/gpu_ledger.py): concurrent drivers never share a GPU, a lease dies with
its process, and ``num_gpus`` tasks learn their GPU (VERDICT r2 item 8 / missing #5). GPUs are
fake here (CPU host): only the bookkeeping is under test."""
import multiprocessing as mp
import os
import time

import pytest

from gke_ray_train_amd.runtime import core
from gke_ray_train_amd.runtime.gpu_ledger import GpuLedger


@pytest.fixture
def lease_dir(tmp_path, monkeypatch):
    d = str(tmp_path / "leases")
    monkeypatch.setenv("GRT_GPU_LEASE_DIR", d)
    return d


def test_two_ledgers_never_overlap(lease_dir):
    a, b = GpuLedger(4, lease_dir), GpuLedger(4, lease_dir)
    assert a.try_acquire(3) == [0, 1, 2]
    assert b.try_acquire(2) is None and b.held() == []  # all-or-nothing
    assert b.try_acquire(1) == [3]
    assert a.num_free() == 0 and b.num_free() == 0
    a.release([1])
    assert b.try_acquire(1) == [1]
    a.close()
    b.close()
    assert GpuLedger(4, lease_dir).num_free() == 4


def _hold(d, q):
    led = GpuLedger(2, d)
    q.put(led.try_acquire(2))
    time.sleep(60)


def test_lease_dies_with_its_process(lease_dir):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_hold, args=(lease_dir, q))
    p.start()
    try:
        assert q.get(timeout=60) == [0, 1]
        assert GpuLedger(2, lease_dir).try_acquire(1) is None
    finally:
        p.kill()
        p.join(10)
    assert GpuLedger(2, lease_dir).try_acquire(2) == [0, 1]


def _gpu_ids():
    from gke_ray_train_amd import runtime
    time.sleep(0.5)
    return runtime.get_gpu_ids()


class _Holder:
    def gpus(self):
        from gke_ray_train_amd import runtime
        return runtime.get_gpu_ids()


def test_tasks_get_their_gpu_and_drivers_share_the_ledger(lease_dir, monkeypatch):
    monkeypatch.setenv("GRT_PLACEMENT_TIMEOUT_S", "1")
    r1 = core.Runtime(num_cpus=2, num_gpus=2)
    r2 = core.Runtime(num_cpus=2, num_gpus=2)
    try:
        refs = [r1.submit(_gpu_ids, (), {}, "g", num_cpus=1, num_gpus=1) for _ in range(2)]
        got = sorted(tuple(r1.get(r, timeout=120)) for r in refs)
        assert got == [(0,), (1,)]  # concurrent tasks hold different GPUs and see them
        # driver 1 holds both GPUs with an actor: driver 2 (another job on the node) cannot place one
        st = r1.create_actor(_Holder, (), {}, num_gpus=2, name="h1")
        assert sorted(st.gpus) == [0, 1]
        with pytest.raises(RuntimeError, match="cannot place actor"):
            r2.create_actor(_Holder, (), {}, num_gpus=1, name="h2")
        st.kill()
        st2 = r2.create_actor(_Holder, (), {}, num_gpus=1, name="h3")
        assert r2.get(st2.call("gpus", (), {}), timeout=120) == [0]
        st2.kill()
    finally:
        r1.shutdown()
        r2.shutdown()
