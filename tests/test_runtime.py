"""Node-local runtime: tasks, ObjectRefs, get(timeout), error propagation, actors, worker death."""
import os
import time

import numpy as np
import pytest

from gke_ray_train_amd import runtime as rt


@pytest.fixture(scope="module", autouse=True)
def _runtime():
    rt.init(num_cpus=4, num_gpus=0, ignore_reinit_error=True)
    yield
    rt.shutdown()


@rt.remote(num_cpus=1)
def add(a, b):
    return a + b


@rt.remote
def boom():
    raise ValueError("kaboom")


@rt.remote
def sleepy(t):
    time.sleep(t)
    return t


@rt.remote
def big(n):
    return np.arange(n, dtype=np.float32)


@rt.remote
def die():
    os._exit(3)


@rt.remote
class Counter:
    def __init__(self, start):
        self.n = start

    def inc(self, k=1):
        self.n += k
        return self.n

    def pid(self):
        return os.getpid()


def test_task_and_deps():
    r1 = add.remote(1, 2)
    r2 = add.remote(r1, 10)  # ObjectRef dependency
    assert rt.get(r2, timeout=60) == 13
    assert rt.get([add.remote(i, i) for i in range(6)], timeout=60) == [2 * i for i in range(6)]
    assert rt.is_initialized()


def test_put_get():
    r = rt.put({"a": 1})
    assert rt.get(r) == {"a": 1}


def test_error_propagates():
    with pytest.raises(rt.RayTaskError) as ei:
        rt.get(boom.remote(), timeout=60)
    assert "kaboom" in str(ei.value)
    assert isinstance(ei.value.cause, ValueError)


def test_get_timeout():
    r = sleepy.remote(3)
    with pytest.raises(rt.GetTimeoutError):
        rt.get(r, timeout=0.2)
    assert rt.get(r, timeout=60) == 3


def test_large_result_via_shared_memory():
    a = rt.get(big.remote(3_000_000), timeout=60)
    assert a.shape == (3_000_000,) and a[-1] == 2_999_999


def test_worker_death_is_an_error():
    with pytest.raises(rt.WorkerCrashedError):
        rt.get(die.remote(), timeout=60)
    assert rt.get(add.remote(2, 2), timeout=60) == 4  # runtime still usable


def test_actor_state_and_kill():
    c = Counter.remote(5)
    assert rt.get(c.inc.remote(), timeout=60) == 6
    assert rt.get(c.inc.remote(k=4), timeout=60) == 10
    pid = rt.get(c.pid.remote(), timeout=60)
    assert pid != os.getpid()
    rt.kill(c)
    with pytest.raises(rt.ActorDiedError):
        rt.get(c.inc.remote(), timeout=60)


def test_wait():
    refs = [sleepy.remote(0.01), sleepy.remote(2.0)]
    ready, rest = rt.wait(refs, num_returns=1, timeout=30)
    assert len(ready) == 1 and len(rest) == 1
