"""Native shared-memory ring (csrc/runtime/shm_ring.cpp): ordering, back-pressure, timeouts,
close semantics, zero-copy slots, and a producer process streaming token batches."""
import multiprocessing as mp
import time

import numpy as np
import pytest

from gke_ray_train_amd.runtime.shm_ring import RingBatchStream, RingClosed, RingTimeout, ShmRing


def _producer(name, n):
    r = ShmRing(name)
    for i in range(n):
        r.push(np.full(1000 + (i % 7), i, dtype=np.int32))
    r.close()


def test_ring_cross_process_order_and_close():
    name = f"/grt_test_ring_{time.time_ns()}"
    ring = ShmRing(name, slot_bytes=8192, n_slots=4, create=True)
    p = mp.get_context("spawn").Process(target=_producer, args=(name, 500))
    p.start()
    got = []
    while True:
        try:
            a = ring.pop(timeout=60).view(np.int32)
        except RingClosed:
            break
        assert len(a) == 1000 + (len(got) % 7) and (a == len(got)).all()
        got.append(int(a[0]))
    p.join(30)
    assert p.exitcode == 0 and got == list(range(500))
    ring.destroy()


def test_ring_backpressure_timeout_and_zero_copy():
    ring = ShmRing(f"/grt_test_ring2_{time.time_ns()}", slot_bytes=64, n_slots=2, create=True)
    ring.push(b"a" * 10)
    ring.push(b"b" * 20)
    assert len(ring) == 2
    with pytest.raises(RingTimeout):
        ring.push(b"c", timeout=0.05)  # full
    with pytest.raises(ValueError):
        ring.push(b"x" * 65)
    v = ring.read_slot()
    assert bytes(v) == b"a" * 10
    ring.release()
    view, commit = ring.write_slot()
    view[:3] = np.frombuffer(b"xyz", dtype=np.uint8)
    commit(3)
    assert bytes(ring.pop()) == b"b" * 20
    assert bytes(ring.pop()) == b"xyz"
    with pytest.raises(RingTimeout):
        ring.pop(timeout=0.05)
    ring.close()
    with pytest.raises(RingClosed):
        ring.pop(timeout=1)
    ring.destroy()


def _token_batches():
    rng = np.random.default_rng(0)
    toks = rng.integers(0, 32000, 100_000)
    for i in range(20):
        s = rng.integers(0, len(toks) - 129, 8)
        x = np.stack([toks[j:j + 128] for j in s])
        y = np.stack([toks[j + 1:j + 129] for j in s])
        yield {"input_ids": x[: 8 if i < 19 else 5], "labels": y[: 8 if i < 19 else 5]}


def test_ring_batch_stream_producer_process():
    stream = RingBatchStream(_token_batches, {"input_ids": ("int64", (8, 128)), "labels": ("int64", (8, 128))})
    ref = list(_token_batches())
    got = list(stream)
    assert len(got) == len(ref) == 20
    for a, b in zip(got, ref):
        assert np.array_equal(a["input_ids"], b["input_ids"]) and np.array_equal(a["labels"], b["labels"])
    assert got[-1]["input_ids"].shape == (5, 128)
