"""Python side of the native shared-memory ring (csrc/runtime/shm_ring.cpp) and a process-backed
batch stream built on it.

``ShmRing`` is a single-producer / single-consumer ring of fixed-size slots in ``/dev/shm``;
``RingBatchStream`` runs a batch generator in a separate (spawned) producer process — the role of a
Ray Data streaming worker — and yields its batches to the training process as
numpy arrays read straight out of the shared slots (one memcpy into the caller's buffer, usually
a pinned staging tensor for the async H2D copy). Batches are dicts of fixed-schema arrays.
"""
from __future__ import annotations

import ctypes
import json
import multiprocessing as mp
import os
import uuid
from typing import Callable, Dict, Iterator, Optional, Tuple

import numpy as np

from .. import _native

_c = None


def _lib():
    global _c
    if _c is None:
        lib = _native.runtime_lib()
        vp, u64, i64, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int
        sig = {
            "grt_ring_create": (vp, [ctypes.c_char_p, u64, u64]),
            "grt_ring_open": (vp, [ctypes.c_char_p]),
            "grt_ring_slot_size": (u64, [vp]),
            "grt_ring_capacity": (u64, [vp]),
            "grt_ring_size": (u64, [vp]),
            "grt_ring_acquire_write": (vp, [vp, i64, ctypes.POINTER(ci)]),
            "grt_ring_commit_write": (ci, [vp, u64]),
            "grt_ring_push": (ci, [vp, vp, u64, i64]),
            "grt_ring_acquire_read": (vp, [vp, i64, ctypes.POINTER(u64), ctypes.POINTER(ci)]),
            "grt_ring_release_read": (ci, [vp]),
            "grt_ring_pop": (i64, [vp, vp, u64, i64]),
            "grt_ring_close": (None, [vp]),
            "grt_ring_closed": (ci, [vp]),
            "grt_ring_destroy": (None, [vp, ctypes.c_char_p, ci]),
        }
        for name, (res, args) in sig.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        _c = lib
    return _c


class RingTimeout(TimeoutError):
    pass


class RingClosed(EOFError):
    pass


class ShmRing:
    def __init__(self, name: str, slot_bytes: int = 0, n_slots: int = 0, create: bool = False):
        self.name = name if name.startswith("/") else "/" + name
        self._create = create
        c = _lib()
        self._h = c.grt_ring_create(self.name.encode(), slot_bytes, n_slots) if create else \
            c.grt_ring_open(self.name.encode())
        if not self._h:
            raise OSError(f"shm ring {self.name}: {'create' if create else 'open'} failed")
        self.slot_bytes = int(c.grt_ring_slot_size(self._h))
        self.capacity = int(c.grt_ring_capacity(self._h))

    def __len__(self):
        return int(_lib().grt_ring_size(self._h))

    def push(self, data, timeout: float = -1.0):
        buf = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray))
                                   else data).view(np.uint8).reshape(-1)
        rc = _lib().grt_ring_push(self._h, buf.ctypes.data, buf.nbytes, int(timeout * 1000) if timeout >= 0 else -1)
        self._check(rc)

    def write_slot(self, timeout: float = -1.0) -> Tuple[np.ndarray, Callable[[int], None]]:
        """Zero-copy produce: (uint8 view of the free slot, commit(nbytes))."""
        err = ctypes.c_int(0)
        p = _lib().grt_ring_acquire_write(self._h, int(timeout * 1000) if timeout >= 0 else -1, ctypes.byref(err))
        if not p:
            self._check(err.value)
        view = np.ctypeslib.as_array((ctypes.c_uint8 * self.slot_bytes).from_address(p))

        def commit(nbytes: int):
            self._check(_lib().grt_ring_commit_write(self._h, nbytes))
        return view, commit

    def read_slot(self, timeout: float = -1.0) -> np.ndarray:
        """Zero-copy consume: uint8 view of the oldest filled slot; call ``release()`` when done."""
        n = ctypes.c_uint64(0)
        err = ctypes.c_int(0)
        p = _lib().grt_ring_acquire_read(self._h, int(timeout * 1000) if timeout >= 0 else -1, ctypes.byref(n),
                                         ctypes.byref(err))
        if not p:
            self._check(err.value)
        return np.ctypeslib.as_array((ctypes.c_uint8 * n.value).from_address(p))

    def release(self):
        _lib().grt_ring_release_read(self._h)

    def pop(self, out: Optional[np.ndarray] = None, timeout: float = -1.0) -> np.ndarray:
        if out is None:
            out = np.empty(self.slot_bytes, dtype=np.uint8)
        o = out.view(np.uint8).reshape(-1)
        rc = _lib().grt_ring_pop(self._h, o.ctypes.data, o.nbytes, int(timeout * 1000) if timeout >= 0 else -1)
        self._check(rc)
        return o[:rc]

    def close(self):
        _lib().grt_ring_close(self._h)

    @property
    def closed(self) -> bool:
        return bool(_lib().grt_ring_closed(self._h))

    def destroy(self):
        if self._h:
            _lib().grt_ring_destroy(self._h, self.name.encode(), 1 if self._create else 0)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    @staticmethod
    def _check(rc):
        if rc == -1:
            raise RingTimeout("shm ring: timed out")
        if rc == -2:
            raise RingClosed("shm ring: closed")
        if rc == -3:
            raise ValueError("shm ring: payload larger than the slot")
        if rc is not None and rc < 0:
            raise OSError(f"shm ring error {rc}")


# ------------------------------------------------------------------------------- batch stream
Schema = Dict[str, Tuple[str, Tuple[int, ...]]]


def _layout(schema: Schema):
    off, out = 0, {}
    for k, (dt, shape) in schema.items():
        n = int(np.prod(shape)) * np.dtype(dt).itemsize
        out[k] = (off, np.dtype(dt), tuple(shape), n)
        off += (n + 63) // 64 * 64
    return out, off


def _producer_main(name: str, payload: bytes, schema_json: str):
    import cloudpickle
    make_iter = cloudpickle.loads(payload)
    schema = {k: (v[0], tuple(v[1])) for k, v in json.loads(schema_json).items()}
    lay, _ = _layout(schema)
    ring = ShmRing(name)
    try:
        for batch in make_iter():
            view, commit = ring.write_slot()
            rows = None
            for k, (off, dt, shape, n) in lay.items():
                a = np.ascontiguousarray(batch[k], dtype=dt)
                if a.shape[1:] != shape[1:] or a.shape[0] > shape[0]:
                    raise ValueError(f"batch field {k}: shape {a.shape} does not fit schema {shape}")
                rows = a.shape[0] if rows is None else rows
                view[off:off + a.nbytes] = a.view(np.uint8).reshape(-1)
            view[-8:] = np.frombuffer(np.int64(rows or 0).tobytes(), dtype=np.uint8)
            commit(len(view))
    except RingClosed:
        pass
    finally:
        ring.close()


class RingBatchStream:
    """Iterate batches produced by ``make_iter()`` in a separate process, through an ShmRing.

    ``schema`` gives each field's dtype and MAXIMUM shape (first dim = rows; a shorter last batch
    is allowed). Yields dicts of numpy arrays copied out of the slot (``copy=False`` yields views
    valid until the next iteration step).
    """

    def __init__(self, make_iter: Callable[[], Iterator[Dict[str, np.ndarray]]], schema: Schema, n_slots: int = 4,
                 copy: bool = True, timeout: float = 300.0):
        import cloudpickle
        self.schema = {k: (np.dtype(d).str, tuple(s)) for k, (d, s) in schema.items()}
        self._lay, body = _layout(self.schema)
        self.slot_bytes = body + 64
        self.copy = copy
        self.timeout = timeout
        self.name = f"/grt_ring_{os.getpid()}_{uuid.uuid4().hex[:10]}"
        self.ring = ShmRing(self.name, self.slot_bytes, n_slots, create=True)
        ctx = mp.get_context("spawn")
        self.proc = ctx.Process(target=_producer_main, daemon=True,
                                args=(self.name, cloudpickle.dumps(make_iter),
                                      json.dumps({k: [d, list(s)] for k, (d, s) in self.schema.items()})))
        self.proc.start()

    def __iter__(self):
        try:
            while True:
                try:
                    view = self.ring.read_slot(timeout=self.timeout)
                except RingClosed:
                    break
                except RingTimeout:
                    if not self.proc.is_alive():
                        raise RuntimeError(f"batch producer died (exit code {self.proc.exitcode})") from None
                    raise
                rows = int(np.frombuffer(view[self.slot_bytes - 8:self.slot_bytes].tobytes(), dtype=np.int64)[0])
                out = {}
                for k, (off, dt, shape, n) in self._lay.items():
                    cnt = rows * (n // shape[0]) if shape else n
                    a = view[off:off + cnt].view(dt).reshape((rows,) + shape[1:])
                    out[k] = a.copy() if self.copy else a
                yield out
                self.ring.release()
        finally:
            self.shutdown()

    def shutdown(self):
        if self.ring is not None:
            self.ring.close()
            self.proc.join(timeout=10)
            if self.proc.is_alive():
                self.proc.kill()
                self.proc.join(timeout=5)
            self.ring.destroy()
            self.ring = None
