"""Shared-memory object store for large task arguments/results (the plasma role).

Values are serialised with pickle protocol 5; every out-of-band buffer larger than
``INLINE_LIMIT`` (numpy arrays, CPU torch tensors via their numpy view) is copied ONCE into a POSIX
shared-memory segment and the consumer maps it zero-copy. Small values stay inline in the
message. Segments are unlinked by the consumer after it has mapped them (single-reader objects,
which is how task results and actor arguments are used here).
"""
from __future__ import annotations

import pickle
import uuid
from multiprocessing import shared_memory

import cloudpickle

INLINE_LIMIT = 1 << 20


class _ShmBuf:
    __slots__ = ("name", "size")

    def __init__(self, name, size):
        self.name, self.size = name, size


def pack(value) -> bytes:
    bufs = []
    data = cloudpickle.dumps(value, protocol=5, buffer_callback=bufs.append)
    out_bufs = []
    for b in bufs:
        raw = b.raw()
        if raw.nbytes > INLINE_LIMIT:
            name = "grt_" + uuid.uuid4().hex[:20]
            shm = shared_memory.SharedMemory(name=name, create=True, size=raw.nbytes)
            shm.buf[:raw.nbytes] = raw.cast("B")
            shm.close()
            _untrack(name)
            out_bufs.append(_ShmBuf(name, raw.nbytes))
        else:
            out_bufs.append(bytes(raw.cast("B")))
    return pickle.dumps((data, out_bufs), protocol=5)


def unpack(payload: bytes):
    data, bufs = pickle.loads(payload)
    views = []
    keep = []
    for b in bufs:
        if isinstance(b, _ShmBuf):
            shm = shared_memory.SharedMemory(name=b.name)
            _untrack(b.name)
            mv = bytearray(shm.buf[:b.size])  # private copy, then release the segment
            shm.close()
            try:
                shm.unlink()
            except FileNotFoundError:
                pass
            views.append(mv)
        else:
            views.append(b)
    return pickle.loads(data, buffers=views)


def _untrack(name):
    # The resource tracker would unlink segments when the *creating* process exits; ownership
    # is handed to the consumer instead.
    try:
        from multiprocessing import resource_tracker
        resource_tracker.unregister("/" + name, "shared_memory")
    except Exception:
        pass


class _Packed:
    __slots__ = ("payload",)

    def __init__(self, payload):
        self.payload = payload


def pack_args(obj):
    """Arguments: large values are moved through shared memory, small ones stay inline."""
    return _Packed(pack(obj))


def materialize(obj):
    if isinstance(obj, _Packed):
        return unpack(obj.payload)
    return obj
