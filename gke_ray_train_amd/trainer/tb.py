"""Minimal TensorBoard event-file writer (scalars), no tensorboard dependency.

The reference sets ``report_to="tensorboard"`` (fine_tune_config.json:26) and names its BasicLLM
experiment after TensorBoard (pytorch_llm_ray.py:320). tensorboard is not installed here, so this
writes ``events.out.tfevents.<ts>.<host>`` records directly: TFRecord framing (length, masked
CRC32C of the length, payload, masked CRC32C of the payload) around hand-encoded ``Event`` /
``Summary`` protobufs (wall_time=1, step=2, summary=5 / value=1 {tag=1, simple_value=2}).
"""
from __future__ import annotations

import os
import socket
import struct
import time


def _crc32c_table():
    poly = 0x82F63B78
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        t.append(c)
    return t


_T = _crc32c_table()


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _T[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked(c: int) -> int:
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wire: int, payload: bytes) -> bytes:
    return _varint((num << 3) | wire) + payload


def _event(step: int, wall: float, tag: str = None, value: float = None, file_version: str = None) -> bytes:
    ev = _field(1, 1, struct.pack("<d", wall)) + _field(2, 0, _varint(step))
    if file_version is not None:
        fv = file_version.encode()
        ev += _field(3, 2, _varint(len(fv)) + fv)
    if tag is not None:
        tb = tag.encode()
        val = _field(1, 2, _varint(len(tb)) + tb) + _field(2, 5, struct.pack("<f", float(value)))
        summ = _field(1, 2, _varint(len(val)) + val)
        ev += _field(5, 2, _varint(len(summ)) + summ)
    return ev


class SummaryWriter:
    def __init__(self, log_dir: str):
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}")
        self.f = open(self.path, "wb")
        self._write(_event(0, time.time(), file_version="brain.Event:2"))

    def _write(self, rec: bytes):
        hdr = struct.pack("<Q", len(rec))
        self.f.write(hdr + struct.pack("<I", _masked(crc32c(hdr))) + rec + struct.pack("<I", _masked(crc32c(rec))))

    def add_scalar(self, tag: str, value: float, global_step: int = 0, walltime: float = None):
        self._write(_event(global_step, walltime or time.time(), tag, value))

    def flush(self):
        self.f.flush()

    def close(self):
        self.f.close()


def read_scalars(path: str):
    """Parse back (tag, step, value) records — used by the tests."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        rec = data[i + 12:i + 12 + n]
        i += 12 + n + 4
        j, step, tag, val = 0, 0, None, None

        def rv(b, k):
            r, s = 0, 0
            while True:
                x = b[k]
                k += 1
                r |= (x & 0x7F) << s
                s += 7
                if not x & 0x80:
                    return r, k
        while j < len(rec):
            key, j = rv(rec, j)
            fn, wt = key >> 3, key & 7
            if wt == 0:
                v, j = rv(rec, j)
                if fn == 2:
                    step = v
            elif wt == 1:
                j += 8
            elif wt == 5:
                j += 4
            elif wt == 2:
                ln, j = rv(rec, j)
                sub = rec[j:j + ln]
                j += ln
                if fn == 5:
                    _, k = rv(sub, 0)
                    vl, k = rv(sub, k)
                    v = sub[k:k + vl]
                    _, m = rv(v, 0)
                    tl, m = rv(v, m)
                    tag = v[m:m + tl].decode()
                    m += tl + 1
                    (val,) = struct.unpack_from("<f", v, m)
        if tag is not None:
            out.append((tag, step, val))
    return out
