"""Token datasets and the HBM streaming loader.

* ``TextDataset`` — the reference's sliding-window next-char dataset (ray-jobs/pytorch_llm_ray.py:
  107-119): item i = (ids[i:i+S], ids[i+1:i+S+1]), len = N - S - 1.
* ``TokenBatchLoader`` — the MI355X input path: a worker thread assembles each batch of windows with
  ONE native call (``_rt.so`` ``grt_gather_windows_*``) into a pinned host buffer from a small ring,
  and the H2D copy is issued on a side HIP stream one batch ahead, so the training stream never
  waits on Python indexing, collation or a pageable copy.
"""
from __future__ import annotations

import ctypes
import queue
import threading
from typing import Optional

import numpy as np
import torch
from torch.utils.data import Dataset

from .. import _native


class TextDataset(Dataset):
    def __init__(self, token_ids_tensor: torch.Tensor, seq_len: int):
        self.token_ids = token_ids_tensor
        self.seq_len = seq_len
        self.num_sequences = max(0, len(self.token_ids) - self.seq_len - 1)

    def __len__(self) -> int:
        return self.num_sequences

    def __getitem__(self, idx: int):
        return self.token_ids[idx: idx + self.seq_len], self.token_ids[idx + 1: idx + self.seq_len + 1]


def gather_windows(tokens: np.ndarray, starts: np.ndarray, seq_len: int, out_x: Optional[np.ndarray] = None,
                   out_y: Optional[np.ndarray] = None, nthreads: int = 4):
    """Native batch assembly: out_x[b] = tokens[s_b : s_b+S], out_y[b] = tokens[s_b+1 : s_b+S+1]."""
    lib = _native.runtime_lib()
    B = len(starts)
    starts = np.ascontiguousarray(starts, dtype=np.int64)
    out_x = np.empty((B, seq_len), dtype=np.int64) if out_x is None else out_x
    out_y = np.empty((B, seq_len), dtype=np.int64) if out_y is None else out_y
    P = ctypes.c_void_p
    if tokens.dtype == np.int64:
        fn = lib.grt_gather_windows_i64
    elif tokens.dtype == np.int32:
        fn = lib.grt_gather_windows_i32
    else:
        raise TypeError(f"tokens must be int32/int64, got {tokens.dtype}")
    fn.restype = ctypes.c_int
    rc = fn(P(tokens.ctypes.data), ctypes.c_int64(len(tokens)), P(starts.ctypes.data), ctypes.c_int64(B),
            ctypes.c_int64(seq_len), P(out_x.ctypes.data), P(out_y.ctypes.data), ctypes.c_int(nthreads))
    if rc != 0:
        raise IndexError("window out of range")
    return out_x, out_y


class TokenBatchLoader:
    """Sharded, shuffled, prefetching loader of (inputs, targets) windows, yielding device tensors.

    ``rank``/``world`` shard the window index space like a DistributedSampler; ``set_epoch``
    reshuffles. ``max_windows`` caps the windows used (the reference's ``test_run`` keeps the
    first 16,000, ray-jobs/pytorch_llm_ray.py:198-201).
    """

    def __init__(self, tokens, seq_len: int, batch_size: int, device=None, rank: int = 0, world: int = 1,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = True, max_windows: Optional[int] = None,
                 prefetch: int = 2, stride: int = 1):
        self.tokens = tokens.numpy() if isinstance(tokens, torch.Tensor) else np.asarray(tokens)
        self.S = seq_len
        self.B = batch_size
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.rank, self.world = rank, world
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        n = max(0, (len(self.tokens) - seq_len - 1 + stride - 1) // stride) if stride > 1 else max(0, len(self.tokens) - seq_len - 1)
        if max_windows is not None:
            n = min(n, max_windows)
        self.n_windows = n
        self.stride = stride
        self.prefetch = max(1, prefetch)
        self.epoch = 0
        self.pin = self.device.type == "cuda"

    def set_epoch(self, e: int):
        self.epoch = e

    def _indices(self):
        idx = np.arange(self.n_windows, dtype=np.int64)
        if self.shuffle:
            rng = np.random.default_rng(self.seed + self.epoch)
            rng.shuffle(idx)
        per = (len(idx) // self.world) if self.drop_last else -(-len(idx) // self.world)
        mine = idx[self.rank * per: (self.rank + 1) * per] if self.drop_last else idx[self.rank::self.world]
        return mine * self.stride

    def __len__(self):
        per = len(self._indices())
        return per // self.B if self.drop_last else -(-per // self.B)

    def __iter__(self):
        starts = self._indices()
        nb = len(self)
        ring = [(torch.empty((self.B, self.S), dtype=torch.long, pin_memory=self.pin),
                 torch.empty((self.B, self.S), dtype=torch.long, pin_memory=self.pin)) for _ in range(self.prefetch + 1)]
        q: "queue.Queue" = queue.Queue(maxsize=self.prefetch)
        free: "queue.Queue" = queue.Queue()
        for i in range(len(ring)):
            free.put(i)
        stop = threading.Event()

        def producer():
            for b in range(nb):
                if stop.is_set():
                    return
                slot = free.get()
                s = starts[b * self.B:(b + 1) * self.B]
                x, y = ring[slot]
                xb, yb = x[: len(s)], y[: len(s)]
                gather_windows(self.tokens, s, self.S, xb.numpy(), yb.numpy())
                q.put((slot, len(s)))
            q.put(None)

        th = threading.Thread(target=producer, daemon=True)
        th.start()
        stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        pending = []  # (slot, event): pinned slots whose H2D copy may still be in flight
        try:
            while True:
                while pending and pending[0][1].query():
                    free.put(pending.pop(0)[0])
                if q.empty() and pending:  # producer may be starved of slots: retire the oldest copy
                    s0, ev0 = pending.pop(0)
                    ev0.synchronize()
                    free.put(s0)
                item = q.get()
                if item is None:
                    break
                slot, n = item
                x, y = ring[slot]
                if stream is not None:
                    with torch.cuda.stream(stream):
                        xd = x[:n].to(self.device, non_blocking=True)
                        yd = y[:n].to(self.device, non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(stream)
                    torch.cuda.current_stream(self.device).wait_event(ev)
                    xd.record_stream(torch.cuda.current_stream(self.device))
                    yd.record_stream(torch.cuda.current_stream(self.device))
                    pending.append((slot, ev))
                else:
                    xd, yd = x[:n].clone(), y[:n].clone()
                    free.put(slot)
                yield xd, yd
        finally:
            stop.set()
            while not free.empty():
                free.get_nowait()
            for i in range(len(ring)):
                free.put(i)
            th.join(timeout=5)


def synthetic_tokens(n_tokens: int, vocab_size: int, seed: int = 0, zipf: float = 1.1) -> np.ndarray:
    """Synthetic Zipf-distributed token stream (Wikitext-shaped statistics) for LM benchmarks."""
    rng = np.random.default_rng(seed)
    ranks = np.arange(1, vocab_size + 1, dtype=np.float64)
    p = ranks ** (-zipf)
    p /= p.sum()
    return rng.choice(vocab_size, size=n_tokens, p=p).astype(np.int32)
