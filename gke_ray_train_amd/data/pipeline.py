"""A streaming, block-parallel dataset (the Ray Data surface used for the data pipeline).

``BASELINE.json`` asks for the Wikitext-2 preparation to become a Ray-Data pipeline that shards
and streams token batches into HBM. Semantics follow Ray Data where the reference ecosystem uses
it: lazy transforms (``map``, ``map_batches``, ``filter``, ``flat_map``, ``random_shuffle``),
``split``/``streaming_split(n)`` for per-rank shards (``train.get_dataset_shard``), and
``iter_batches`` / ``iter_torch_batches`` consumption.

Execution model on one node: data is a list of columnar blocks (``dict[str, np.ndarray]``);
transforms are applied block by block WHEN the block is consumed (streaming), with a producer
thread running one or more blocks ahead of the consumer; ``materialize()`` runs the transforms
of all blocks as parallel runtime tasks when the node-local runtime is up. Torch batches are
assembled in pinned host memory and copied to the GPU with non-blocking H2D copies.
"""
from __future__ import annotations

import os
import queue
import threading
from typing import Any, Callable, Dict, Iterable, Iterator, List, Optional

import numpy as np

Block = Dict[str, np.ndarray]


def _rows_to_block(rows: List[Any]) -> Block:
    if not rows:
        return {}
    if isinstance(rows[0], dict):
        keys = list(rows[0].keys())
        out = {}
        for k in keys:
            vals = [r[k] for r in rows]
            try:
                out[k] = np.asarray(vals)
                if out[k].dtype == object and not isinstance(vals[0], (str, bytes)):
                    out[k] = np.array(vals, dtype=object)
            except Exception:
                out[k] = np.array(vals, dtype=object)
        return out
    return {"item": np.asarray(rows)}


def _block_len(b: Block) -> int:
    for v in b.values():
        return len(v)
    return 0


def _block_rows(b: Block) -> Iterator[Dict[str, Any]]:
    n = _block_len(b)
    keys = list(b.keys())
    for i in range(n):
        yield {k: b[k][i] for k in keys}


def _slice(b: Block, s: int, e: int) -> Block:
    return {k: v[s:e] for k, v in b.items()}


def _concat(blocks: List[Block]) -> Block:
    blocks = [b for b in blocks if _block_len(b)]
    if not blocks:
        return {}
    return {k: np.concatenate([b[k] for b in blocks]) for k in blocks[0]}


def _apply_ops(block: Block, ops) -> Block:
    for kind, fn, kw in ops:
        if not _block_len(block):
            break
        if kind == "map":
            block = _rows_to_block([fn(r) for r in _block_rows(block)])
        elif kind == "flat_map":
            block = _rows_to_block([x for r in _block_rows(block) for x in fn(r)])
        elif kind == "filter":
            keep = np.array([bool(fn(r)) for r in _block_rows(block)], dtype=bool)
            block = {k: v[keep] for k, v in block.items()}
        elif kind == "map_batches":
            bs = kw.get("batch_size")
            n = _block_len(block)
            bs = n if not bs or bs <= 0 else bs
            outs = []
            for s in range(0, n, bs):
                part = _slice(block, s, min(n, s + bs))
                fmt = kw.get("batch_format", "numpy")
                if fmt == "pandas":
                    import pandas as pd
                    res = fn(pd.DataFrame({k: list(v) if v.ndim > 1 else v for k, v in part.items()}))
                    res = {c: np.asarray(res[c].tolist()) for c in res.columns}
                else:
                    res = fn(part, **kw.get("fn_kwargs", {}))
                outs.append({k: np.asarray(v) for k, v in res.items()})
            block = _concat(outs)
        elif kind == "shuffle":
            rng = np.random.default_rng(kw.get("seed"))
            perm = rng.permutation(_block_len(block))
            block = {k: v[perm] for k, v in block.items()}
        elif kind == "select":
            block = {k: block[k] for k in fn}
    return block


def _run_block(block, ops):
    return _apply_ops(block, ops)


class Dataset:
    def __init__(self, blocks: List[Block], ops=None):
        self._blocks = blocks
        self._ops = list(ops or [])

    # ------------------------------------------------------------------ creation
    @staticmethod
    def from_items(items: List[Any], parallelism: int = 8) -> "Dataset":
        n = len(items)
        k = max(1, min(parallelism, n))
        bounds = np.linspace(0, n, k + 1).astype(int)
        return Dataset([_rows_to_block(items[bounds[i]:bounds[i + 1]]) for i in range(k)])

    @staticmethod
    def range(n: int, parallelism: int = 8) -> "Dataset":
        bounds = np.linspace(0, n, max(1, parallelism) + 1).astype(np.int64)
        return Dataset([{"id": np.arange(bounds[i], bounds[i + 1])} for i in range(len(bounds) - 1)])

    @staticmethod
    def from_numpy(arr, parallelism: int = 8) -> "Dataset":
        cols = arr if isinstance(arr, dict) else {"data": np.asarray(arr)}
        n = len(next(iter(cols.values())))
        bounds = np.linspace(0, n, max(1, min(parallelism, n)) + 1).astype(int)
        return Dataset([{k: v[bounds[i]:bounds[i + 1]] for k, v in cols.items()} for i in range(len(bounds) - 1)])

    @staticmethod
    def from_pandas(df, parallelism: int = 8) -> "Dataset":
        return Dataset.from_numpy({c: df[c].to_numpy() for c in df.columns}, parallelism)

    @staticmethod
    def read_text(paths, parallelism: int = 8, encoding: str = "utf-8") -> "Dataset":
        paths = [paths] if isinstance(paths, str) else list(paths)
        rows = []
        for p in paths:
            with open(p, encoding=encoding) as f:
                rows.extend({"text": line.rstrip("\n")} for line in f)
        return Dataset.from_items(rows, parallelism)

    # ------------------------------------------------------------------ transforms (lazy)
    def _with(self, op) -> "Dataset":
        return Dataset(self._blocks, self._ops + [op])

    def map(self, fn: Callable) -> "Dataset":
        return self._with(("map", fn, {}))

    def flat_map(self, fn: Callable) -> "Dataset":
        return self._with(("flat_map", fn, {}))

    def filter(self, fn: Callable) -> "Dataset":
        return self._with(("filter", fn, {}))

    def map_batches(self, fn: Callable, batch_size: Optional[int] = None, batch_format: str = "numpy",
                    fn_kwargs: Optional[dict] = None, **_) -> "Dataset":
        if isinstance(fn, type):
            fn = fn()
        return self._with(("map_batches", fn, {"batch_size": batch_size, "batch_format": batch_format,
                                               "fn_kwargs": fn_kwargs or {}}))

    def select_columns(self, cols: List[str]) -> "Dataset":
        return self._with(("select", list(cols), {}))

    def random_shuffle(self, seed: Optional[int] = None) -> "Dataset":
        ds = self.materialize()
        allb = _concat(ds._blocks)
        rng = np.random.default_rng(seed)
        perm = rng.permutation(_block_len(allb))
        allb = {k: v[perm] for k, v in allb.items()}
        return Dataset._from_block(allb, max(1, len(self._blocks)))

    def shuffle(self, seed=None):
        return self.random_shuffle(seed)

    def limit(self, n: int) -> "Dataset":
        b = _concat(self.materialize()._blocks)
        return Dataset._from_block(_slice(b, 0, n), max(1, len(self._blocks)))

    def select(self, indices) -> "Dataset":
        b = _concat(self.materialize()._blocks)
        idx = np.asarray(list(indices), dtype=np.int64)
        return Dataset._from_block({k: v[idx] for k, v in b.items()}, max(1, len(self._blocks)))

    def repartition(self, n: int) -> "Dataset":
        return Dataset._from_block(_concat(self.materialize()._blocks), n)

    @staticmethod
    def _from_block(b: Block, k: int) -> "Dataset":
        n = _block_len(b)
        bounds = np.linspace(0, n, max(1, min(k, max(n, 1))) + 1).astype(int)
        return Dataset([_slice(b, bounds[i], bounds[i + 1]) for i in range(len(bounds) - 1)])

    # ------------------------------------------------------------------ execution
    def materialize(self) -> "Dataset":
        if not self._ops:
            return self
        from .. import runtime as rt
        if rt.is_initialized() and len(self._blocks) > 1 and os.environ.get("GRT_DATA_INLINE", "0") != "1":
            task = rt.remote(_run_block).options(num_cpus=1)
            refs = [task.remote(b, self._ops) for b in self._blocks]
            blocks = rt.get(refs)
        else:
            blocks = [_apply_ops(b, self._ops) for b in self._blocks]
        return Dataset(blocks)

    def _stream_blocks(self, ahead: int = 2) -> Iterator[Block]:
        """Streaming executor: transforms run on a producer thread `ahead` blocks in front."""
        if not self._ops:
            yield from self._blocks
            return
        q: "queue.Queue" = queue.Queue(maxsize=ahead)

        def prod():
            for b in self._blocks:
                q.put(_apply_ops(b, self._ops))
            q.put(None)
        threading.Thread(target=prod, daemon=True).start()
        while True:
            b = q.get()
            if b is None:
                return
            yield b

    def count(self) -> int:
        return sum(_block_len(b) for b in self.materialize()._blocks)

    def __len__(self):
        return self.count()

    def take(self, n: int = 20) -> List[Dict[str, Any]]:
        out = []
        for b in self._stream_blocks():
            for r in _block_rows(b):
                out.append(r)
                if len(out) >= n:
                    return out
        return out

    def take_all(self):
        return [r for b in self._stream_blocks() for r in _block_rows(b)]

    def columns(self):
        for b in self._stream_blocks():
            return list(b.keys())
        return []

    def schema(self):
        for b in self._stream_blocks():
            return {k: v.dtype for k, v in b.items()}
        return {}

    def to_pandas(self):
        import pandas as pd
        b = _concat(self.materialize()._blocks)
        return pd.DataFrame({k: list(v) if v.ndim > 1 else v for k, v in b.items()})

    def train_test_split(self, test_size: float, shuffle: bool = False, seed=None):
        ds = self.random_shuffle(seed) if shuffle else self.materialize()
        b = _concat(ds._blocks)
        n = _block_len(b)
        k = int(round(n * (1 - test_size))) if test_size < 1 else n - int(test_size)
        return Dataset._from_block(_slice(b, 0, k), len(self._blocks)), Dataset._from_block(_slice(b, k, n), len(self._blocks))

    # ------------------------------------------------------------------ sharding
    def split(self, n: int, equal: bool = True) -> List["Dataset"]:
        b = _concat(self.materialize()._blocks)
        tot = _block_len(b)
        per = tot // n if equal else -(-tot // n)
        return [Dataset._from_block(_slice(b, i * per, min(tot, (i + 1) * per)), 1) for i in range(n)]

    def streaming_split(self, n: int, equal: bool = True) -> List["DataIterator"]:
        return [DataIterator(self, i, n, equal) for i in range(n)]

    def shard_for_rank(self, rank: int, world: int) -> "DataIterator":
        return DataIterator(self, rank, world, True)

    # ------------------------------------------------------------------ iteration
    def iter_rows(self):
        for b in self._stream_blocks():
            yield from _block_rows(b)

    def iter_batches(self, batch_size: int = 256, batch_format: str = "numpy", drop_last: bool = False,
                     local_shuffle_buffer_size: Optional[int] = None, local_shuffle_seed=None, prefetch_batches: int = 1):
        return _batches(self._stream_blocks(), batch_size, batch_format, drop_last, local_shuffle_buffer_size,
                        local_shuffle_seed)

    def iter_torch_batches(self, batch_size: int = 256, dtypes=None, device="auto", collate_fn=None,
                           drop_last: bool = False, prefetch_batches: int = 1, **kw):
        return _torch_batches(self.iter_batches(batch_size, drop_last=drop_last, **kw), dtypes, device, collate_fn)


class DataIterator:
    """Per-rank shard of a dataset: rank r takes every world-th row block-by-block (streaming)."""

    def __init__(self, ds: Dataset, rank: int, world: int, equal: bool = True):
        self.ds, self.rank, self.world, self.equal = ds, rank, world, equal

    def _blocks(self):
        for b in self.ds._stream_blocks():
            n = _block_len(b)
            idx = np.arange(self.rank, n, self.world)
            if self.equal:
                idx = idx[: n // self.world]
            yield {k: v[idx] for k, v in b.items()}

    def iter_rows(self):
        for b in self._blocks():
            yield from _block_rows(b)

    def iter_batches(self, batch_size: int = 256, batch_format: str = "numpy", drop_last: bool = False,
                     local_shuffle_buffer_size=None, local_shuffle_seed=None, **_):
        return _batches(self._blocks(), batch_size, batch_format, drop_last, local_shuffle_buffer_size,
                        local_shuffle_seed)

    def iter_torch_batches(self, batch_size: int = 256, dtypes=None, device="auto", collate_fn=None,
                           drop_last: bool = False, producer_process: bool = False, **kw):
        """``producer_process=True`` runs the shard's read -> map -> batch pipeline in a separate
        process that streams fixed-schema numeric batches through the native shared-memory ring
        (runtime/shm_ring.py), keeping host-side data work off the training process."""
        if producer_process:
            batches = _process_batches(lambda: self.iter_batches(batch_size, drop_last=drop_last, **kw), batch_size)
        else:
            batches = self.iter_batches(batch_size, drop_last=drop_last, **kw)
        return _torch_batches(batches, dtypes, device, collate_fn)


def _process_batches(factory, batch_size: int):
    """Batches of ``factory()`` produced in another process through an ShmRing (numeric fields
    with fixed trailing shapes); falls back to in-process iteration otherwise."""
    from ..runtime.shm_ring import RingBatchStream
    probe = next(iter(factory()), None)
    if probe is None:
        return iter(())
    if any(v.dtype == object for v in probe.values()):
        return factory()
    schema = {k: (v.dtype.str, (max(batch_size, v.shape[0]),) + tuple(v.shape[1:])) for k, v in probe.items()}
    return iter(RingBatchStream(factory, schema))


def _batches(blocks: Iterable[Block], batch_size, batch_format, drop_last, shuffle_buf=None, seed=None):
    rng = np.random.default_rng(seed) if shuffle_buf else None
    buf: List[Block] = []
    have = 0
    for b in blocks:
        if rng is not None:
            perm = rng.permutation(_block_len(b))
            b = {k: v[perm] for k, v in b.items()}
        buf.append(b)
        have += _block_len(b)
        while have >= batch_size:
            allb = _concat(buf)
            yield _fmt(_slice(allb, 0, batch_size), batch_format)
            rest = _slice(allb, batch_size, have)
            buf = [rest]
            have -= batch_size
    if have and not drop_last:
        yield _fmt(_concat(buf), batch_format)


def _fmt(b: Block, fmt: str):
    if fmt == "pandas":
        import pandas as pd
        return pd.DataFrame({k: list(v) if v.ndim > 1 else v for k, v in b.items()})
    return b


def _torch_batches(batches, dtypes, device, collate_fn):
    import torch
    if device == "auto":
        from ..train.torch import get_device
        device = get_device()
    device = torch.device(device) if device is not None else None
    for b in batches:
        if collate_fn is not None:
            yield collate_fn(b)
            continue
        out = {}
        for k, v in b.items():
            if v.dtype == object:
                out[k] = v
                continue
            t = torch.from_numpy(np.ascontiguousarray(v))
            if dtypes is not None:
                dt = dtypes.get(k) if isinstance(dtypes, dict) else dtypes
                if dt is not None:
                    t = t.to(dt)
            if device is not None and device.type == "cuda":
                t = t.pin_memory().to(device, non_blocking=True)
            elif device is not None:
                t = t.to(device)
            out[k] = t
        yield out


# module-level constructors (ray.data.from_items / range / read_text ...)
from_items = Dataset.from_items
range_ = Dataset.range
from_numpy = Dataset.from_numpy
from_pandas = Dataset.from_pandas
read_text = Dataset.read_text
