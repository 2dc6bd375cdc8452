"""A streaming, block-parallel dataset (the Ray Data surface used for the data pipeline).

``BASELINE.json`` asks for the Wikitext-2 preparation (reference
ray-jobs/prepare_wikitext2_ray_job.py:18,56-71,106-109) to become a Ray-Data pipeline that shards
and streams token batches into HBM (config #4). Semantics follow Ray Data where the reference
ecosystem uses it: lazy transforms (``map``, ``map_batches``, ``filter``, ``flat_map``,
``random_shuffle``), ``streaming_split(n)`` for per-rank shards (``train.get_dataset_shard``), and
``iter_batches`` / ``iter_torch_batches`` consumption.

Execution model on one MI355X node:
* data is a list of columnar blocks (``dict[str, np.ndarray]``); a plan is the source blocks plus
  stages: per-block transforms and windowed shuffles. ``_stream`` executes it lazily — a bounded
  thread pool runs the per-block transforms a few blocks ahead of the consumer (numpy releases
  the GIL), so memory stays O(window) instead of O(dataset);
* ``random_shuffle(seed)`` is a STREAMING shuffle: the source block order is permuted up front
  (free), then rows are mixed across a sliding window of ``window_blocks`` transformed blocks.
  ``random_shuffle(seed, window_blocks=0)`` keeps the exact full shuffle (materialises);
* ``streaming_split(n)`` runs ONE executor for the dataset in a coordinator process and DEALS rows
  to the n consumers (``equal=True``: every split gets exactly the same row count, the < n
  leftover rows of an epoch are dropped) — no consumer re-executes the pipeline. Splits are
  picklable handles (address + authkey) usable from any process of the node, so TorchTrainer
  hands one to each worker; ``streaming_split_for_rank`` does the same for a torch.distributed
  job (rank 0 hosts the coordinator, the address is broadcast);
* ``iter_torch_batches`` assembles batches on a background thread, stages them in a ring of
  pinned host buffers and issues the H2D copies on a dedicated HIP stream, ``prefetch_batches``
  ahead of the training loop; the compute stream waits on the copy's event and the batch tensors
  are recorded on it (no allocator reuse while the step still reads them).
"""
from __future__ import annotations

import collections
import os
import queue
import secrets
import threading
import traceback
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Callable, Dict, Iterable, Iterator, List, Optional

import numpy as np

Block = Dict[str, np.ndarray]
_SHUFFLE_WINDOW = int(os.environ.get("GRT_SHUFFLE_WINDOW_BLOCKS", "4"))


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
    if len(blocks) == 1:
        return blocks[0]
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
        elif kind == "select":
            block = {k: block[k] for k in fn}
    return block


def _run_block(block, ops):
    return _apply_ops(block, ops)


class Dataset:
    """Source blocks + a lazy plan: ``("ops", [op...])`` per-block transform stages and
    ``("shuffle", seed, window_blocks)`` streaming-shuffle stages."""

    def __init__(self, blocks: List[Block], ops=None, stages=None):
        self._blocks = blocks
        stages = list(stages or [])
        if ops:
            stages.append(("ops", list(ops)))
        self._stages = stages

    # back-compat view: the per-block ops of a plan without shuffle stages
    @property
    def _ops(self):
        return [op for st in self._stages if st[0] == "ops" for op in st[1]]

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
        st = [(s[0], list(s[1])) if s[0] == "ops" else s for s in self._stages]
        if st and st[-1][0] == "ops":
            st[-1][1].append(op)
        else:
            st.append(("ops", [op]))
        return Dataset(self._blocks, stages=st)

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

    def random_shuffle(self, seed: Optional[int] = None, window_blocks: Optional[int] = None) -> "Dataset":
        """Streaming shuffle: permuted block order + row mixing across ``window_blocks`` blocks
        (default ``GRT_SHUFFLE_WINDOW_BLOCKS`` = 4). ``window_blocks=0``: exact full shuffle."""
        w = _SHUFFLE_WINDOW if window_blocks is None else int(window_blocks)
        if w <= 0:
            ds = self.materialize()
            allb = _concat(ds._blocks)
            rng = np.random.default_rng(seed)
            perm = rng.permutation(_block_len(allb))
            allb = {k: v[perm] for k, v in allb.items()}
            return Dataset._from_block(allb, max(1, len(self._blocks)))
        if seed is None:
            seed = int(np.random.SeedSequence().entropy % (1 << 63))
        return Dataset(self._blocks, stages=self._stages + [("shuffle", int(seed), w)])

    def shuffle(self, seed=None):
        return self.random_shuffle(seed)

    def randomize_block_order(self, seed: Optional[int] = None) -> "Dataset":
        return self.random_shuffle(seed, window_blocks=1)

    def limit(self, n: int) -> "Dataset":
        out, have = [], 0
        for b in self._stream():
            k = min(_block_len(b), n - have)
            if k > 0:
                out.append(_slice(b, 0, k))
                have += k
            if have >= n:
                break
        return Dataset._from_block(_concat(out), max(1, len(self._blocks)))

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
        if not self._stages:
            return self
        if len(self._stages) == 1 and self._stages[0][0] == "ops":
            from .. import runtime as rt
            ops = self._stages[0][1]
            if rt.is_initialized() and len(self._blocks) > 1 and os.environ.get("GRT_DATA_INLINE", "0") != "1":
                task = rt.remote(_run_block).options(num_cpus=1)
                return Dataset(rt.get([task.remote(b, ops) for b in self._blocks]))
        return Dataset(list(self._stream()))

    def _source_order(self) -> List[int]:
        order = list(range(len(self._blocks)))
        sh = next((s for s in self._stages if s[0] == "shuffle"), None)
        if sh is not None:  # the block order permutation is free: blocks are independent until the shuffle
            order = [int(i) for i in np.random.default_rng(sh[1]).permutation(len(order))]
        return order

    def _stream(self, ahead: int = 2, source: Optional[List[int]] = None) -> Iterator[Block]:
        """Streaming executor over ``source`` block indices (default: all, shuffle order)."""
        src = self._source_order() if source is None else source
        it: Iterator[Block] = (self._blocks[i] for i in src)
        for st in self._stages:
            if st[0] == "ops":
                it = _map_ahead(it, st[1], ahead)
            else:
                it = _window_shuffle(it, st[1], st[2])
        return it

    # back-compat name
    def _stream_blocks(self, ahead: int = 2) -> Iterator[Block]:
        return self._stream(ahead)

    def count(self) -> int:
        if not self._stages:
            return sum(_block_len(b) for b in self._blocks)
        return sum(_block_len(b) for b in self._stream())

    def __len__(self):
        return self.count()

    def num_blocks(self) -> int:
        return len(self._blocks)

    def take(self, n: int = 20) -> List[Dict[str, Any]]:
        out = []
        for b in self._stream():
            for r in _block_rows(b):
                out.append(r)
                if len(out) >= n:
                    return out
        return out

    def take_all(self):
        return [r for b in self._stream() for r in _block_rows(b)]

    def columns(self):
        for b in self._stream():
            return list(b.keys())
        return []

    def schema(self):
        for b in self._stream():
            return {k: v.dtype for k, v in b.items()}
        return {}

    def to_pandas(self):
        import pandas as pd
        b = _concat(list(self._stream()))
        return pd.DataFrame({k: list(v) if v.ndim > 1 else v for k, v in b.items()})

    def train_test_split(self, test_size: float, shuffle: bool = False, seed=None):
        ds = self.random_shuffle(seed, window_blocks=0) if shuffle else self.materialize()
        b = _concat(ds._blocks)
        n = _block_len(b)
        k = int(round(n * (1 - test_size))) if test_size < 1 else n - int(test_size)
        return Dataset._from_block(_slice(b, 0, k), len(self._blocks)), Dataset._from_block(_slice(b, k, n), len(self._blocks))

    # ------------------------------------------------------------------ sharding
    def split(self, n: int, equal: bool = True) -> List["Dataset"]:
        b = _concat(list(self._stream()))
        tot = _block_len(b)
        per = tot // n if equal else -(-tot // n)
        return [Dataset._from_block(_slice(b, i * per, min(tot, (i + 1) * per)), 1) for i in range(n)]

    def streaming_split(self, n: int, equal: bool = True, locality_hints=None) -> List["StreamSplit"]:
        """n coordinated consumers of ONE execution of this dataset (see module doc)."""
        coord = SplitCoordinator.start(self, n, equal)
        splits = [StreamSplit(coord.address, coord.authkey, i, n) for i in range(n)]
        for sp in splits:
            sp._coordinator = coord  # creator-side handle (not pickled): shutdown() ends the process
        return splits

    def streaming_split_for_rank(self, rank: int, world: int, group=None, equal: bool = True) -> "StreamSplit":
        """torch.distributed job: rank 0 starts the coordinator, every rank gets its split."""
        import torch.distributed as dist
        obj = [None]
        if rank == 0:
            coord = SplitCoordinator.start(self, world, equal)
            obj = [(coord.address, coord.authkey)]
            self._coordinator = coord  # keep alive with the dataset
        if world > 1 and dist.is_available() and dist.is_initialized():
            dist.broadcast_object_list(obj, src=0, group=group)
        addr, key = obj[0]
        return StreamSplit(addr, key, rank, world)

    def shard_for_rank(self, rank: int, world: int, equal: bool = True) -> "DataIterator":
        """Static per-rank shard without a coordinator.

        ``equal=True`` (what ``train.get_dataset_shard`` uses): every rank gets exactly
        floor(rows / world) rows — rank r takes row r of every complete round of ``world`` rows of
        the one execution order — so data-parallel ranks run the same number of steps (unequal
        counts would hang DDP collectives) whatever the block sizes or length-changing transforms.
        Each rank executes the whole pipeline for that. ``equal=False``: rank r executes only source
        blocks r, r + world, ... (1/world of the work); counts can differ. ``streaming_split`` gives
        exact balance with one execution."""
        return DataIterator(self, rank, world, equal)

    # ------------------------------------------------------------------ iteration
    def iter_rows(self):
        for b in self._stream():
            yield from _block_rows(b)

    def iter_batches(self, batch_size: int = 256, batch_format: str = "numpy", drop_last: bool = False,
                     local_shuffle_buffer_size: Optional[int] = None, local_shuffle_seed=None, prefetch_batches: int = 1):
        return _prefetch(_batches(self._stream(), batch_size, batch_format, drop_last, local_shuffle_buffer_size,
                                  local_shuffle_seed), prefetch_batches)

    def iter_torch_batches(self, batch_size: int = 256, dtypes=None, device="auto", collate_fn=None,
                           drop_last: bool = False, prefetch_batches: int = 2, **kw):
        return _torch_batches(_batches(self._stream(), batch_size, "numpy", drop_last,
                                       kw.get("local_shuffle_buffer_size"), kw.get("local_shuffle_seed")),
                              dtypes, device, collate_fn, prefetch_batches)


def _map_ahead(blocks: Iterator[Block], ops, ahead: int) -> Iterator[Block]:
    """Ordered per-block transforms on a small thread pool, ``ahead`` blocks in flight."""
    workers = max(1, min(int(os.environ.get("GRT_DATA_THREADS", "4")), ahead + 1))
    ex = ThreadPoolExecutor(max_workers=workers, thread_name_prefix="grt-data")
    try:
        pending = collections.deque()
        for b in blocks:
            pending.append(ex.submit(_apply_ops, b, ops))
            if len(pending) > ahead:
                yield pending.popleft().result()
        while pending:
            yield pending.popleft().result()
    finally:
        ex.shutdown(wait=False, cancel_futures=True)


def _window_shuffle(blocks: Iterator[Block], seed: int, window: int) -> Iterator[Block]:
    """Mix rows across ``window`` consecutive blocks; each window is re-cut into its block sizes."""
    rng = np.random.default_rng(seed + 0x9E3779B9)
    buf: List[Block] = []

    def flush():
        sizes = [_block_len(b) for b in buf]
        allb = _concat(buf)
        perm = rng.permutation(_block_len(allb))
        allb = {k: v[perm] for k, v in allb.items()}
        off = 0
        for s in sizes:
            yield _slice(allb, off, off + s)
            off += s

    for b in blocks:
        if not _block_len(b):
            continue
        buf.append(b)
        if len(buf) >= window:
            yield from flush()
            buf = []
    if buf:
        yield from flush()


class DataIterator:
    """Static per-rank shard (``Dataset.shard_for_rank``): equal row rounds, or source blocks
    rank::world when ``equal`` is False."""

    def __init__(self, ds: Dataset, rank: int, world: int, equal: bool = True):
        self.ds, self.rank, self.world, self.equal = ds, rank, world, equal

    def _blocks(self):
        if not self.equal or self.world == 1:
            order = self.ds._source_order()
            yield from self.ds._stream(source=order[self.rank::self.world])
            return
        carry: Block = {}
        for b in self.ds._stream():
            cur = _concat([carry, b]) if _block_len(carry) else b
            n = _block_len(cur)
            full = n // self.world * self.world
            if full:
                yield {k: v[self.rank:full:self.world] for k, v in cur.items()}
            carry = _slice(cur, full, n)
        # the incomplete last round is dropped on every rank

    def iter_rows(self):
        for b in self._blocks():
            yield from _block_rows(b)

    def iter_batches(self, batch_size: int = 256, batch_format: str = "numpy", drop_last: bool = False,
                     local_shuffle_buffer_size=None, local_shuffle_seed=None, prefetch_batches: int = 1, **_):
        return _prefetch(_batches(self._blocks(), batch_size, batch_format, drop_last, local_shuffle_buffer_size,
                                  local_shuffle_seed), prefetch_batches)

    def iter_torch_batches(self, batch_size: int = 256, dtypes=None, device="auto", collate_fn=None,
                           drop_last: bool = False, producer_process: bool = False, prefetch_batches: int = 2, **kw):
        """``producer_process=True`` runs the shard's read -> map -> batch pipeline in a separate
        process that streams fixed-schema numeric batches through the native shared-memory ring
        (runtime/shm_ring.py), keeping host-side data work off the training process."""
        if producer_process:
            batches = _process_batches(lambda: self.iter_batches(batch_size, drop_last=drop_last, **kw), batch_size)
        else:
            batches = _batches(self._blocks(), batch_size, "numpy", drop_last, kw.get("local_shuffle_buffer_size"),
                               kw.get("local_shuffle_seed"))
        return _torch_batches(batches, dtypes, device, collate_fn, prefetch_batches)


# ====================================================================== coordinated split
def _coordinator_main(payload: bytes, n: int, equal: bool, authkey: bytes, conn_back, parent: int):
    import time

    import cloudpickle
    from multiprocessing.connection import Listener

    def watchdog():  # the coordinator lives exactly as long as the process that created the split
        while os.getppid() == parent:
            time.sleep(1.0)
        os._exit(0)
    threading.Thread(target=watchdog, daemon=True, name="grt-split-watchdog").start()
    ds = cloudpickle.loads(payload)
    listener = Listener(("127.0.0.1", 0), authkey=authkey, backlog=128)  # many consumers connect at once
    conn_back.send(listener.address)
    conn_back.close()
    _CoordinatorState(ds, n, equal).serve(listener)


class _CoordinatorState:
    """One streaming execution per epoch; rows dealt evenly to the n splits as they arrive."""

    def __init__(self, ds: Dataset, n: int, equal: bool):
        self.ds, self.n, self.equal = ds, n, equal
        self.cv = threading.Condition()
        self.epoch = -1
        self.finished = [True] * n              # split i received the end of the current epoch
        self.abandoned = [False] * n            # split i stopped consuming the current epoch early
        self.queues = [collections.deque() for _ in range(n)]
        self.qbytes = [0] * n
        self.done = True
        self.error: Optional[str] = None
        self.cap = int(float(os.environ.get("GRT_SPLIT_BUFFER_MB", "512")) * 2 ** 20)
        self.stats = {"blocks_executed": 0, "rows_dealt": [0] * n, "epochs": 0}

    def _start_epoch(self):
        self.epoch += 1
        self.stats["epochs"] += 1
        self.finished = [False] * self.n
        self.abandoned = [False] * self.n
        self.queues = [collections.deque() for _ in range(self.n)]
        self.qbytes = [0] * self.n
        self.done = False
        threading.Thread(target=self._produce, daemon=True, name="grt-split-exec").start()

    def _deal(self, parts: List[Block]):
        with self.cv:
            while any(q > self.cap for q in self.qbytes) and not self.error:
                self.cv.wait(0.5)  # backpressure: a slow consumer's queue is full
            for i, p in enumerate(parts):
                if _block_len(p) and not self.abandoned[i]:
                    self.queues[i].append(p)
                    self.qbytes[i] += sum(v.nbytes for v in p.values())
                    self.stats["rows_dealt"][i] += _block_len(p)
            self.cv.notify_all()

    def _produce(self):
        n = self.n
        try:
            rem: Block = {}
            for b in self.ds._stream():
                self.stats["blocks_executed"] += 1
                cur = _concat([rem, b]) if _block_len(rem) else b
                tot = _block_len(cur)
                per = tot // n
                if per == 0:
                    rem = cur
                    continue
                self._deal([_slice(cur, i * per, (i + 1) * per) for i in range(n)])
                rem = _slice(cur, n * per, tot)
            if _block_len(rem) and not self.equal:  # unequal split: the leftover rows go to the first splits
                self._deal([_slice(rem, i, i + 1) if i < _block_len(rem) else {} for i in range(n)])
        except BaseException:
            with self.cv:
                self.error = traceback.format_exc()
        with self.cv:
            self.done = True
            self.cv.notify_all()

    def _next(self, i: int, epoch: int):
        with self.cv:
            if epoch == self.epoch + 1:
                # every split must finish epoch e before e + 1 starts (another split's request may
                # start it while this one waits)
                while epoch == self.epoch + 1 and not all(self.finished):
                    self.cv.wait(0.5)
                if epoch == self.epoch + 1:
                    self._start_epoch()
            elif epoch != self.epoch:
                return ("error", f"split {i} asked for epoch {epoch}, coordinator is at {self.epoch}")
            while True:
                if self.error:
                    return ("error", self.error)
                if self.abandoned[i]:
                    return ("end", None)
                if self.queues[i]:
                    b = self.queues[i].popleft()
                    self.qbytes[i] -= sum(v.nbytes for v in b.values())
                    self.cv.notify_all()
                    return ("block", b)
                if self.done:
                    self.finished[i] = True
                    self.cv.notify_all()
                    return ("end", None)
                self.cv.wait(0.5)

    def _abandon(self, i: int, epoch: int):
        """Split i stopped iterating epoch ``epoch``: drop its queue, count it as finished."""
        with self.cv:
            if epoch != self.epoch or self.finished[i]:
                return
            self.abandoned[i] = True
            self.finished[i] = True
            self.queues[i].clear()
            self.qbytes[i] = 0
            self.cv.notify_all()

    def _client(self, conn):
        from ..runtime import object_store
        try:
            while True:
                msg = conn.recv()
                if msg[0] == "next":
                    kind, val = self._next(msg[1], msg[2])
                    conn.send_bytes(object_store.pack((kind, val)))
                elif msg[0] == "abandon":
                    self._abandon(msg[1], msg[2])
                    conn.send_bytes(object_store.pack(("ok", None)))
                elif msg[0] == "stats":
                    conn.send_bytes(object_store.pack(("stats", dict(self.stats, epoch=self.epoch))))
                elif msg[0] == "close":
                    return
        except (EOFError, OSError):
            return
        except BaseException:  # keep the coordinator alive; the client sees its connection close
            import sys
            print(f"[grt] streaming_split coordinator: client handler failed\n{traceback.format_exc()}",
                  file=sys.stderr, flush=True)

    def serve(self, listener):
        while True:
            try:
                conn = listener.accept()
            except OSError:
                return
            threading.Thread(target=self._client, args=(conn,), daemon=True).start()


class SplitCoordinator:
    """Handle to a coordinator process (started by the split's creator, dies with it)."""

    def __init__(self, proc, address, authkey):
        self.proc, self.address, self.authkey = proc, address, authkey

    @staticmethod
    def start(ds: Dataset, n: int, equal: bool) -> "SplitCoordinator":
        import multiprocessing as mp

        import cloudpickle
        ctx = mp.get_context("spawn")
        key = secrets.token_bytes(16)
        a, b = ctx.Pipe(duplex=False)
        p = ctx.Process(target=_coordinator_main, args=(cloudpickle.dumps(ds), n, equal, key, b, os.getpid()),
                        daemon=True, name="grt-split-coordinator")
        p.start()
        b.close()
        if not a.poll(120):
            p.kill()
            raise RuntimeError("streaming_split coordinator did not start")
        coord = SplitCoordinator(p, a.recv(), key)
        import atexit
        atexit.register(coord.shutdown)
        return coord

    def shutdown(self):
        if self.proc.is_alive():
            self.proc.kill()
            self.proc.join(5)


class StreamSplit:
    """One consumer of a coordinated ``streaming_split`` (Ray's ``DataIterator``). Picklable:
    only the coordinator address travels; each process opens its own connection. Every
    ``iter_*`` call consumes one epoch; all splits must consume epoch e before e + 1 starts."""

    def __init__(self, address, authkey: bytes, index: int, n: int):
        self.address, self.authkey, self.index, self.n = address, authkey, index, n
        self._conn = None
        self._epoch = -1
        self._coordinator: Optional[SplitCoordinator] = None

    def shutdown(self):
        """Stop the coordinator (creator process only; consumers just drop their handle)."""
        if self._coordinator is not None:
            self._coordinator.shutdown()

    def __getstate__(self):
        return {"address": self.address, "authkey": self.authkey, "index": self.index, "n": self.n}

    def __setstate__(self, st):
        self.__dict__.update(st)
        self._conn = None
        self._epoch = -1
        self._coordinator = None

    def _connect(self):
        from multiprocessing.connection import Client
        return Client(tuple(self.address), authkey=self.authkey)

    def _call(self, msg):
        """Control requests (stats, abandon) on this handle's own connection; the per-epoch block
        stream uses a separate connection, so the two never interleave."""
        from ..runtime import object_store
        if self._conn is None:
            self._conn = self._connect()
        self._conn.send(msg)
        return object_store.unpack(self._conn.recv_bytes())

    def stats(self) -> Dict[str, Any]:
        return self._call(("stats",))[1]

    def _blocks(self, ahead: int = 2) -> Iterator[Block]:
        """One epoch. A consumer may stop early (break on max_steps): closing this generator stops
        the pull thread and tells the coordinator the split abandoned the epoch, so epoch e + 1 can
        start for every split (Ray starts the next epoch the same way, on the remaining requests)."""
        from ..runtime import object_store
        self._epoch += 1
        epoch = self._epoch
        q: "queue.Queue" = queue.Queue(maxsize=max(1, ahead))
        stop = threading.Event()

        def put(item) -> bool:
            while not stop.is_set():
                try:
                    q.put(item, timeout=0.2)
                    return True
                except queue.Full:
                    continue
            return False

        def pull():  # overlap the next request's round trip with the consumer's work
            conn = None
            try:
                conn = self._connect()
                while not stop.is_set():
                    conn.send(("next", self.index, epoch))
                    kind, val = object_store.unpack(conn.recv_bytes())
                    if not put((kind, val)) or kind != "block":
                        return
            except BaseException:
                if not stop.is_set():
                    put(("error", traceback.format_exc()))
            finally:
                if conn is not None:
                    try:
                        conn.send(("close",))
                        conn.close()
                    except OSError:
                        pass
        threading.Thread(target=pull, daemon=True, name="grt-split-pull").start()
        ended = False
        try:
            while True:
                kind, val = q.get()
                if kind == "block":
                    yield val
                elif kind == "end":
                    ended = True
                    return
                else:
                    ended = True
                    raise RuntimeError(f"streaming_split coordinator failed:\n{val}")
        finally:
            stop.set()
            if not ended:
                try:
                    self._call(("abandon", self.index, epoch))
                except (OSError, EOFError):
                    pass

    def iter_rows(self):
        for b in self._blocks():
            yield from _block_rows(b)

    def iter_batches(self, batch_size: int = 256, batch_format: str = "numpy", drop_last: bool = False,
                     local_shuffle_buffer_size=None, local_shuffle_seed=None, prefetch_batches: int = 1, **_):
        return _prefetch(_batches(self._blocks(), batch_size, batch_format, drop_last, local_shuffle_buffer_size,
                                  local_shuffle_seed), prefetch_batches)

    def iter_torch_batches(self, batch_size: int = 256, dtypes=None, device="auto", collate_fn=None,
                           drop_last: bool = False, prefetch_batches: int = 2, **kw):
        return _torch_batches(_batches(self._blocks(), batch_size, "numpy", drop_last,
                                       kw.get("local_shuffle_buffer_size"), kw.get("local_shuffle_seed")),
                              dtypes, device, collate_fn, prefetch_batches)


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
        if have < batch_size:
            continue
        allb = _concat(buf)
        s = 0
        while have - s >= batch_size:
            yield _fmt(_slice(allb, s, s + batch_size), batch_format)
            s += batch_size
        buf = [_slice(allb, s, have)]
        have -= s
    if have and not drop_last:
        yield _fmt(_concat(buf), batch_format)


def _fmt(b: Block, fmt: str):
    if fmt == "pandas":
        import pandas as pd
        return pd.DataFrame({k: list(v) if v.ndim > 1 else v for k, v in b.items()})
    return b


class _Handoff:
    """Bounded producer -> consumer queue of a background thread. When the consumer stops early
    (its generator is closed), ``stop`` is set and the producer's ``put`` gives up instead of
    blocking forever; the producer then closes its own source so upstream stages (a streaming
    split's pull thread, the coordinator's epoch) are released too."""

    def __init__(self, depth: int):
        self.q: "queue.Queue" = queue.Queue(maxsize=max(1, depth))
        self.stop = threading.Event()

    def put(self, item) -> bool:
        while not self.stop.is_set():
            try:
                self.q.put(item, timeout=0.2)
                return True
            except queue.Full:
                continue
        return False

    def close_source(self, it):
        if self.stop.is_set() and hasattr(it, "close"):
            try:
                it.close()
            except BaseException:  # noqa: BLE001 - best effort on an abandoned source
                pass


def _prefetch(it: Iterator, depth: int) -> Iterator:
    """Run ``it`` on a background thread ``depth`` items ahead (``prefetch_batches``)."""
    if depth <= 0:
        yield from it
        return
    h = _Handoff(depth)
    end = object()

    def run():
        try:
            for x in it:
                if not h.put((True, x)):
                    break
            else:
                h.put((True, end))
        except BaseException as e:  # noqa: BLE001 - re-raised in the consumer
            h.put((False, e))
        finally:
            h.close_source(it)
    threading.Thread(target=run, daemon=True, name="grt-prefetch").start()
    try:
        while True:
            ok, x = h.q.get()
            if not ok:
                raise x
            if x is end:
                return
            yield x
    finally:
        h.stop.set()


_NP_OF_TORCH = None


def _np_dtype(dt):
    global _NP_OF_TORCH
    import torch
    if _NP_OF_TORCH is None:
        _NP_OF_TORCH = {torch.int64: np.int64, torch.int32: np.int32, torch.float32: np.float32,
                        torch.float64: np.float64, torch.int16: np.int16, torch.uint8: np.uint8, torch.bool: np.bool_}
    return _NP_OF_TORCH.get(dt)


def _torch_batches(batches, dtypes, device, collate_fn, prefetch_batches: int = 2):
    import torch
    if device == "auto":
        from ..train.torch import get_device
        device = get_device()
    device = torch.device(device) if device is not None else None
    if collate_fn is not None:
        for b in _prefetch(batches, prefetch_batches):
            yield collate_fn(b)
        return

    def cast(k, v):
        dt = dtypes.get(k) if isinstance(dtypes, dict) else dtypes
        return dt

    if device is None or device.type != "cuda":
        for b in _prefetch(batches, prefetch_batches):
            out = {}
            for k, v in b.items():
                if v.dtype == object:
                    out[k] = v
                    continue
                t = torch.from_numpy(np.ascontiguousarray(v))
                dt = cast(k, v)
                if dt is not None:
                    t = t.to(dt)
                out[k] = t.to(device) if device is not None else t
            yield out
        return
    yield from _PinnedH2D(device, max(1, prefetch_batches)).run(batches, cast)


class _PinnedH2D:
    """Batches -> pinned host ring slot -> async H2D on a copy stream, ``depth`` batches ahead
    of the consumer, all issued from a background thread."""

    def __init__(self, device, depth: int):
        self.device, self.depth = device, depth

    def run(self, batches, cast):
        import torch
        dev = self.device
        copy = torch.cuda.Stream(dev)
        nslot = self.depth + 1
        slots: List[Dict[str, torch.Tensor]] = [dict() for _ in range(nslot)]
        done: List[Optional[torch.cuda.Event]] = [None] * nslot
        h = _Handoff(self.depth)
        end = object()

        def produce():
            try:
                torch.cuda.set_device(dev)
                for i, b in enumerate(batches):
                    s = i % nslot
                    if done[s] is not None:
                        done[s].synchronize()  # the slot's previous H2D has drained
                    out = {}
                    for k, v in b.items():
                        if v.dtype == object:
                            out[k] = v
                            continue
                        dt = cast(k, v)
                        npd = _np_dtype(dt) if dt is not None else None
                        a = np.ascontiguousarray(v, dtype=npd) if npd is not None else np.ascontiguousarray(v)
                        if a.size:
                            buf = slots[s].get(k)
                            if buf is None or buf.numel() < a.nbytes:
                                buf = torch.empty(a.nbytes, dtype=torch.uint8, pin_memory=True)
                                slots[s][k] = buf
                            tdt = torch.from_numpy(a.reshape(-1)[:0]).dtype
                            host = buf[:a.nbytes].view(tdt).view(a.shape)  # pinned storage
                            host.numpy()[...] = a
                        else:
                            host = torch.from_numpy(a)
                        with torch.cuda.stream(copy):
                            t = host.to(dev, non_blocking=True)
                            if dt is not None and npd is None:
                                t = t.to(dt)
                        out[k] = t
                    ev = torch.cuda.Event()
                    ev.record(copy)
                    done[s] = ev
                    if not h.put((True, (out, ev))):
                        break
                else:
                    h.put((True, end))
            except BaseException as e:  # noqa: BLE001
                h.put((False, e))
            finally:
                h.close_source(batches)

        threading.Thread(target=produce, daemon=True, name="grt-h2d").start()
        try:
            while True:
                ok, item = h.q.get()
                if not ok:
                    raise item
                if item is end:
                    return
                out, ev = item
                cur = torch.cuda.current_stream(dev)
                cur.wait_event(ev)
                for t in out.values():
                    if isinstance(t, torch.Tensor) and t.is_cuda:
                        t.record_stream(cur)
                yield out
        finally:
            h.stop.set()


# module-level constructors (ray.data.from_items / range / read_text ...)
from_items = Dataset.from_items
range_ = Dataset.range
from_numpy = Dataset.from_numpy
from_pandas = Dataset.from_pandas
read_text = Dataset.read_text
