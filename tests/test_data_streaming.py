"""Ray-Data streaming semantics: one coordinated execution per streaming_split
(no per-consumer re-execution), exactly equal splits, windowed (non-materialising) shuffle,
epoch barrier, picklable split handles used from other processes, TorchTrainer datasets."""
import multiprocessing as mp
import pickle

import numpy as np
import pytest

from gke_ray_train_amd.data.pipeline import Dataset


def _ids(ds_rows):
    return sorted(int(r) for r in ds_rows)


def test_windowed_shuffle_is_a_lazy_permutation():
    ds = Dataset.from_numpy({"x": np.arange(1000)}, parallelism=20)
    sh = ds.random_shuffle(seed=5)
    assert sh._stages[-1][0] == "shuffle"          # lazy: nothing executed yet
    a = [int(r["x"]) for r in sh.iter_rows()]
    b = [int(r["x"]) for r in ds.random_shuffle(seed=5).iter_rows()]
    c = [int(r["x"]) for r in ds.random_shuffle(seed=6).iter_rows()]
    assert sorted(a) == list(range(1000)) and a == b and a != c
    assert a != sorted(a)
    # rows move across block boundaries (window mixing), not only the block order
    first_block = set(a[:50])
    assert len({v // 50 for v in first_block}) > 1
    exact = [int(r["x"]) for r in ds.random_shuffle(seed=5, window_blocks=0).iter_rows()]
    assert sorted(exact) == list(range(1000))


def _consume(split, out_q, epochs):
    got = []
    for _ in range(epochs):
        got.append([int(v) for b in split.iter_batches(batch_size=7) for v in b["x"]])
    out_q.put((split.index, got))


def test_streaming_split_one_execution_equal_rows_across_processes():
    calls = mp.get_context("spawn").Value("i", 0)  # noqa: F841  (the count is read from the coordinator)
    ds = Dataset.from_numpy({"x": np.arange(1003)}, parallelism=16).map_batches(lambda b: {"x": b["x"] * 1})
    splits = ds.streaming_split(3, equal=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_consume, args=(pickle.loads(pickle.dumps(s)), q, 2)) for s in splits]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    for ep in range(2):
        parts = [res[i][ep] for i in range(3)]
        assert len(parts[0]) == len(parts[1]) == len(parts[2]) == 1003 // 3
        allv = [v for p in parts for v in p]
        assert len(set(allv)) == len(allv)           # disjoint
        assert set(allv) <= set(range(1003)) and len(allv) == 1002
    st = splits[0].stats()
    assert st["epochs"] == 2 and st["blocks_executed"] == 2 * 16  # each block ran once per epoch
    splits[0].shutdown()


def test_streaming_split_unequal_keeps_every_row():
    ds = Dataset.from_numpy({"x": np.arange(101)}, parallelism=4)
    splits = ds.streaming_split(2, equal=False)
    # sequential consumption in one process works: the coordinator buffers the other split
    a = [int(v) for b in splits[0].iter_batches(batch_size=10) for v in b["x"]]
    b = [int(v) for b in splits[1].iter_batches(batch_size=10) for v in b["x"]]
    assert sorted(a + b) == list(range(101)) and abs(len(a) - len(b)) <= 1
    splits[0].shutdown()


def test_shard_for_rank_partitions_rows():
    seen = []
    ds = Dataset.from_numpy({"x": np.arange(80)}, parallelism=8).map_batches(lambda b: {"x": b["x"]})
    parts = [[int(v) for b in ds.shard_for_rank(r, 2).iter_batches(batch_size=5) for v in b["x"]] for r in range(2)]
    assert sorted(parts[0] + parts[1]) == list(range(80)) and len(parts[0]) == len(parts[1]) == 40
    del seen


def test_prefetch_batches_and_torch_batches_cpu():
    import torch
    ds = Dataset.from_numpy({"x": np.arange(64, dtype=np.int32)}, parallelism=4)
    got = list(ds.iter_torch_batches(batch_size=16, device="cpu", dtypes={"x": torch.int64}, prefetch_batches=3))
    assert len(got) == 4 and got[0]["x"].dtype == torch.int64
    assert torch.cat([g["x"] for g in got]).tolist() == list(range(64))


def _loop(config):
    from gke_ray_train_amd import train
    shard = train.get_dataset_shard("train")
    n = sum(len(b["x"]) for b in shard.iter_batches(batch_size=8))
    train.report({"rows": n, "kind": type(shard).__name__})


def test_torch_trainer_hands_each_worker_a_coordinated_split(tmp_path):
    from gke_ray_train_amd import runtime as rt
    from gke_ray_train_amd.train import RunConfig, ScalingConfig, TorchTrainer
    ds = Dataset.from_numpy({"x": np.arange(240)}, parallelism=6)
    try:
        res = TorchTrainer(_loop, scaling_config=ScalingConfig(num_workers=2, use_gpu=False),
                           run_config=RunConfig(name="ds", storage_path=str(tmp_path), verbose=0),
                           datasets={"train": ds}).fit()
    finally:
        rt.shutdown()
    assert res.metrics["rows"] == 120 and res.metrics["kind"] == "StreamSplit"


def test_streaming_split_consumer_breaks_early_then_next_epoch_runs():
    """A split that stops iterating an epoch early (max_steps) must not wedge the coordinator:
    the next epoch starts for every split and carries all rows again."""
    import threading
    ds = Dataset.from_numpy({"x": np.arange(400)}, parallelism=8)
    splits = ds.streaming_split(2)
    try:
        got = {}

        def consume(i, limit):
            n = 0
            for b in splits[i].iter_batches(batch_size=10):
                n += len(b["x"])
                if limit and n >= limit:
                    break  # early exit in epoch 0
            got[(i, 0)] = n
            got[(i, 1)] = sorted(int(v) for b in splits[i].iter_batches(batch_size=10) for v in b["x"])

        ts = [threading.Thread(target=consume, args=(0, 30)), threading.Thread(target=consume, args=(1, 0))]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
        assert not any(t.is_alive() for t in ts), "epoch 1 never started after an early break"
        assert got[(0, 0)] == 30 and got[(1, 0)] == 200
        assert len(got[(0, 1)]) == len(got[(1, 1)]) == 200
        assert sorted(got[(0, 1)] + got[(1, 1)]) == list(range(400))
    finally:
        splits[0].shutdown()


def test_shard_for_rank_equal_counts_with_uneven_blocks_and_filters():
    """equal=True gives every rank the same row count even when blocks are uneven and a filter
    changes lengths (unequal counts hang DDP collectives)."""
    ds = Dataset.from_numpy({"x": np.arange(103)}, parallelism=5).filter(lambda r: r["x"] % 7 != 0)
    parts = [[int(v) for b in ds.shard_for_rank(r, 3).iter_batches(batch_size=4) for v in b["x"]] for r in range(3)]
    kept = [v for v in range(103) if v % 7 != 0]
    assert len(parts[0]) == len(parts[1]) == len(parts[2]) == len(kept) // 3
    assert sorted(parts[0] + parts[1] + parts[2]) == kept[: len(kept) // 3 * 3]
    # equal=False: block-level shards (cheap), counts may differ
    blk = [[int(v) for b in ds.shard_for_rank(r, 3, equal=False).iter_batches(batch_size=4) for v in b["x"]]
           for r in range(3)]
    assert sorted(blk[0] + blk[1] + blk[2]) == kept
