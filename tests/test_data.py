"""Data layer: char tokenizer (reference semantics), TextDataset, synthetic Wikitext-2 files, native
window gather, sharded prefetching loader, Ray-Data-like pipeline."""
import json
import os

import numpy as np
import pytest
import torch

from gke_ray_train_amd import data
from gke_ray_train_amd.data import wikitext


def test_char_tokenizer_roundtrip(tmp_path):
    tok = data.CharTokenizer()
    text = "hello wörld = = Test = =\n"
    tok.fit_on_text(text)
    assert tok.vocab_size == len(set(text))
    ids = tok.encode(text)
    assert tok.decode(ids) == text
    assert tok.encode("Z") == [-1]  # reference: unknown -> -1
    assert tok.encode("Z", unk=0) == [0]
    assert np.array_equal(tok.encode_np(text + "Z"), np.array(tok.encode(text + "Z")))
    p = tmp_path / "v" / "char_vocab.json"
    tok.save_vocab(str(p))
    d = json.load(open(p))
    assert set(d) == {"char_to_idx", "idx_to_char", "vocab_size"}
    t2 = data.CharTokenizer(str(p))
    assert t2.decode(ids) == text and t2.vocab_size == tok.vocab_size


def test_text_dataset():
    ids = torch.arange(100)
    ds = data.TextDataset(ids, 10)
    assert len(ds) == 100 - 10 - 1
    x, y = ds[5]
    assert torch.equal(x, torch.arange(5, 15)) and torch.equal(y, torch.arange(6, 16))


def test_wikitext_synthetic_idempotent(tmp_path):
    paths = wikitext.prepare(str(tmp_path), scale=0.01)
    assert set(paths) == {"train", "validation", "test"}
    sizes = {k: os.path.getsize(p) for k, p in paths.items()}
    assert all(s > 0 for s in sizes.values())
    txt = open(paths["train"], encoding="utf-8").read()
    assert " = " in txt and "\n" in txt
    mt = os.path.getmtime(paths["train"])
    wikitext.prepare(str(tmp_path), scale=0.01)  # second call skips
    assert os.path.getmtime(paths["train"]) == mt
    tok = data.CharTokenizer()
    tok.fit_on_text(txt)
    assert 40 < tok.vocab_size < 400


def test_gather_windows_native():
    toks = np.arange(1000, dtype=np.int32) * 3
    starts = np.array([0, 5, 900], dtype=np.int64)
    x, y = data.gather_windows(toks, starts, 16)
    for i, s in enumerate(starts):
        assert np.array_equal(x[i], toks[s:s + 16]) and np.array_equal(y[i], toks[s + 1:s + 17])
    with pytest.raises(IndexError):
        data.gather_windows(toks, np.array([990]), 16)


def test_token_loader_sharding():
    toks = np.arange(5000, dtype=np.int64)
    seen = []
    for r in range(2):
        ld = data.TokenBatchLoader(toks, 32, 8, rank=r, world=2, shuffle=True, seed=3, max_windows=1600)
        got = [x for x, y in ld]
        assert len(got) == len(ld) == 1600 // 2 // 8
        for x, y in ld:
            assert torch.equal(y[:, :-1], x[:, 1:])
        seen.append(torch.cat(got)[:, 0])
    a, b = set(seen[0].tolist()), set(seen[1].tolist())
    assert not (a & b) and len(a | b) == 1600


def test_pipeline_ops():
    ds = data.range(100, parallelism=4).map(lambda r: {"x": r["id"] * 2}).filter(lambda r: r["x"] % 4 == 0)
    assert ds.count() == 50
    ds2 = ds.map_batches(lambda b: {"x": b["x"] + 1, "y": b["x"]}, batch_size=7)
    rows = ds2.take_all()
    assert rows[0]["x"] == 1 and rows[0]["y"] == 0
    its = ds2.streaming_split(2)
    parts = [sum(len(b["x"]) for b in it.iter_batches(batch_size=5)) for it in its]
    assert sum(parts) <= 50 and abs(parts[0] - parts[1]) <= 1
    tb = next(iter(ds2.iter_torch_batches(batch_size=10, device="cpu")))
    assert isinstance(tb["x"], torch.Tensor) and tb["x"].shape == (10,)
    tr, te = ds2.train_test_split(0.2)
    assert tr.count() == 40 and te.count() == 10
    assert len(ds2.split(3)) == 3


def test_streaming_split_producer_process_matches_in_process():
    """iter_torch_batches(producer_process=True): the shard's batches come from a producer process
    through the native shared-memory ring and equal the in-process iteration."""
    import numpy as np
    from gke_ray_train_amd.data.pipeline import Dataset
    ds = Dataset.from_numpy(np.arange(4000, dtype=np.int64).reshape(1000, 4)).map_batches(
        lambda b: {"x": b["data"] * 2, "y": b["data"].sum(1)})
    it = ds.shard_for_rank(1, 2)
    a = list(it.iter_torch_batches(batch_size=64, device="cpu"))
    b = list(it.iter_torch_batches(batch_size=64, device="cpu", producer_process=True))
    assert len(a) == len(b) > 3
    for u, v in zip(a, b):
        assert (u["x"] == v["x"]).all() and (u["y"] == v["y"]).all()
