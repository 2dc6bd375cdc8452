"""BASELINE.json config #1: the BasicLLM job (pytorch_llm_ray.py path) as DDP on the local runtime with
num_workers=2, CPU/gloo, synthetic Wikitext-2 — plus the data-prep job."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jobs"))


@pytest.fixture(autouse=True)
def _rt():
    from gke_ray_train_amd import runtime as rt
    rt.init(num_cpus=4, num_gpus=0, ignore_reinit_error=True)
    yield
    rt.shutdown()


def test_prepare_wikitext2_job(tmp_path):
    import prepare_wikitext2_ray_job as job
    rc = job.main(["--target", str(tmp_path / "raw"), "--scale", "0.002"])
    assert rc == 0
    assert sorted(os.listdir(tmp_path / "raw")) == ["wiki.test.tokens", "wiki.train.tokens", "wiki.valid.tokens"]


def test_basic_llm_job_two_cpu_workers(tmp_path):
    import pytorch_llm_ray as job
    res = job.main(["--cpu", "--workers", "2", "--preset", "tiny", "--batch", "4", "--seq", "32",
                    "--data-scale", "0.004", "--pvc", str(tmp_path), "--epochs", "2",
                    "--max-windows", "256"])
    proc = tmp_path / "datasets" / "wikitext-2-processed"
    assert {"train.ids.pt", "char_vocab.json", "vocab_size.txt", "_DATA_PREP_DONE"} <= set(os.listdir(proc))
    assert res.metrics["epoch"] == 2 and res.metrics["loss"] > 0
    trial = res.path
    assert trial.startswith(str(tmp_path / "ray_llm_training_runs" / "wikitext2_manualTB_v1"))
    ck = [d for d in os.listdir(trial) if d.startswith("checkpoint_")]
    assert 1 <= len(ck) <= 2
    latest = res.checkpoint.path
    assert sorted(os.listdir(latest)) == ["model.pth", "optimizer.pth", "scheduler.pth"]
    import torch
    sd = torch.load(os.path.join(latest, "model.pth"), weights_only=True)
    assert "token_embedding.weight" in sd and "transformer_decoder.layers.0.self_attn.in_proj_weight" in sd
    assert "positional_encoding.pe" in sd and "fc_out.bias" in sd
    # the resume path loads optimizer / scheduler state with the no-code-execution loader
    assert "state" in torch.load(os.path.join(latest, "optimizer.pth"), weights_only=True)
    assert "last_epoch" in torch.load(os.path.join(latest, "scheduler.pth"), weights_only=True)
    rows = [json.loads(l) for l in open(os.path.join(trial, "result.json"))]
    assert [r["epoch"] for r in rows] == [1, 2]
    assert rows[1]["loss"] < rows[0]["loss"] + 1.0


def test_data_prep_sentinel_is_atomic_and_tracks_the_raw_text(tmp_path):
    """The sentinel records digests of the raw text and every product: a changed raw file, a legacy
    "done" sentinel or a tampered product redoes the preparation (the reference trusts any sentinel,
    ray-jobs/pytorch_llm_ray.py:160,176)."""
    import torch
    import pytorch_llm_ray as job
    raw = tmp_path / "raw.txt"
    raw.write_text("hello world\n" * 50)
    cfg = {"processed_data_dir": str(tmp_path / "proc"), "raw_data_path": str(raw)}
    ids, vocab = job._prepare_char_data(cfg, 0)
    done = tmp_path / "proc" / "_DATA_PREP_DONE"
    rec = json.loads(done.read_text())
    assert rec["raw_sha256"] == job._file_digest(str(raw)) and set(rec["products"]) == {
        "train.ids.pt", "char_vocab.json", "vocab_size.txt"}
    assert not [f for f in os.listdir(tmp_path / "proc") if ".tmp" in f]
    mtime = os.path.getmtime(tmp_path / "proc" / "train.ids.pt")
    job._prepare_char_data(cfg, 0)  # unchanged: reused
    assert os.path.getmtime(tmp_path / "proc" / "train.ids.pt") == mtime
    raw.write_text("different text, new characters: XYZ\n" * 40)  # changed raw text: redone
    ids2, vocab2 = job._prepare_char_data(cfg, 0)
    assert vocab2 != vocab and len(ids2) == len(raw.read_text())
    done.write_text("done")  # legacy / torn sentinel: redone, not trusted
    job._prepare_char_data(cfg, 0)
    assert json.loads(done.read_text())["raw_sha256"] == job._file_digest(str(raw))
    torch.save(torch.zeros(3, dtype=torch.int64), tmp_path / "proc" / "train.ids.pt")  # tampered product
    ids3, _ = job._prepare_char_data(cfg, 0)
    assert len(ids3) == len(raw.read_text())


def test_eight_bit_optimizers_refuse_loudly():
    """paged_adamw_8bit / adamw_8bit are a different algorithm (block-quantized states): refused with
    a message instead of silently running 32-bit AdamW."""
    import torch
    from gke_ray_train_amd.ops import make_optimizer
    p = [torch.nn.Parameter(torch.zeros(4))]
    for name in ("paged_adamw_8bit", "adamw_8bit"):
        with pytest.raises(ValueError, match="8-bit"):
            make_optimizer(name, p, lr=1e-3, weight_decay=0.0)
    assert make_optimizer("paged_adamw_32bit", p, lr=1e-3, weight_decay=0.0) is not None
