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
