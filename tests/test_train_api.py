"""Ray-Train-compatible API on CPU/gloo: report barrier, checkpoint layout + retention, result
files, worker failure propagation, FailureConfig restart from checkpoint (fault injection)."""
import json
import os
import tempfile

import pytest
import torch

from gke_ray_train_amd import runtime as rt
from gke_ray_train_amd import train
from gke_ray_train_amd.train import (Checkpoint, CheckpointConfig, FailureConfig, RunConfig, ScalingConfig,
                                     TorchTrainer, TrainingFailedError)
from gke_ray_train_amd.train.torch import TorchConfig


@pytest.fixture(scope="module", autouse=True)
def _runtime():
    rt.init(num_cpus=4, num_gpus=0, ignore_reinit_error=True)
    yield
    rt.shutdown()


def loop(config):
    import torch.distributed as dist
    ctx = train.get_context()
    rank, world = ctx.get_world_rank(), ctx.get_world_size()
    assert world == config["world"] and dist.get_world_size() == world
    start = 0
    ck = train.get_checkpoint()
    if ck is not None:
        with open(os.path.join(ck.path, "state.json")) as f:
            start = json.load(f)["epoch"] + 1
    t = torch.ones(1) * (rank + 1)
    dist.all_reduce(t)
    assert t.item() == world * (world + 1) / 2
    for epoch in range(start, config["epochs"]):
        loss = config["losses"][epoch]
        with tempfile.TemporaryDirectory() as d:
            ckpt = None
            if rank == 0:
                with open(os.path.join(d, "state.json"), "w") as f:
                    json.dump({"epoch": epoch}, f)
                ckpt = Checkpoint.from_directory(d)
            train.report({"loss": loss, "epoch": epoch + 1}, checkpoint=ckpt)


def test_fit_layout_and_retention(tmp_path):
    cfg = {"world": 2, "epochs": 4, "losses": [3.0, 1.0, 2.0, 2.5]}
    trainer = TorchTrainer(loop, train_loop_config=cfg, scaling_config=ScalingConfig(num_workers=2, use_gpu=False),
                           run_config=RunConfig(name="exp1", storage_path=str(tmp_path),
                                                checkpoint_config=CheckpointConfig(num_to_keep=1,
                                                                                   checkpoint_score_attribute="loss",
                                                                                   checkpoint_score_order="min")),
                           torch_config=TorchConfig(backend="gloo"))
    res = trainer.fit()
    assert res.error is None
    assert res.metrics["loss"] == 2.5 and res.metrics["training_iteration"] == 4
    trial = res.path
    assert os.path.dirname(trial) == str(tmp_path / "exp1")
    assert os.path.basename(trial).startswith("TorchTrainer_")
    for f in ("params.json", "result.json", "progress.csv"):
        assert os.path.exists(os.path.join(trial, f)), f
    rows = [json.loads(l) for l in open(os.path.join(trial, "result.json"))]
    assert [r["loss"] for r in rows] == cfg["losses"] and rows[-1]["done"] is True
    ckpts = sorted(d for d in os.listdir(trial) if d.startswith("checkpoint_"))
    # best (loss 1.0 -> checkpoint_000001) kept + the latest (checkpoint_000003)
    assert ckpts == ["checkpoint_000001", "checkpoint_000003"], ckpts
    assert res.get_best_checkpoint("loss", "min").path.endswith("checkpoint_000001")
    df = res.metrics_dataframe
    assert list(df["epoch"]) == [1, 2, 3, 4]


def bad_loop(config):
    if train.get_context().get_world_rank() == 1:
        raise ValueError("rank 1 exploded")
    train.report({"x": 1})


def test_worker_error_fails_fit(tmp_path):
    trainer = TorchTrainer(bad_loop, scaling_config=ScalingConfig(num_workers=2),
                           run_config=RunConfig(storage_path=str(tmp_path)))
    with pytest.raises(TrainingFailedError) as ei:
        trainer.fit()
    assert "exploded" in str(ei.value.__cause__)


def test_fault_injection_restart_from_checkpoint(tmp_path, monkeypatch):
    monkeypatch.setenv("GRT_FAULT_INJECT", "1:2")  # rank 1 dies at its 3rd report on attempt 0
    cfg = {"world": 2, "epochs": 4, "losses": [4.0, 3.0, 2.0, 1.0]}
    trainer = TorchTrainer(loop, train_loop_config=cfg, scaling_config=ScalingConfig(num_workers=2),
                           run_config=RunConfig(name="ft", storage_path=str(tmp_path),
                                                failure_config=FailureConfig(max_failures=1)))
    res = trainer.fit()
    rows = [json.loads(l) for l in open(os.path.join(res.path, "result.json"))]
    # epochs 1,2 before the crash; restart resumes at epoch 3 from checkpoint_000001
    assert [r["epoch"] for r in rows] == [1, 2, 3, 4]
    assert res.metrics["loss"] == 1.0


def test_no_failures_allowed_raises(tmp_path, monkeypatch):
    monkeypatch.setenv("GRT_FAULT_INJECT", "0:0")
    cfg = {"world": 2, "epochs": 2, "losses": [1.0, 0.5]}
    trainer = TorchTrainer(loop, train_loop_config=cfg, scaling_config=ScalingConfig(num_workers=2),
                           run_config=RunConfig(storage_path=str(tmp_path)))
    with pytest.raises(TrainingFailedError):
        trainer.fit()
