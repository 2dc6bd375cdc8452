"""Trainer callbacks bridging the SFT trainer to the Ray-Train-compatible session.

Reference: ``RayTrainReportCallback`` / ``prepare_trainer`` are imported by the SFT job but never
used (ray-jobs/fine_tune_llama_ray.py:8), so its ``result.metrics`` are empty. Here they work:
attach ``RayTrainReportCallback()`` to have every log and checkpoint of the trainer reported through
``train.report`` (one report per save, with the checkpoint directory).
"""
from __future__ import annotations


class RayTrainReportCallback:
    def __init__(self):
        self._last = {}

    def on_log(self, trainer, logs):
        self._last.update({k: v for k, v in logs.items() if isinstance(v, (int, float))})

    def on_save(self, trainer, ckpt_dir):
        from ..train import Checkpoint, report
        report(dict(self._last), checkpoint=Checkpoint.from_directory(ckpt_dir) if trainer.rank == 0 else None)

    def on_train_end(self, trainer, metrics):
        from ..train import report
        report(dict(self._last, **metrics))


def prepare_trainer(trainer):
    """Ray's prepare_trainer validates the HF Trainer for Ray; the SFT trainer is already
    distributed-aware, so this is the identity."""
    return trainer
