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
    """Ready an SFT trainer to run as one worker of a Train job (Ray's ``prepare_trainer`` role).

    * Checks that the trainer's distributed view (rank / world it sharded data and optimizer
      state for) matches the Train session's context. A trainer built before the process group
      was initialised would otherwise train as world 1 on every rank, silently replicating the
      job N times; that raises here instead.
    * Attaches a ``RayTrainReportCallback`` when none is attached, so every checkpoint and the
      final metrics reach ``train.report`` and ``result.metrics`` / ``result.checkpoint`` are
      filled (the reference imports both names and uses neither, so its result is empty:
      ray-jobs/fine_tune_llama_ray.py:8).

    Returns the same trainer object.
    """
    from ..train import get_context
    ctx = get_context()
    want = (ctx.get_world_rank(), ctx.get_world_size())
    have = (getattr(trainer, "rank", 0), getattr(trainer, "world", 1))
    if have != want:
        raise RuntimeError(f"trainer was built for rank {have[0]} of {have[1]} but this Train worker is "
                           f"rank {want[0]} of {want[1]}; construct the trainer inside the training "
                           f"function, after the process group is initialised")
    cbs = getattr(trainer, "callbacks", None)
    if cbs is not None and not any(isinstance(cb, RayTrainReportCallback) for cb in cbs):
        cbs.append(RayTrainReportCallback())
    return trainer
