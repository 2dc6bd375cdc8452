"""``prepare_trainer``: validates the trainer's distributed view against the Train session and
attaches the report callback once (trainer/callbacks.py)."""
import pytest


class _T:
    def __init__(self, rank, world, callbacks=()):
        self.rank, self.world, self.callbacks = rank, world, list(callbacks)


@pytest.fixture
def session(monkeypatch):
    from gke_ray_train_amd.train import _session as s
    saved = s._SESSION

    def make(rank, world):
        s._set_session(s._Session(s.TrainContext(world_rank=rank, world_size=world, local_rank=rank,
                                                 local_world_size=world)))
    yield make
    s._set_session(saved)


def test_attaches_report_callback_once(session):
    from gke_ray_train_amd.trainer import RayTrainReportCallback, prepare_trainer
    session(1, 4)
    t = _T(1, 4)
    assert prepare_trainer(t) is t
    assert sum(isinstance(c, RayTrainReportCallback) for c in t.callbacks) == 1
    prepare_trainer(t)
    assert sum(isinstance(c, RayTrainReportCallback) for c in t.callbacks) == 1
    own = RayTrainReportCallback()
    t2 = _T(1, 4, [own])
    prepare_trainer(t2)
    assert t2.callbacks == [own]


def test_rejects_trainer_built_outside_the_process_group(session):
    from gke_ray_train_amd.trainer import prepare_trainer
    session(2, 4)
    with pytest.raises(RuntimeError, match="rank 0 of 1"):
        prepare_trainer(_T(0, 1))
