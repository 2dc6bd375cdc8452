"""Worker-side training session: context, ``report`` (a barrier across ranks), checkpoints.

Reference semantics: ``train.report(metrics, checkpoint)`` must be called the same
number of times on every rank (ray-jobs/pytorch_llm_ray.py:309-310); only rank 0's metrics are
recorded; checkpoints are persisted by the driver under ``checkpoint_%06d``. Here each report
goes over a local socket to the driver, which acknowledges only after EVERY rank has sent that
report index — the call is a barrier, as in Ray.
"""
from __future__ import annotations

import os
import shutil
import tempfile
import time
from dataclasses import dataclass
from multiprocessing.connection import Client
from typing import Any, Dict, Optional

from ._checkpoint import Checkpoint


@dataclass
class TrainContext:
    world_rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    node_rank: int = 0
    trial_name: str = "local"
    trial_id: str = "00000"
    experiment_name: str = "local"
    trial_dir: str = ""
    storage_path: str = ""

    def get_world_rank(self):
        return self.world_rank

    def get_world_size(self):
        return self.world_size

    def get_local_rank(self):
        return self.local_rank

    def get_local_world_size(self):
        return self.local_world_size

    def get_node_rank(self):
        return self.node_rank

    def get_trial_name(self):
        return self.trial_name

    def get_trial_id(self):
        return self.trial_id

    def get_experiment_name(self):
        return self.experiment_name

    def get_trial_dir(self):
        return self.trial_dir

    def get_storage(self):
        return self.storage_path


class _Session:
    def __init__(self, ctx: TrainContext, address=None, authkey=None, checkpoint: Optional[Checkpoint] = None,
                 datasets: Optional[Dict[str, Any]] = None, reports_done: int = 0):
        self.ctx = ctx
        self.conn = Client(address, authkey=authkey) if address else None
        if self.conn is not None:
            self.conn.send(("hello", ctx.world_rank))
        self.checkpoint = checkpoint
        self.datasets = datasets or {}
        self.index = reports_done
        self.last_metrics: Optional[dict] = None
        self.local_reports = []

    def report(self, metrics: Dict[str, Any], checkpoint: Optional[Checkpoint] = None):
        _maybe_inject_fault(self.ctx.world_rank, self.index)
        # a report is a synchronisation point of every rank: a failed xGMI IPC collective since the
        # last one raises here (fail-stop, like an NCCL error) instead of being reported as a result
        from ..parallel.ipc import check_all
        check_all()
        staged = None
        if checkpoint is not None:
            # stage the files: the caller may delete its (temporary) directory right after report()
            staged = tempfile.mkdtemp(prefix=f"grt_report_r{self.ctx.world_rank}_")
            shutil.copytree(checkpoint.path, staged, dirs_exist_ok=True)
        metrics = {k: _plain(v) for k, v in dict(metrics).items()}
        self.last_metrics = metrics
        if self.conn is None:
            self.local_reports.append((metrics, staged))
            self.index += 1
            return
        self.conn.send(("report", self.ctx.world_rank, self.index, metrics, staged, time.time()))
        msg = self.conn.recv()  # barrier: released when all ranks reported this index
        if msg[0] != "ack":
            raise RuntimeError(f"unexpected driver reply {msg!r}")
        self.index += 1
        if msg[1] is not None:
            self.checkpoint = Checkpoint(msg[1])

    def close(self, ok=True, err=None):
        if self.conn is not None:
            try:
                self.conn.send(("done", self.ctx.world_rank, ok, err))
                self.conn.close()
            except Exception:
                pass


def _maybe_inject_fault(rank: int, index: int):
    """Fault injection for tests: GRT_FAULT_INJECT="<rank>:<report index>[:<attempt>]" makes that
    rank's process die (os._exit) when it reaches that report, on that restart attempt (default 0)."""
    spec = os.environ.get("GRT_FAULT_INJECT")
    if not spec:
        return
    parts = [int(x) for x in spec.split(":")]
    r, i = parts[0], parts[1]
    att = parts[2] if len(parts) > 2 else 0
    if rank == r and index == i and int(os.environ.get("GRT_ATTEMPT", "0")) == att:
        os._exit(17)


def _plain(v):
    try:
        import torch
        if isinstance(v, torch.Tensor):
            return v.item() if v.numel() == 1 else v.tolist()
    except Exception:
        pass
    try:
        import numpy as np
        if isinstance(v, np.generic):
            return v.item()
    except Exception:
        pass
    return v


_SESSION: Optional[_Session] = None


def _set_session(s: Optional[_Session]):
    global _SESSION
    _SESSION = s


def _get_session() -> _Session:
    global _SESSION
    if _SESSION is None:  # outside a TorchTrainer: behave as a single local worker
        rank = int(os.environ.get("RANK", 0))
        ws = int(os.environ.get("WORLD_SIZE", 1))
        lr = int(os.environ.get("LOCAL_RANK", 0))
        _SESSION = _Session(TrainContext(world_rank=rank, world_size=ws, local_rank=lr,
                                         local_world_size=int(os.environ.get("LOCAL_WORLD_SIZE", ws))))
    return _SESSION


def get_context() -> TrainContext:
    return _get_session().ctx


def report(metrics: Dict[str, Any], checkpoint: Optional[Checkpoint] = None, checkpoint_dir_name=None):
    _get_session().report(metrics, checkpoint)


def get_checkpoint() -> Optional[Checkpoint]:
    return _get_session().checkpoint


def get_dataset_shard(name: str = "train"):
    s = _get_session()
    ds = s.datasets.get(name)
    if ds is None:
        return None
    if hasattr(ds, "shard_for_rank"):  # a Dataset handed over directly (TorchTrainer passes splits)
        return ds.shard_for_rank(s.ctx.world_rank, s.ctx.world_size)
    return ds  # this rank's StreamSplit of the driver's streaming_split
