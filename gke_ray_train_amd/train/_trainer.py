"""TorchTrainer: launch one worker actor per GPU, rendezvous torch.distributed, run
``train_loop_per_worker(config)``, collect reports / checkpoints, restart on failure.

Reference: ``TorchTrainer(train_loop_per_worker, train_loop_config, scaling_config, run_config,
torch_config).fit() -> Result`` (ray-jobs/pytorch_llm_ray.py:368-376,
fine_tune_llama_ray.py:451-457). MI355X single-node mapping:
* one worker actor per GPU on this node; rank r gets GPU r (``LOCAL_RANK = r``) while every GPU
  stays visible, so RCCL can open xGMI peer paths between all 8 ranks;
* rendezvous is torch's env:// TCPStore on 127.0.0.1 with the backend from ``TorchConfig``
  (``"nccl"`` is RCCL on ROCm; gloo for CPU workers), 1800 s timeout like Ray;
* a worker exception or a dead worker fails the attempt; with ``FailureConfig(max_failures=k)``
  the whole group restarts from the latest persisted checkpoint (``train.get_checkpoint()``),
  otherwise ``fit()`` raises ``TrainingFailedError`` (Ray's default, max_failures=0).
"""
from __future__ import annotations

import inspect
import os
import secrets
import socket
import time
import traceback
from multiprocessing.connection import Listener, wait as conn_wait
from typing import Any, Callable, Dict, Optional

import cloudpickle

from .. import runtime as rt
from ..runtime.errors import RayTaskError, TrainingFailedError
from ._checkpoint import Checkpoint
from ._config import FailureConfig, RunConfig, ScalingConfig
from ._result import Result
from ._session import TrainContext, _Session, _set_session
from ._storage import RunStorage


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class TrainWorker:
    """Actor body: one per rank."""

    def __init__(self):
        self.pid = os.getpid()

    def gpu(self):
        v = os.environ.get("GRT_ASSIGNED_GPU")
        return int(v.split(",")[0]) if v else -1

    def run(self, fn_payload, config, rank, world, local_rank, local_world, master_addr, master_port, backend,
            timeout_s, ctx_fields, address, authkey, ckpt_path, datasets, reports_done, attempt, use_gpu):
        import datetime
        import torch
        import torch.distributed as dist
        os.environ.update({
            "RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(local_rank),
            "LOCAL_WORLD_SIZE": str(local_world), "NODE_RANK": "0", "GROUP_RANK": "0",
            "MASTER_ADDR": master_addr, "MASTER_PORT": str(master_port), "GRT_ATTEMPT": str(attempt),
        })
        if use_gpu:
            torch.cuda.set_device(local_rank)
        kw = {}
        if backend == "nccl" and use_gpu:
            kw["device_id"] = torch.device("cuda", local_rank)
        dist.init_process_group(backend, init_method="env://", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
        ctx = TrainContext(**ctx_fields, world_rank=rank, world_size=world, local_rank=local_rank,
                           local_world_size=local_world)
        sess = _Session(ctx, address=address, authkey=authkey, checkpoint=Checkpoint(ckpt_path) if ckpt_path else None,
                        datasets=datasets, reports_done=reports_done)
        _set_session(sess)
        fn = cloudpickle.loads(fn_payload)
        ok, err = True, None
        try:
            if len(inspect.signature(fn).parameters) == 0:
                fn()
            else:
                fn(config if config is not None else {})
        except BaseException:
            ok, err = False, traceback.format_exc()
            raise
        finally:
            sess.close(ok, err)
            _set_session(None)
            try:
                if dist.is_initialized():
                    if ok:
                        dist.barrier()
                    dist.destroy_process_group()
            except Exception:
                pass
        return {"rank": rank, "reports": sess.index}


class DataParallelTrainer:
    _name = "DataParallelTrainer"

    def __init__(self, train_loop_per_worker: Callable, *, train_loop_config: Optional[Dict[str, Any]] = None,
                 scaling_config: Optional[ScalingConfig] = None, run_config: Optional[RunConfig] = None,
                 backend_config=None, datasets: Optional[Dict[str, Any]] = None, resume_from_checkpoint=None,
                 metadata=None, dataset_config=None):
        self.fn = train_loop_per_worker
        self.config = train_loop_config
        self.scaling = scaling_config or ScalingConfig()
        self.run_config = run_config or RunConfig()
        self.backend_config = backend_config
        self.datasets = datasets or {}
        self.resume_from_checkpoint = resume_from_checkpoint
        self.metadata = metadata or {}

    def _backend(self):
        b = getattr(self.backend_config, "backend", None)
        if b is None:
            import torch
            b = "nccl" if (self.scaling.use_gpu and torch.cuda.device_count() > 0) else "gloo"
        return b

    def fit(self) -> Result:
        storage = RunStorage(self.run_config, self._name, self.config)
        fc = self.run_config.failure_config or FailureConfig()
        failures = 0
        ckpt = self.resume_from_checkpoint
        err = None
        while True:
            try:
                self._run_attempt(storage, ckpt, failures)
                err = None
                break
            except Exception as e:  # noqa: BLE001
                err = e
                failures += 1
                if fc.max_failures != -1 and failures > fc.max_failures:
                    break
                ckpt = storage.latest_checkpoint or ckpt
                if self.run_config.verbose:
                    print(f"[grt] training attempt failed ({e.__class__.__name__}); restarting from "
                          f"{ckpt.path if ckpt else 'scratch'} ({failures}/{fc.max_failures})", flush=True)
        storage.finish()
        result = Result(metrics=storage.last_metrics or {}, checkpoint=storage.latest_checkpoint,
                        path=storage.trial_dir, error=err, best_checkpoints=storage.best_checkpoints(),
                        storage=storage)
        if err is not None:
            raise TrainingFailedError(f"Training failed after {failures} attempt(s): {err}") from err
        return result

    # ------------------------------------------------------------------------------------
    def _run_attempt(self, storage: RunStorage, ckpt: Optional[Checkpoint], attempt: int):
        if not rt.is_initialized():
            rt.init(ignore_reinit_error=True)
        n = self.scaling.num_workers
        use_gpu = self.scaling.use_gpu
        authkey = secrets.token_bytes(16)
        # backlog >= workers: with the default of 1, simultaneous connects beyond the first are
        # dropped by the kernel and retried with SYN back-off (1, 2, 4 ... s); at 8 workers a rank
        # could sit in back-off for minutes (tests/test_world8_cpu.py)
        listener = Listener(("127.0.0.1", 0), authkey=authkey, backlog=max(64, 2 * n))
        address = listener.address
        master_port = _free_port()
        backend = self._backend()
        timeout_s = getattr(self.backend_config, "timeout_s", 1800)
        worker_cls = rt.remote(TrainWorker).options(num_cpus=self.scaling.cpus_per_worker if not use_gpu else 0,
                                                   num_gpus=self.scaling.gpus_per_worker)
        actors = [worker_cls.remote() for _ in range(n)]
        try:
            gpus = rt.get([a.gpu.remote() for a in actors], timeout=600)
            order = sorted(range(n), key=lambda i: (gpus[i], i))
            actors = [actors[i] for i in order]
            gpus = [gpus[i] for i in order]
            ctx_fields = dict(trial_name=storage.trial_name, trial_id=storage.trial_id,
                              experiment_name=storage.experiment_name, trial_dir=storage.trial_dir,
                              storage_path=storage.storage_path)
            payload = cloudpickle.dumps(self.fn)
            # Ray Train: each dataset is streaming_split once in the driver; worker r consumes split r
            # of ONE execution (a coordinator process deals the rows), not its own re-execution
            per_rank = [dict() for _ in range(n)]
            coords = []
            for name, ds in self.datasets.items():
                if hasattr(ds, "streaming_split"):
                    splits = ds.streaming_split(n, equal=True)
                    coords.append(splits)
                    for r in range(n):
                        per_rank[r][name] = splits[r]
                else:
                    for r in range(n):
                        per_rank[r][name] = ds
            refs = []
            for r, a in enumerate(actors):
                local_rank = gpus[r] if (use_gpu and gpus[r] >= 0) else r
                refs.append(a.run.remote(payload, self.config, r, n, local_rank, n, "127.0.0.1", master_port, backend,
                                         timeout_s, ctx_fields, address, authkey, ckpt.path if ckpt else None,
                                         per_rank[r], storage.iteration if ckpt else 0, attempt, use_gpu))
            self._serve(listener, refs, n, storage)
            rt.get(refs, timeout=600)
        finally:
            listener.close()
            for splits in locals().get("coords", []):
                splits[0].shutdown()
            for a in actors:
                try:
                    rt.kill(a)
                except Exception:
                    pass

    def _serve(self, listener: Listener, refs, n, storage: RunStorage):
        conns = {}
        listener._listener._socket.settimeout(1.0)
        t0 = time.time()
        while len(conns) < n:
            self._check_failed(refs)
            try:
                c = listener.accept()
            except (socket.timeout, OSError):
                if time.time() - t0 > 1800:
                    raise TimeoutError("workers did not connect")
                continue
            kind, rank = c.recv()
            conns[rank] = c
        pending: Dict[int, Dict[int, tuple]] = {}
        done = set()
        while len(done) < n:
            ready = conn_wait(list(c for r, c in conns.items() if r not in done), timeout=0.5)
            if not ready:
                self._check_failed(refs)
                continue
            for c in ready:
                try:
                    msg = c.recv()
                except (EOFError, OSError):
                    self._check_failed(refs, force=True)
                    raise RuntimeError("lost connection to a training worker")
                if msg[0] == "report":
                    _, rank, idx, metrics, staged, _ts = msg
                    pending.setdefault(idx, {})[rank] = (metrics, staged)
                    if len(pending[idx]) == n:
                        items = pending.pop(idx)
                        dirs = [items[r][1] for r in sorted(items) if items[r][1]]
                        path = storage.record(items[0][0], dirs)
                        if self.run_config.verbose >= 2:
                            print(f"[grt] report {idx}: {items[0][0]}", flush=True)
                        for r in sorted(conns):
                            conns[r].send(("ack", path))
                elif msg[0] == "done":
                    _, rank, ok, err = msg
                    done.add(rank)
                    if not ok:
                        self._check_failed(refs, force=True)
                        raise RayTaskError("train_loop_per_worker", err or "worker failed")

    @staticmethod
    def _check_failed(refs, force=False):
        ready, _ = rt.wait(refs, num_returns=len(refs), timeout=0)
        for r in ready:
            rt.get(r)  # raises RayTaskError / ActorDiedError for a failed rank
        if force:
            deadline = time.time() + 30
            while time.time() < deadline:
                ready, _ = rt.wait(refs, num_returns=len(refs), timeout=0)
                for r in ready:
                    rt.get(r)
                if len(ready) == len(refs):
                    return
                time.sleep(0.1)


class TorchTrainer(DataParallelTrainer):
    _name = "TorchTrainer"

    def __init__(self, train_loop_per_worker, *, train_loop_config=None, torch_config=None, scaling_config=None,
                 run_config=None, datasets=None, resume_from_checkpoint=None, metadata=None, dataset_config=None):
        super().__init__(train_loop_per_worker, train_loop_config=train_loop_config, scaling_config=scaling_config,
                         run_config=run_config, backend_config=torch_config, datasets=datasets,
                         resume_from_checkpoint=resume_from_checkpoint, metadata=metadata,
                         dataset_config=dataset_config)
