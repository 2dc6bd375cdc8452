"""Local single-node task/actor runtime (the Ray-Core surface the reference uses).

Reference usage: ``ray.init(address='auto', ignore_reinit_error=True)``, ``ray.is_initialized()``,
``@ray.remote(num_cpus=1)`` + ``.remote()``, ``ray.get(ref, timeout=1800)`` with
RayTaskError / GetTimeoutError semantics (reference ray-jobs/prepare_wikitext2_ray_job.py:18,95-109),
and the worker actors that Ray Train places one per GPU.

Design for one MI355X node instead of a GKE/KubeRay cluster:
* the "head" lives in the driver process: a scheduler thread dispatches tasks to a pool of
  spawned worker processes and tracks per-node resources (CPU slots, the 8 GPUs);
* actors are dedicated processes executing their method calls serially; GPU actors get a GPU
  index (``GRT_ASSIGNED_GPU``) but keep every device visible so RCCL can use xGMI peer access;
* arguments/results travel as cloudpickle payloads over pipes; large numpy / torch CPU payloads
  go through the shared-memory object store (``runtime/object_store.py``) instead;
* GPUs are LEASED from a node-wide ledger (``runtime/gpu_ledger.py``: one ``flock``-ed file per
  GPU under the node's grt tmpdir), so concurrent drivers — e.g. two jobs submitted to one
  ``grt start --head`` cluster, each attaching with ``ray.init(address='auto')`` — never hold the
  same GPU; a lease dies with its process. Tasks and actors learn their GPUs through
  ``GRT_ASSIGNED_GPU`` / ``get_gpu_ids()`` (Ray's ``ray.get_gpu_ids()``);
* failures surface exactly where the reference expects them: a raising task -> ``RayTaskError``
  from ``get``; a dead worker/actor process -> ``WorkerCrashedError`` / ``ActorDiedError``;
  ``get(timeout=)`` -> ``GetTimeoutError``.
"""
from __future__ import annotations

import itertools
import multiprocessing as mp
import os
import queue
import sys
import threading
import time
import traceback
import uuid
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import cloudpickle

from .errors import ActorDiedError, GetTimeoutError, RayTaskError, WorkerCrashedError
from . import object_store

_CTX = mp.get_context("spawn")


# --------------------------------------------------------------------------------- refs
class ObjectRef:
    __slots__ = ("id", "_owner")

    def __init__(self, oid: str, owner=None):
        self.id = oid
        self._owner = owner

    def __repr__(self):
        return f"ObjectRef({self.id[:16]})"

    def __hash__(self):
        return hash(self.id)

    def __eq__(self, other):
        return isinstance(other, ObjectRef) and other.id == self.id

    def __reduce__(self):
        return (ObjectRef, (self.id,))

    def hex(self):
        return self.id


@dataclass
class _Entry:
    event: threading.Event = field(default_factory=threading.Event)
    ok: bool = True
    value: Any = None
    payload: Optional[bytes] = None


# --------------------------------------------------------------------------------- worker
def _apply_env(env: Dict[str, str], working_dir: Optional[str]):
    os.environ.update({k: str(v) for k, v in (env or {}).items()})
    if working_dir:
        os.chdir(working_dir)
        if working_dir not in sys.path:
            sys.path.insert(0, working_dir)


def _orphan_watchdog(parent: int):
    """Workers are not daemonic (so they may start their own children: DataLoader workers, data
    coordinators — as Ray actors can); instead each exits when its driver disappears."""
    while True:
        time.sleep(1.0)
        if os.getppid() != parent:
            os._exit(1)


def _worker_main(q_in, q_out, env, working_dir, actor_spec, parent=None):
    if parent is not None:
        threading.Thread(target=_orphan_watchdog, args=(parent,), daemon=True, name="grt-orphan").start()
    _apply_env(env, working_dir)
    instance = None
    if actor_spec is not None:
        try:
            cls, args, kwargs = cloudpickle.loads(actor_spec)
            instance = cls(*object_store.materialize(args), **object_store.materialize(kwargs))
            q_out.put(("__actor_ready__", True, None))
        except BaseException:
            q_out.put(("__actor_ready__", False, cloudpickle.dumps(RayTaskError("__init__", traceback.format_exc()))))
            return
    while True:
        msg = q_in.get()
        if msg is None:
            break
        task_id, payload, gpus = msg if len(msg) == 3 else (*msg, None)
        if gpus is not None:  # this task's GPU lease (pooled workers run tasks of different GPUs)
            if gpus:
                os.environ["GRT_ASSIGNED_GPU"] = ",".join(map(str, gpus))
            else:
                os.environ.pop("GRT_ASSIGNED_GPU", None)
        name = "?"
        try:
            fn, args, kwargs, name = cloudpickle.loads(payload)
            args = object_store.materialize(args)
            kwargs = object_store.materialize(kwargs)
            if instance is not None:
                result = getattr(instance, fn)(*args, **kwargs)
            else:
                result = fn(*args, **kwargs)
            q_out.put((task_id, True, object_store.pack(result)))
        except BaseException as e:  # noqa: BLE001 - propagated to the caller
            err = RayTaskError(name, traceback.format_exc(), cause=_safe_exc(e))
            q_out.put((task_id, False, cloudpickle.dumps(err)))
            if isinstance(e, (KeyboardInterrupt, SystemExit)):
                break


def _safe_exc(e):
    try:
        cloudpickle.dumps(e)
        return e
    except Exception:
        return RuntimeError(repr(e))


class _Proc:
    def __init__(self, env, working_dir, actor_spec=None, name="worker"):
        self.q_in = _CTX.Queue()
        self.q_out = _CTX.Queue()
        self.proc = _CTX.Process(target=_worker_main, args=(self.q_in, self.q_out, env, working_dir, actor_spec,
                                                            os.getpid()),
                                 daemon=False, name=name)
        self.proc.start()
        self.busy: Optional[str] = None
        self.pending: List[str] = []

    def alive(self):
        return self.proc.is_alive()

    def stop(self, timeout=2.0):
        try:
            self.q_in.put(None)
        except Exception:
            pass
        self.proc.join(timeout)
        if self.proc.is_alive():
            self.proc.kill()
            self.proc.join(timeout)


# --------------------------------------------------------------------------------- runtime
@dataclass
class _Task:
    task_id: str
    fn: Any
    args: tuple
    kwargs: dict
    name: str
    num_cpus: float
    num_gpus: float
    max_retries: int = 0


class Runtime:
    def __init__(self, num_cpus=None, num_gpus=None, runtime_env=None, namespace=None):
        self.num_cpus = float(num_cpus if num_cpus is not None else (os.cpu_count() or 1))
        if num_gpus is None:
            num_gpus = _count_gpus()
        self.num_gpus = float(num_gpus)
        self.runtime_env = runtime_env or {}
        self.namespace = namespace or "default"
        self.session_id = uuid.uuid4().hex[:12]
        self._lock = threading.RLock()
        self._objects: Dict[str, _Entry] = {}
        self._pending: "queue.Queue[_Task]" = queue.Queue()
        self._waiting: List[_Task] = []
        self._idle: List[_Proc] = []
        self._all: List[_Proc] = []
        self._free_cpus = self.num_cpus
        from .gpu_ledger import GpuLedger
        self._ledger = GpuLedger.for_node(int(self.num_gpus))
        self._task_res: Dict[str, tuple] = {}
        self._actors: Dict[str, "_ActorState"] = {}
        self._stop = threading.Event()
        self._ids = itertools.count()
        self._sched = threading.Thread(target=self._scheduler_loop, daemon=True, name="grt-sched")
        self._sched.start()

    # -- object table
    def _new_ref(self) -> ObjectRef:
        oid = f"{self.session_id}{next(self._ids):012x}"
        with self._lock:
            self._objects[oid] = _Entry()
        return ObjectRef(oid)

    def _set(self, oid, ok, payload=None, value=None):
        with self._lock:
            e = self._objects.setdefault(oid, _Entry())
        e.ok = ok
        e.payload = payload
        e.value = value
        e.event.set()

    def put(self, value) -> ObjectRef:
        ref = self._new_ref()
        self._set(ref.id, True, value=value)
        return ref

    def _resolve(self, e: _Entry):
        if e.payload is not None:
            e.value = object_store.unpack(e.payload) if e.ok else cloudpickle.loads(e.payload)
            e.payload = None
        if not e.ok:
            raise e.value
        return e.value

    def get(self, refs, timeout=None):
        single = isinstance(refs, ObjectRef)
        lst = [refs] if single else list(refs)
        deadline = None if timeout is None else time.monotonic() + timeout
        out = []
        for r in lst:
            if not isinstance(r, ObjectRef):
                raise TypeError(f"get() expects ObjectRef(s), got {type(r)}")
            with self._lock:
                e = self._objects.get(r.id)
            if e is None:
                raise ValueError(f"unknown object {r}")
            rem = None if deadline is None else max(0.0, deadline - time.monotonic())
            if not e.event.wait(rem):
                raise GetTimeoutError(f"get timed out after {timeout}s waiting for {r}")
            out.append(self._resolve(e))
        return out[0] if single else out

    def wait(self, refs, num_returns=1, timeout=None):
        refs = list(refs)
        deadline = None if timeout is None else time.monotonic() + timeout
        while True:
            ready = [r for r in refs if self._objects[r.id].event.is_set()]
            if len(ready) >= num_returns or (deadline is not None and time.monotonic() >= deadline):
                ready = ready[:num_returns]
                return ready, [r for r in refs if r not in ready]
            time.sleep(0.002)

    # -- tasks
    def submit(self, fn, args, kwargs, name, num_cpus=1.0, num_gpus=0.0, max_retries=0) -> ObjectRef:
        if num_cpus > self.num_cpus or num_gpus > self.num_gpus:
            raise ValueError(f"task {name} requests cpus={num_cpus} gpus={num_gpus}, node has "
                             f"cpus={self.num_cpus} gpus={self.num_gpus}")
        ref = self._new_ref()
        self._pending.put(_Task(ref.id, fn, args, kwargs, name, num_cpus, num_gpus, max_retries))
        return ref

    def _deps_ready(self, t: _Task):
        for a in itertools.chain(t.args, t.kwargs.values()):
            if isinstance(a, ObjectRef) and not self._objects[a.id].event.is_set():
                return False
        return True

    def _materialize_args(self, t: _Task):
        def rv(a):
            if isinstance(a, ObjectRef):
                return self.get(a)
            return a
        return tuple(rv(a) for a in t.args), {k: rv(v) for k, v in t.kwargs.items()}

    def _scheduler_loop(self):
        while not self._stop.is_set():
            try:
                t = self._pending.get(timeout=0.01)
                self._waiting.append(t)
            except queue.Empty:
                pass
            self._drain_results()
            still = []
            for t in self._waiting:
                if not self._deps_ready(t):
                    still.append(t)
                    continue
                if t.num_cpus > self._free_cpus:
                    still.append(t)
                    continue
                gpus = self._ledger.try_acquire(int(t.num_gpus))
                if gpus is None:  # held by this or another driver on the node: wait (Ray semantics)
                    still.append(t)
                    continue
                try:
                    args, kwargs = self._materialize_args(t)
                except BaseException as e:  # dependency failed: propagate
                    self._ledger.release(gpus)
                    self._set(t.task_id, False, payload=cloudpickle.dumps(
                        e if isinstance(e, RayTaskError) else RayTaskError(t.name, traceback.format_exc())))
                    continue
                self._free_cpus -= t.num_cpus
                w = self._idle.pop() if self._idle else self._spawn(gpus)
                w.busy = t.task_id
                self._task_res[t.task_id] = (t, w, gpus)
                payload = cloudpickle.dumps((t.fn, object_store.pack_args(args), object_store.pack_args(kwargs), t.name))
                w.q_in.put((t.task_id, payload, gpus))
            self._waiting = still

    def _spawn(self, gpus):
        env = dict(self.runtime_env.get("env_vars", {}))  # the GPU lease travels with each task
        p = _Proc(env, self.runtime_env.get("working_dir"), name="grt-worker")
        self._all.append(p)
        return p

    def _drain_results(self):
        for tid, (t, w, gpus) in list(self._task_res.items()):
            got = False
            try:
                while True:
                    rid, ok, payload = w.q_out.get_nowait()
                    self._set(rid, ok, payload=payload)
                    got = True
            except queue.Empty:
                pass
            except (EOFError, OSError):
                pass
            if got or not w.alive():
                if not got:
                    if t.max_retries > 0:
                        t.max_retries -= 1
                        self._pending.put(t)
                    else:
                        self._set(tid, False, payload=cloudpickle.dumps(
                            WorkerCrashedError(f"worker running task {t.name} died (exitcode {w.proc.exitcode})")))
                    self._all.remove(w)
                else:
                    w.busy = None
                    self._idle.append(w)
                self._free_cpus += t.num_cpus
                self._ledger.release(gpus)
                del self._task_res[tid]

    # -- actors
    def create_actor(self, cls, args, kwargs, num_cpus=0.0, num_gpus=0.0, name=None, env=None):
        ngpu = int(num_gpus)
        if ngpu > self.num_gpus:
            raise ValueError(f"actor {name or cls.__name__} requests {ngpu} GPUs, node has {int(self.num_gpus)}")
        deadline = time.monotonic() + float(os.environ.get("GRT_PLACEMENT_TIMEOUT_S", "600"))
        while True:
            with self._lock:
                gpus = self._ledger.try_acquire(ngpu)
            if gpus is not None:
                break
            if time.monotonic() > deadline:
                raise RuntimeError(f"cannot place actor needing {ngpu} GPUs (leased: {self._ledger.describe()})")
            time.sleep(0.05)
        aenv = dict(self.runtime_env.get("env_vars", {}))
        aenv.update(env or {})
        if gpus:
            aenv["GRT_ASSIGNED_GPU"] = ",".join(map(str, gpus))
        spec = cloudpickle.dumps((cls, object_store.pack_args(args), object_store.pack_args(kwargs)))
        p = _Proc(aenv, self.runtime_env.get("working_dir"), actor_spec=spec, name=f"grt-actor-{name or cls.__name__}")
        st = _ActorState(self, p, gpus, name or cls.__name__)
        self._actors[st.actor_id] = st
        return st

    def release_actor(self, st: "_ActorState"):
        with self._lock:
            self._ledger.release(st.gpus)
            st.gpus = []
        self._actors.pop(st.actor_id, None)

    def available_resources(self):
        return {"CPU": self._free_cpus, "GPU": float(self._ledger.num_free())}

    def cluster_resources(self):
        return {"CPU": self.num_cpus, "GPU": self.num_gpus}

    def shutdown(self):
        self._stop.set()
        for st in list(self._actors.values()):
            st.kill()
        for p in self._all:
            p.stop()
        self._all.clear()
        self._ledger.close()


class _ActorState:
    def __init__(self, rt: Runtime, proc: _Proc, gpus, name):
        self.rt = rt
        self.proc = proc
        self.gpus = gpus
        self.name = name
        self.actor_id = uuid.uuid4().hex
        self.ready = rt._new_ref()
        self._refs: Dict[str, ObjectRef] = {}
        self._lock = threading.Lock()
        self._dead = False
        self._thread = threading.Thread(target=self._pump, daemon=True, name=f"grt-actor-pump-{name}")
        self._thread.start()

    def _pump(self):
        while True:
            try:
                rid, ok, payload = self.proc.q_out.get(timeout=0.05)
            except queue.Empty:
                if not self.proc.alive():
                    self._fail_all(f"actor {self.name} died (exitcode {self.proc.proc.exitcode})")
                    return
                continue
            except (EOFError, OSError):
                self._fail_all(f"actor {self.name} pipe closed")
                return
            if rid == "__actor_ready__":
                self.rt._set(self.ready.id, ok, payload=payload if not ok else None, value=True)
                if not ok:
                    self._dead = True
                continue
            self.rt._set(rid, ok, payload=payload)
            with self._lock:
                self._refs.pop(rid, None)

    def _fail_all(self, msg):
        self._dead = True
        with self._lock:
            refs = list(self._refs.values())
            self._refs.clear()
        err = cloudpickle.dumps(ActorDiedError(msg))
        for r in refs:
            self.rt._set(r.id, False, payload=err)
        if not self.rt._objects[self.ready.id].event.is_set():
            self.rt._set(self.ready.id, False, payload=err)
        self.rt.release_actor(self)

    def call(self, method, args, kwargs) -> ObjectRef:
        ref = self.rt._new_ref()
        if self._dead:
            self.rt._set(ref.id, False, payload=cloudpickle.dumps(ActorDiedError(f"actor {self.name} is dead")))
            return ref
        with self._lock:
            self._refs[ref.id] = ref
        args = tuple(self.rt.get(a) if isinstance(a, ObjectRef) else a for a in args)
        kwargs = {k: (self.rt.get(v) if isinstance(v, ObjectRef) else v) for k, v in kwargs.items()}
        self.proc.q_in.put((ref.id, cloudpickle.dumps((method, object_store.pack_args(args),
                                                        object_store.pack_args(kwargs), f"{self.name}.{method}"))))
        return ref

    def kill(self):
        if self.proc.alive():
            self.proc.proc.kill()
            self.proc.proc.join(5)
        self._fail_all(f"actor {self.name} was killed")


def _count_gpus() -> int:
    env = os.environ.get("GRT_NUM_GPUS")
    if env is not None:
        return int(env)
    from ..cluster.head import read_current_cluster
    cur = read_current_cluster()  # a `grt start --head` cluster caps the GPUs this driver may use
    if cur is not None and cur.get("num_gpus") is not None:
        return int(cur["num_gpus"])
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


# --------------------------------------------------------------------------------- module API
_RUNTIME: Optional[Runtime] = None
_RLOCK = threading.Lock()


def init(address: Optional[str] = None, *, num_cpus=None, num_gpus=None, ignore_reinit_error=False,
         runtime_env=None, namespace=None, **_ignored) -> Runtime:
    """Start (or, with ``address='auto'``, attach to) the node-local runtime."""
    global _RUNTIME
    with _RLOCK:
        if _RUNTIME is not None:
            if ignore_reinit_error or address == "auto":
                return _RUNTIME
            raise RuntimeError("runtime already initialised (pass ignore_reinit_error=True)")
        if address not in (None, "auto", "local") and not str(address).startswith(("grt://", "local")):
            from ..cluster.config import resolve_address  # e.g. the dashboard address of `grt cluster`
            resolve_address(address)
        if runtime_env and runtime_env.get("env_vars"):
            os.environ.update({k: str(v) for k, v in runtime_env["env_vars"].items()})
        _RUNTIME = Runtime(num_cpus=num_cpus, num_gpus=num_gpus, runtime_env=runtime_env, namespace=namespace)
        import atexit
        atexit.register(shutdown)  # before multiprocessing joins its (non-daemonic) children
        return _RUNTIME


def is_initialized() -> bool:
    return _RUNTIME is not None


def _rt() -> Runtime:
    return _RUNTIME if _RUNTIME is not None else init()


def shutdown():
    global _RUNTIME
    with _RLOCK:
        if _RUNTIME is not None:
            _RUNTIME.shutdown()
            _RUNTIME = None


def get(refs, timeout=None):
    return _rt().get(refs, timeout=timeout)


def put(value) -> ObjectRef:
    return _rt().put(value)


def wait(refs, num_returns=1, timeout=None):
    return _rt().wait(refs, num_returns=num_returns, timeout=timeout)


def available_resources():
    return _rt().available_resources()


def cluster_resources():
    return _rt().cluster_resources()


def nodes():
    rt = _rt()
    return [{"NodeID": rt.session_id, "Alive": True, "Resources": rt.cluster_resources(),
             "NodeManagerAddress": "127.0.0.1"}]


def kill(actor_handle, no_restart=True):
    actor_handle._state.kill()


def get_gpu_ids() -> List[int]:
    """GPU indices leased to the calling task / actor (``ray.get_gpu_ids()``)."""
    v = os.environ.get("GRT_ASSIGNED_GPU", "")
    return [int(x) for x in v.split(",") if x.strip()]
