"""Node-local cluster spec: the MI355X replacement for the reference's RayCluster custom resource.

The reference brings up a KubeRay ``RayCluster`` on GKE (reference a3-mega/ray-cluster-config.yaml:1-111,
a3-ultra/ray-cluster-config.yaml:1-127): a CPU-less head (``rayStartParams: num-cpus: "0"``,
dashboard on 0.0.0.0:8265), ``${NUM_NODES}`` worker pods with ``${NUM_GPUS_PER_NODE}`` GPUs, a GCS
FUSE bucket mounted at ``/mnt/pvc`` and env vars, templated with ``envsubst``
(a3-mega/gke-ray-cluster-setup.sh:60). Here the cluster is ONE MI355X node: the spec keeps the same
knobs (head port / CPU reservation, GPUs per node, worker env, storage path, uid/gid/mode of the
mount) and the same ``${VAR}`` / ``${VAR:-default}`` templating, and is validated against the GPUs
actually present.
"""
from __future__ import annotations

import os
import re
from dataclasses import asdict, dataclass, field
from typing import Dict, Optional

import yaml

_VAR = re.compile(r"\$\{([A-Za-z_][A-Za-z0-9_]*)(?::-([^}]*))?\}|\$([A-Za-z_][A-Za-z0-9_]*)")


def envsubst(text: str, env: Optional[Dict[str, str]] = None) -> str:
    """``envsubst`` semantics plus ``${VAR:-default}``; unset variables become empty strings."""
    env = os.environ if env is None else env

    def rep(m):
        name = m.group(1) or m.group(3)
        if name in env and env[name] != "":
            return env[name]
        return m.group(2) if m.group(2) is not None else ""
    return _VAR.sub(rep, text)


@dataclass
class HeadSpec:
    dashboard_host: str = "127.0.0.1"
    dashboard_port: int = 8265
    num_cpus: float = 0.0  # reference head reserves no CPUs for tasks (a3-mega/ray-cluster-config.yaml:11)


@dataclass
class WorkerSpec:
    num_gpus_per_node: int = 8
    num_cpus: Optional[float] = None
    memory_gb: Optional[float] = None
    env: Dict[str, str] = field(default_factory=dict)


@dataclass
class StorageSpec:
    path: str = "/tmp/grt_storage"  # replaces the GCS FUSE bucket mounted at /mnt/pvc
    mode: str = "0775"


@dataclass
class ClusterSpec:
    name: str = "grt-mi355x"
    head: HeadSpec = field(default_factory=HeadSpec)
    workers: WorkerSpec = field(default_factory=WorkerSpec)
    storage: StorageSpec = field(default_factory=StorageSpec)

    @property
    def address(self) -> str:
        return f"http://{self.head.dashboard_host}:{self.head.dashboard_port}"

    def to_dict(self):
        return asdict(self)

    @classmethod
    def from_dict(cls, d: dict) -> "ClusterSpec":
        d = dict(d or {})
        known = {"name", "head", "workers", "storage"}
        unknown = set(d) - known
        if unknown:
            raise ValueError(f"unknown cluster spec keys: {sorted(unknown)}")
        h = d.get("head") or {}
        w = d.get("workers") or {}
        s = d.get("storage") or {}
        w_env = {str(k): str(v) for k, v in (w.pop("env", None) or {}).items()} if isinstance(w, dict) else {}
        spec = cls(name=str(d.get("name", "grt-mi355x")),
                   head=HeadSpec(**{k: _num(v) for k, v in h.items()}),
                   workers=WorkerSpec(env=w_env, **{k: _num(v) for k, v in w.items()}),
                   storage=StorageSpec(**{k: str(v) for k, v in s.items()}))
        return spec

    @classmethod
    def load(cls, path: str, env: Optional[Dict[str, str]] = None) -> "ClusterSpec":
        with open(path) as f:
            text = envsubst(f.read(), env)
        return cls.from_dict(yaml.safe_load(text))

    def validate(self, available_gpus: Optional[int] = None):
        if self.workers.num_gpus_per_node < 0:
            raise ValueError("num_gpus_per_node must be >= 0")
        if available_gpus is not None and self.workers.num_gpus_per_node > available_gpus:
            raise ValueError(f"spec asks for {self.workers.num_gpus_per_node} GPUs but the node has {available_gpus}")
        if not (0 < int(self.head.dashboard_port) < 65536):
            raise ValueError("dashboard_port out of range")
        return self


def _num(v):
    if isinstance(v, str):
        for t in (int, float):
            try:
                return t(v)
            except ValueError:
                pass
    return v
