"""Node-local task / actor runtime (Ray-Core equivalent for one 8-GPU MI355X node)."""
from .api import ActorClass, ActorHandle, RemoteFunction, remote
from .core import (ObjectRef, available_resources, cluster_resources, get, get_gpu_ids, init, is_initialized, kill,
                   nodes, put, shutdown, wait)
from .errors import ActorDiedError, GetTimeoutError, RayError, RayTaskError, TrainingFailedError, WorkerCrashedError

__all__ = ["ActorClass", "ActorHandle", "RemoteFunction", "remote", "ObjectRef", "available_resources",
           "cluster_resources", "get", "get_gpu_ids", "init", "is_initialized", "kill", "nodes", "put", "shutdown", "wait",
           "ActorDiedError", "GetTimeoutError", "RayError", "RayTaskError", "TrainingFailedError",
           "WorkerCrashedError"]
