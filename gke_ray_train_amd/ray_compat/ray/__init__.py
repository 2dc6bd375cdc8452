"""``ray`` compatibility package backed by gke_ray_train_amd's node-local runtime."""
from gke_ray_train_amd.runtime import (ObjectRef, available_resources, cluster_resources, get, get_gpu_ids, init,
                                       is_initialized, kill, nodes, put, remote, shutdown, wait)
from gke_ray_train_amd.runtime import errors as exceptions  # noqa: F401
from . import cloudpickle  # noqa: F401
from . import train  # noqa: F401

__version__ = "2.46.0+grt"
__all__ = ["ObjectRef", "available_resources", "cluster_resources", "get", "get_gpu_ids", "init", "is_initialized", "kill", "nodes",
           "put", "remote", "shutdown", "wait", "train", "cloudpickle", "exceptions"]
