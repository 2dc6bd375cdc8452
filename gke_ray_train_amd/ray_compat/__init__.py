"""Drop-in ``ray`` import shim: put ``gke_ray_train_amd/ray_compat`` on ``sys.path`` (or call
``gke_ray_train_amd.ray_compat.install()``) and reference-style scripts (``import ray``,
``from ray.train.torch import TorchTrainer``) run unmodified on this framework."""
import os
import sys

SHIM_DIR = os.path.dirname(os.path.abspath(__file__))


def install():
    if SHIM_DIR not in sys.path:
        sys.path.insert(0, SHIM_DIR)
    import ray  # noqa: F401
    return ray
