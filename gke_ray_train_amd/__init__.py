"""gke_ray_train_amd: MI355X-native training framework (PyTorch-ROCm + gfx950 HIP kernels + RCCL)."""
import os as _os

# HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory: +0.35 % headline, +1.6 % reference
# SFT job, profiles/r4_batch1.md) is set by the launch entry points (bench.py, jobs/*.py) before
# their first GPU call, not by importing the package: the HIP runtime reads it once when it
# initialises, so an import-time default would depend on import order and leak into every importer.
