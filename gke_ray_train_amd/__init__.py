"""gke_ray_train_amd: MI355X-native training framework (PyTorch-ROCm + gfx950 HIP kernels + RCCL)."""
import os as _os

# Kernel arguments in device memory: shorter launch latency for the many small kernels of a step
# (headline +0.35 %, reference SFT job +1.6 %: scripts/gpu_r4_envab.sh, profiles/r4_batch1.md). The
# HIP runtime reads it when it initialises, i.e. at the first GPU call after this import; a value
# already in the environment wins.
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
