"""Loader for the in-tree native libraries (``_C.so`` HIP kernels, ``_rt.so`` CPU runtime).

Policy: on a host with a visible GPU the HIP kernels are MANDATORY — any op on a GPU tensor
raises if ``_C.so`` is missing or fails to load (no silent eager fallback). On CPU-only hosts
the ops use their pure-PyTorch reference implementations (``ops/_ref.py``), which are also the
numerics oracles of the GPU tests.
"""
from __future__ import annotations

import ctypes
import importlib.util
import os
import threading
from pathlib import Path

_PKG = Path(__file__).resolve().parent
_lock = threading.Lock()
_C = None
_C_err: Exception | None = None
_RT = None


def _load_ext(name: str, path: Path):
    import torch  # noqa: F401  — torch's HIP runtime must be loaded before our extension

    spec = importlib.util.spec_from_file_location(f"gke_ray_train_amd.{name}", str(path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class _SyncChecked:
    """``GRT_DEBUG_SYNC=1``: every native op is followed by a device synchronize, so an illegal
    access / kernel fault is reported at the op that launched it (the HIP_LAUNCH_BLOCKING /
    AMD_SERIALIZE_KERNEL debugging mode of SURVEY §5.2) instead of at a later sync point."""

    def __init__(self, mod):
        self._mod = mod

    def __getattr__(self, name):
        fn = getattr(self._mod, name)
        if not callable(fn):
            return fn

        def wrapped(*a, **k):
            import torch
            out = fn(*a, **k)
            try:
                torch.cuda.synchronize()
            except RuntimeError as e:
                raise RuntimeError(f"native op {name} failed on the device: {e}") from e
            return out
        return wrapped


def kernels():
    """Return the ``_C`` extension module; raise with a clear message if unavailable."""
    global _C, _C_err
    if _C is not None:
        return _C
    with _lock:
        if _C is None and _C_err is None:
            so = _PKG / "_C.so"
            if not so.exists() and os.environ.get("GRT_AUTO_BUILD", "1") == "1":
                try:
                    from . import _build
                    _build.build_kernels()
                except Exception as e:  # pragma: no cover - reported below
                    _C_err = e
            if _C_err is None:
                try:
                    _C = _load_ext("_C", so)
                    if os.environ.get("GRT_DEBUG_SYNC", "0") == "1":
                        _C = _SyncChecked(_C)
                except Exception as e:
                    _C_err = e
    if _C is None:
        raise RuntimeError(
            "gke_ray_train_amd HIP kernels (_C.so) are not available: "
            f"{_C_err!r}. Build them with `python -m gke_ray_train_amd._build`.")
    return _C


def kernels_available() -> bool:
    try:
        kernels()
        return True
    except RuntimeError:
        return False


def runtime_lib():
    """ctypes handle to ``_rt.so`` (CPU native runtime), building it on first use."""
    global _RT
    if _RT is not None:
        return _RT
    with _lock:
        if _RT is None:
            so = _PKG / "_rt.so"
            if not so.exists():
                from . import _build
                _build.build_runtime()
            _RT = ctypes.CDLL(str(so))
    return _RT
