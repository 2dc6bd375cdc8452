"""ROCTX ranges/markers (shown by ``rocprofv3 --marker-trace`` next to the kernel trace).

The reference has no tracing (grep profiler/rocprof/record_function -> 0 hits); its only
observability is GKE's managed Ray logging (a3-mega/gke-ray-cluster-setup.sh:21-22). Here the hot
loop annotates forward / backward / grad-sync / optimizer with ROCTX ranges by calling the ROCm
profiler SDK's C API directly through ctypes — no torch.profiler dependency, ~1 µs per call, a
no-op when the library is absent (CPU-only hosts) or ``GRT_ROCTX=0``.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading

_LIB = None
_LOCK = threading.Lock()
_CANDIDATES = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so")


def _lib():
    global _LIB
    if _LIB is None:
        with _LOCK:
            if _LIB is None:
                lib = False
                if os.environ.get("GRT_ROCTX", "1") != "0":
                    for name in _CANDIDATES:
                        for path in (name, os.path.join("/opt/rocm/lib", name)):
                            try:
                                lib = ctypes.CDLL(path)
                                break
                            except OSError:
                                continue
                        if lib:
                            break
                if lib:
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangeStartA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangeStartA.restype = ctypes.c_uint64
                    lib.roctxRangeStop.argtypes = [ctypes.c_uint64]
                    if hasattr(lib, "roctxNameOsThread"):
                        lib.roctxNameOsThread.argtypes = [ctypes.c_char_p]
                _LIB = lib
    return _LIB or None


def available() -> bool:
    return _lib() is not None


def push(name: str) -> int:
    lib = _lib()
    return lib.roctxRangePushA(name.encode()) if lib else -1


def pop() -> int:
    lib = _lib()
    return lib.roctxRangePop() if lib else -1


def mark(name: str):
    lib = _lib()
    if lib:
        lib.roctxMarkA(name.encode())


def start(name: str) -> int:
    """Process-wide (non-nested) range, may end on another thread: returns an id for ``stop``."""
    lib = _lib()
    return lib.roctxRangeStartA(name.encode()) if lib else 0


def stop(range_id: int):
    lib = _lib()
    if lib and range_id:
        lib.roctxRangeStop(range_id)


def name_thread(name: str):
    lib = _lib()
    if lib and hasattr(lib, "roctxNameOsThread"):
        lib.roctxNameOsThread(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors the ROCTX vocabulary
    pushed = push(name) >= 0
    try:
        yield
    finally:
        if pushed:
            pop()
