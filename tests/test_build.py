"""Native build checks on the CPU host: the gfx950 kernels cross-compile (also in the
GRT_KERNEL_CHECKS debugging configuration) and the C++ runtime library exports its C API."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_checked_kernel_build_compiles(tmp_path):
    inc = os.path.join(ROOT, "gke_ray_train_amd", "csrc", "include")
    for k in ("gemm", "attention"):
        src = os.path.join(ROOT, "gke_ray_train_amd", "csrc", "kernels", f"{k}.hip")
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-std=c++17", "-DGRT_KERNEL_CHECKS=1", "-I", inc,
                            "-c", src, "-o", str(tmp_path / f"{k}.o")], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]


def test_runtime_library_exports():
    from gke_ray_train_amd import _native
    lib = _native.runtime_lib()
    for sym in ("grt_gather_windows_i64", "grt_pad_collate", "grt_ring_create", "grt_ring_pop"):
        assert hasattr(lib, sym), sym
