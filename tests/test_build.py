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


@pytest.mark.parametrize("sanitizer", ["thread", "address,undefined"])
def test_runtime_under_sanitizers(tmp_path, sanitizer):
    """the native runtime (shm ring, batch gather, pad-collate) under TSan and
    ASan+UBSan — producer/consumer threads on two mappings of one ring, zero-copy and copying
    paths, close/timeout semantics, multi-threaded gathers; any report fails the run."""
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    rt = os.path.join(ROOT, "gke_ray_train_amd", "csrc", "runtime")
    exe = str(tmp_path / "stress")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", f"-fsanitize={sanitizer}", "-fno-omit-frame-pointer",
                    os.path.join(rt, "tests", "sanitize_stress.cpp"), os.path.join(rt, "shm_ring.cpp"),
                    os.path.join(rt, "batch_gather.cpp"), "-o", exe, "-lrt"], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, "20000"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "sanitize_stress ok" in r.stdout, r.stdout + r.stderr
