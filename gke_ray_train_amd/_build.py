"""In-tree native build for gke_ray_train_amd.

Builds two shared objects next to this file:

* ``_C.so``   – the gfx950 HIP kernels (``csrc/kernels/*.hip``, compiled by ``hipcc
  --offload-arch=gfx950``) plus the torch bindings (``csrc/bindings/ops.cpp``).
* ``_rt.so``  – the CPU-side native runtime (``csrc/runtime/*.cpp``): shared-memory ring
  buffer, token-window batch assembler and the store barrier helpers used by the local
  cluster runtime and the data pipeline. It does not link torch or HIP, so it loads (and is
  tested) on CPU-only hosts.

No hipify, no torch JIT cache: objects go to ``<repo>/build/`` and the ``.so`` files land in
the package directory, so they travel with the source tree to a GPU box.

Usage: ``python -m gke_ray_train_amd._build [--force] [--jobs N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = ROOT / "build" / ("native-checked" if os.environ.get("GRT_KERNEL_CHECKS", "0") == "1" else "native")
ARCH = os.environ.get("GRT_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def _torch_paths():
    import torch  # noqa: F401  (only for paths / ABI flag)
    tdir = Path(torch.__file__).resolve().parent
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return tdir, abi


def _hipcc() -> str:
    p = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    return p


def _newer(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n  " + " ".join(map(str, cmd)) + "\n" + r.stdout)
    return r.stdout


def _headers():
    return sorted((CSRC / "include").glob("*.h"))


def _check_flags():
    """``GRT_KERNEL_CHECKS=1``: compile the device-side bounds checks (GRT_DEVICE_CHECK in
    grt_common.h) into the kernels — a debugging build, slower; objects go to build/native-checked."""
    return ["-DGRT_KERNEL_CHECKS=1"] if os.environ.get("GRT_KERNEL_CHECKS", "0") == "1" else []


def build_kernels(force=False, jobs=8, verbose=False) -> Path:
    tdir, abi = _torch_paths()
    BUILD.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    inc = ["-I", str(CSRC / "include")]
    objs = []
    tasks = []
    hdrs = _headers()
    for src in sorted((CSRC / "kernels").glob("*.hip")):
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if force or _newer(obj, [src, *hdrs]):
            cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast",
                   "-munsafe-fp-atomics", *_check_flags(), *inc, "-c", str(src), "-o", str(obj)]
            tasks.append(cmd)
    pyinc = sysconfig.get_paths()["include"]
    # host sources: the pybind module (ops.cpp) and the host-side runtime pieces it binds (the
    # HSA SDMA copier), compiled by g++ against the HIP / HSA / torch headers
    for bind_src in sorted((CSRC / "bindings").glob("*.cpp")):
        bind_obj = BUILD / ("ops_bind.o" if bind_src.stem == "ops" else bind_src.stem + "_host.o")
        objs.append(bind_obj)
        if force or _newer(bind_obj, [bind_src, *hdrs]):
            cmd = ["g++", "-O2", "-fPIC", "-std=c++17", "-pthread", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                   "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                   "-I", str(tdir / "include"), "-I", str(tdir / "include" / "torch" / "csrc" / "api" / "include"),
                   "-I", pyinc, "-I", str(ROCM / "include"), *inc, "-Wno-deprecated-declarations",
                   "-c", str(bind_src), "-o", str(bind_obj)]
            tasks.append(cmd)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for out in ex.map(_run, tasks):
            if verbose and out.strip():
                print(out)
    so = PKG / "_C.so"
    if force or tasks or not so.exists():
        lib = tdir / "lib"
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(so),
               "-L", str(lib), "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
               f"-Wl,-rpath,{lib}", "-L", str(ROCM / "lib"), "-lhsa-runtime64"]
        _run(cmd)
    return so


def build_runtime(force=False, jobs=8) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    so = PKG / "_rt.so"
    if not srcs:
        return so
    deps = [*srcs, *sorted((CSRC / "runtime").glob("*.h"))]
    if force or _newer(so, deps):
        cmd = ["g++", "-O3", "-fPIC", "-shared", "-std=c++17", "-pthread", "-Wall", "-I", str(CSRC / "runtime"),
               *map(str, srcs), "-o", str(so), "-lrt"]
        _run(cmd)
    return so


def build_all(force=False, jobs=8, verbose=False):
    rt = build_runtime(force=force, jobs=jobs)
    k = build_kernels(force=force, jobs=jobs, verbose=verbose)
    return k, rt


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    k, rt = build_all(force=a.force, jobs=a.jobs, verbose=a.verbose)
    print(f"built {k}\nbuilt {rt}")


if __name__ == "__main__":
    sys.exit(main())
