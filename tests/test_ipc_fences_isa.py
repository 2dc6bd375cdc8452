"""The IPC collectives' cross-GPU memory ordering, checked in the gfx950 ISA on the CPU.

The one-GPU tests (tests/test_ipc_gpu.py) map every peer on one device, where a missing
system-scope fence would still pass; here the compiled kernels of csrc/kernels/ipc_comm.hip are
inspected instead: every cross-rank flag store is a SYSTEM-scope store (``sc0 sc1``) preceded by a
system-scope L2 write-back (the release of the data it publishes), every flag poll is a
system-scope load, and each wait ends in a system-scope invalidate (the acquire) before the
peer's data is read."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gke_ray_train_amd", "csrc", "kernels", "ipc_comm.hip")


@pytest.fixture(scope="module")
def isa(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "ipc.s"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I",
                    os.path.join(ROOT, "gke_ray_train_amd", "csrc", "include"), "--cuda-device-only", "-S",
                    "-o", str(out), SRC], check=True, capture_output=True, timeout=300)
    return out.read_text()


def _kernels(isa):
    """{kernel symbol: its instruction lines} for the ipc kernels."""
    out, cur = {}, None
    for line in isa.splitlines():
        m = re.match(r"^(_Z\S*ipc\S*):", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):  # a kernel can hold several s_endpgm (early returns)
                cur = None
                continue
            t = line.strip()
            if t and not t.startswith((";", ".")):
                out[cur].append(t)
    return out


def test_flag_stores_are_released_at_system_scope(isa):
    ks = _kernels(isa)
    assert ks, "no ipc kernels found in the ISA"
    n_checked = 0
    for name, ins in ks.items():
        stores = [i for i, t in enumerate(ins) if t.startswith("global_store_dword ") and t.endswith("sc0 sc1")]
        for i in stores:
            # the release: a system-scope L2 write-back since the previous flag store
            prev = max([j for j in stores if j < i], default=-1)
            assert any(t.startswith("buffer_wbl2") and "sc0 sc1" in t for t in ins[prev + 1:i]), \
                f"{name}: flag store at {i} without a system-scope write-back before it"
            n_checked += 1
    assert n_checked >= 3, n_checked


def test_flag_polls_acquire_at_system_scope(isa):
    for name, ins in _kernels(isa).items():
        polls = [i for i, t in enumerate(ins) if t.startswith("global_load_dword ") and t.endswith("sc0 sc1")]
        if not polls:
            continue
        # after the last poll of a wait, a system-scope invalidate precedes any further peer read
        assert any(t.startswith("buffer_inv") and "sc0 sc1" in t for t in ins[polls[0]:]), \
            f"{name}: system-scope poll without a system-scope invalidate (acquire) after it"
