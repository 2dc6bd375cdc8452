#!/usr/bin/env python3
"""Which engine carries a device -> host copy into pinned memory? Run under
``rocprofv3 --kernel-trace --memory-copy-trace``: SDMA copies appear as MEMORY_COPY_DEVICE_TO_HOST,
blit copies as ``__amd_rocclr_copyBuffer`` kernels. Variants (argv[1]): ``torch`` (copy_ into a
hipHostMalloc'ed pin_memory tensor), ``nocu`` (copy_sdma = hipMemcpyDeviceToDeviceNoCU),
``registered`` (copy_ into a hipHostRegister'ed plain host tensor), ``hsa`` (``sdma_d2h``: the HSA
runtime's async copy on an SDMA engine, stream-ordered by csrc/bindings/sdma_copy.cpp). Prints GB/s."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(mode, mib=256, reps=4):
    n = mib * 2 ** 20 // 4
    d = torch.arange(n, dtype=torch.float32, device="cuda")
    if mode == "registered":
        h = torch.empty(n, dtype=torch.float32)
        rt = torch.cuda.cudart()
        err = rt.cudaHostRegister(h.data_ptr(), n * 4, 0)
        assert int(err) == 0, err
    else:
        h = torch.empty(n, dtype=torch.float32).pin_memory()
    s = torch.cuda.Stream()
    if mode in ("nocu", "hsa"):
        from gke_ray_train_amd import _native
        C = _native.kernels()
        fn = (lambda: C.copy_sdma(h, d)) if mode == "nocu" else (lambda: C.sdma_d2h(h, d))
    else:
        fn = lambda: h.copy_(d, non_blocking=True)  # noqa: E731
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    ok = bool(torch.equal(h[:1000], d[:1000].cpu()))
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        for _ in range(reps):
            fn()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{mode}: {reps * n * 4 / dt / 1e9:.1f} GB/s exact={ok}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
