#!/usr/bin/env python3
"""Host link of one MI355X as the offloaded optimizer uses it: pinned host <-> HBM copies of 512 MiB
chunks (torch ``copy_(non_blocking=True)`` on side streams, as parallel/offload.py issues them),
alone, both directions at once, and beside a GEMM loop on the compute stream (the GEMM's slowdown is
what an overlapped copy costs the step). Under ``rocprofv3 --kernel-trace --memory-copy-trace`` the
trace shows which engine each direction uses (SDMA copies vs ``__amd_rocclr_copyBuffer`` blit
kernels on the CUs). The ``*_sdma`` rows issue the same copies through the extension's
``copy_sdma`` (hipMemcpyDeviceToDeviceNoCU: a DMA engine, never a kernel).

    python tools/hostlink_bench.py [--mib 512] [--reps 4]
"""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=512)
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    n = a.mib * 2 ** 20 // 4
    dev = torch.device("cuda")
    h_src = torch.ones(n, dtype=torch.float32).pin_memory()
    h_dst = torch.empty(n, dtype=torch.float32).pin_memory()
    d_a = torch.empty(n, device=dev)
    d_b = torch.ones(n, device=dev)
    up, down = torch.cuda.Stream(), torch.cuda.Stream()
    nbytes = n * 4
    out = {"chunk_mib": a.mib}

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def h2d():
        with torch.cuda.stream(up):
            for _ in range(a.reps):
                d_a.copy_(h_src, non_blocking=True)

    def d2h():
        with torch.cuda.stream(down):
            for _ in range(a.reps):
                h_dst.copy_(d_b, non_blocking=True)

    C = None
    try:
        import os, sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from gke_ray_train_amd import _native
        C = _native.kernels()
    except Exception as e:  # noqa: BLE001
        out["copy_sdma"] = f"unavailable: {e}"

    def d2h_sdma():
        with torch.cuda.stream(down):
            for _ in range(a.reps):
                C.copy_sdma(h_dst, d_b)

    def h2d_sdma():
        with torch.cuda.stream(up):
            for _ in range(a.reps):
                C.copy_sdma(d_a, h_src)

    h2d(), d2h()  # warm
    t = timed(h2d)
    out["h2d_GBps"] = round(a.reps * nbytes / t / 1e9, 1)
    t = timed(d2h)
    out["d2h_GBps"] = round(a.reps * nbytes / t / 1e9, 1)
    t = timed(lambda: (h2d(), d2h()))
    out["duplex_total_GBps"] = round(2 * a.reps * nbytes / t / 1e9, 1)

    if C is not None:
        d_b.copy_(torch.arange(n, dtype=torch.float32, device=dev))
        h_dst.zero_()
        d2h_sdma()
        torch.cuda.synchronize()
        out["d2h_sdma_exact"] = bool(torch.equal(h_dst, d_b.cpu()))
        h_src.copy_(torch.arange(n, dtype=torch.float32) * 3)
        d_a.zero_()
        h2d_sdma()
        torch.cuda.synchronize()
        out["h2d_sdma_exact"] = bool(torch.equal(d_a.cpu(), h_src))
        d2h_sdma(), h2d_sdma()
        t = timed(d2h_sdma)
        out["d2h_sdma_GBps"] = round(a.reps * nbytes / t / 1e9, 1)
        t = timed(h2d_sdma)
        out["h2d_sdma_GBps"] = round(a.reps * nbytes / t / 1e9, 1)
        t = timed(lambda: (h2d_sdma(), d2h_sdma()))
        out["duplex_sdma_total_GBps"] = round(2 * a.reps * nbytes / t / 1e9, 1)

    x = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    y = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    z = torch.empty(8192, 8192, device=dev, dtype=torch.bfloat16)

    def gemms(k=40):
        for _ in range(k):
            torch.mm(x, y, out=z)

    gemms(5)
    tg = timed(gemms)
    out["gemm_alone_ms"] = round(tg * 1e3, 1)
    modes = [("h2d", h2d), ("d2h", d2h), ("both", lambda: (h2d(), d2h()))]
    if C is not None:
        modes += [("d2h_sdma", d2h_sdma), ("both_sdma", lambda: (h2d(), d2h_sdma()))]
    for name, fn in modes:
        def run():
            fn()
            gemms()
        torch.cuda.synchronize()
        t = timed(run)
        out[f"gemm_with_{name}_ms"] = round(t * 1e3, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
