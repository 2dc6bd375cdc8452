#!/usr/bin/env python3
"""Measure the per-collective cost model t(B) = alpha + B / beta that ``parallel/comm.py`` sizes its
gradient buckets with, on the node the job will run on, and write it as JSON:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        tools/rccl_calibrate.py --out tuning/comm_calibration.json
    GRT_COMM_CALIBRATION=tuning/comm_calibration.json python bench.py --gpus 8 ...

For all-reduce, reduce-scatter and all-gather (B = bytes of the collective's full-size tensor, as the
DDP / ZeRO buckets pass it) it times ``--reps`` calls per message size (median, barrier-separated;
CUDA events on GPUs, wall clock on gloo), then fits alpha and beta by least squares over the sizes.
Rank 0 writes the JSON: per op alpha_us, beta_GBps, busbw_GBps at the largest size, and the raw
medians. With ``--device cpu`` (gloo) it runs anywhere (tests/test_planner.py).
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, reps, cuda):
    ts = []
    for _ in range(reps):
        dist.barrier()
        if cuda:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) * 1e-3)
        else:
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
    # the slowest rank's median decides (collectives finish together; launch skew shows here)
    t = torch.tensor([statistics.median(ts)], dtype=torch.float64)
    if cuda:
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def fit(sizes, times):
    """Least-squares alpha (s) and 1/beta (s/B) of t = alpha + B / beta."""
    n = len(sizes)
    mx, my = sum(sizes) / n, sum(times) / n
    sxx = sum((x - mx) ** 2 for x in sizes)
    sxy = sum((x - mx) * (y - my) for x, y in zip(sizes, times))
    inv_beta = max(sxy / sxx, 1e-15) if sxx > 0 else 1e-15
    alpha = max(my - inv_beta * mx, 0.0)
    return alpha, inv_beta


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="comm_calibration.json")
    ap.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    ap.add_argument("--min-kib", type=int, default=256)
    ap.add_argument("--max-mib", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args(argv)
    cuda = a.device == "cuda" or (a.device == "auto" and torch.cuda.is_available())
    if cuda:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group("nccl" if cuda else "gloo")
    W, R = dist.get_world_size(), dist.get_rank()
    dev = torch.device("cuda") if cuda else torch.device("cpu")
    sizes = []
    b = a.min_kib * 1024
    while b <= a.max_mib * 2 ** 20:
        sizes.append(b)
        b *= 4
    res = {"world": W, "backend": dist.get_backend(), "device": dev.type, "sizes_bytes": sizes}
    for op in ("all_reduce", "reduce_scatter", "all_gather"):
        meds = []
        for nb in sizes:
            n = max(W, nb // 2 // W * W)  # bf16 elements, divisible by W
            full = torch.ones(n, dtype=torch.bfloat16 if cuda else torch.float32, device=dev)
            part = torch.empty(n // W, dtype=full.dtype, device=dev)
            if op == "all_reduce":
                fn = lambda: dist.all_reduce(full)  # noqa: E731
            elif op == "reduce_scatter":
                if cuda:
                    fn = lambda: dist.reduce_scatter_tensor(part, full)  # noqa: E731
                else:  # gloo: no reduce-scatter; all-reduce of the full tensor is what the gloo path runs
                    fn = lambda: dist.all_reduce(full)  # noqa: E731
            else:
                if cuda:
                    fn = lambda: dist.all_gather_into_tensor(full, part)  # noqa: E731
                else:
                    fn = lambda: dist.all_gather(list(full.chunk(W)), part)  # noqa: E731
            fn()
            meds.append(_time(fn, a.reps, cuda))
        nbytes = [s - s % (2 * W) for s in sizes]
        alpha, inv_beta = fit(nbytes, meds)
        scale = 2.0 * (W - 1) / W if op == "all_reduce" else (W - 1.0) / W
        res[op] = {"alpha_us": round(alpha * 1e6, 2), "beta_GBps": round(1.0 / inv_beta / 1e9, 2),
                   "busbw_GBps_at_max": round(nbytes[-1] / meds[-1] * scale / 1e9, 2),
                   "median_s": [round(t, 7) for t in meds]}
    if R == 0:  # one entry per world size (by_world); runs at other world sizes are kept
        import os
        out = {}
        if os.path.exists(a.out):
            with open(a.out) as f:
                out = json.load(f)
            if "by_world" not in out and out.get("world") is not None:
                out = {"by_world": {str(out["world"]): out}}
        out.setdefault("by_world", {})[str(W)] = res
        out.update({k: v for k, v in res.items()})  # the latest run also at top level (older readers)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps({k: v for k, v in res.items() if k in ("world", "all_reduce", "reduce_scatter")}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
