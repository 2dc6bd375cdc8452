"""Profiling helpers: a torch.profiler window over selected steps and the rocprofv3 recipe.

Kernel-level evidence on MI355X comes from ``rocprofv3 --kernel-trace --stats`` (per-kernel time),
optionally with ``--marker-trace`` to see the ROCTX phase ranges; hardware counters (MFMA
utilisation, LDS bank conflicts, HBM bytes) are collected in a SEPARATE ``--pmc`` run, never combined
with the runtime/marker trace domains.
"""
from __future__ import annotations

import contextlib
import os
import shlex
from typing import List, Optional, Sequence


def rocprof_command(program: Sequence[str], out_dir: str = "gpurun_out/prof", pmc: Optional[List[str]] = None,
                    markers: bool = False) -> str:
    """Command line for a rocprofv3 run of ``program`` (the program itself goes right after ``--``)."""
    args = ["rocprofv3"]
    if pmc:
        args += ["--pmc", *pmc]  # counters: kernel trace only, no marker/runtime domains in this run
        args += ["--kernel-trace"]
    else:
        args += ["--kernel-trace", "--stats"]
        if markers:
            args += ["--marker-trace"]
    args += ["--output-format", "csv", "-d", out_dir, "--"] + list(program)
    return " ".join(shlex.quote(a) for a in args)


@contextlib.contextmanager
def profile_steps(out_dir: Optional[str], active: bool = True, row_limit: int = 60):
    """torch.profiler (CPU + HIP activity) around a block; writes trace.json + a kernel table."""
    if not out_dir or not active:
        yield None
        return
    from torch.profiler import ProfilerActivity, profile
    prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA])
    prof.__enter__()
    try:
        yield prof
    finally:
        prof.__exit__(None, None, None)
        os.makedirs(out_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(out_dir, "trace.json"))
        with open(os.path.join(out_dir, "kernels.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=row_limit))
