"""Offline-tuned GEMM selection for the library GEMMs (forward / input-gradient projections).

The weight-gradient GEMMs run on the framework's own MFMA kernel (csrc/kernels/gemm.hip); the
forward and dX GEMMs go through torch -> hipBLASLt / rocBLAS. Their default heuristic pick is not
the fastest solution on every Llama projection shape (profiles/r1_microbench_gemm_tunableop.jsonl:
-13 % on the QKV forward and dX, -14 % on gate_up forward). ``tools/tune_gemms.py`` benchmarks the
candidate solutions ONCE per (shape, layout) on an MI355X with torch's TunableOp and stores the
winners in ``tuning/tunableop_mi355x.csv`` (validated against the torch / HIP / hipBLASLt / rocBLAS
versions and gfx950); ``enable_tuned_gemms()`` makes every later GEMM of a listed shape use the
stored solution, with tuning itself OFF (no benchmarking inside a training step). Shapes not in the
file keep the library default. ``GRT_TUNED_GEMM=0`` disables it.
"""
from __future__ import annotations

import os
from pathlib import Path

import torch

RESULTS = Path(__file__).resolve().parent.parent / "tuning" / "tunableop_mi355x.csv"
_enabled = False


def enable_tuned_gemms(path: str | os.PathLike | None = None) -> bool:
    """Use the stored TunableOp results (no online tuning). Returns True if a results file was loaded."""
    global _enabled
    if os.environ.get("GRT_TUNED_GEMM", "1") == "0" or not torch.cuda.is_available():
        return False
    p = Path(path or os.environ.get("GRT_TUNED_GEMM_FILE") or RESULTS)
    if not p.exists():
        return False
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    ok = bool(tun.read_file(str(p)))
    _enabled = ok
    return ok


def tuned_gemms_enabled() -> bool:
    return _enabled
