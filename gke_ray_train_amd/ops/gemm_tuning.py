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
    rec = os.environ.get("GRT_TUNED_GEMM_RECORD_UNTUNED")  # path: log every GEMM shape the table misses
    if rec:
        os.environ["PYTORCH_TUNABLEOP_UNTUNED_FILENAME"] = rec
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(bool(rec))
    ok = bool(tun.read_file(str(p)))
    _enabled = ok
    return ok


def tuned_gemms_enabled() -> bool:
    return _enabled


_DT = {"BFloat16": torch.bfloat16, "Half": torch.float16, "float": torch.float32}
_TAIL = 1 << 16  # poisoned elements past each operand's last element


def _poisoned(rows: int, ld: int, cols: int, dtype, dev):
    """Row-major [rows, ld] buffer (+ tail); logical region [:, :cols] random, everything else NaN."""
    flat = torch.full((rows * ld + _TAIL,), float("nan"), dtype=dtype, device=dev)
    buf = flat[:rows * ld].view(rows, ld)
    buf[:, :cols] = torch.randn(rows, cols, device=dev).to(dtype)
    return buf[:, :cols]


def check_gemm_row(op_sig: str, params: str, dev=None) -> tuple:
    """Run one table row's column-major BLAS problem (``GemmTunableOp_<dtype>_<TA><TB>``,
    ``<ta><tb>_m_n_k_ld_lda_ldb_ldc``) as ``C += op(A) op(B)`` with the table's solution, on operands
    whose padding (between the logical columns and the leading dimension) and tail hold NaN, and
    compare with an fp32 reference. A solution that reads outside its operands turns the result
    NaN; one that computes the wrong product shows a large error. Returns (finite, rel_err)."""
    dev = dev or torch.device("cuda", torch.cuda.current_device())
    dtype = _DT[op_sig.split("_")[1]]
    ta, tb = params[0], params[1]
    f = params.split("_")
    m, n, k, lda, ldb, ldc = (int(f[i]) for i in (1, 2, 3, 5, 6, 7))
    a = _poisoned(k, lda, m, dtype, dev).t() if ta == "n" else _poisoned(m, lda, k, dtype, dev)
    b = _poisoned(n, ldb, k, dtype, dev).t() if tb == "n" else _poisoned(k, ldb, n, dtype, dev)
    c = _poisoned(n, ldc, m, dtype, dev).t()  # [m, n], column-major with ldc
    ref = c.float() + a.float() @ b.float()
    c.addmm_(a, b)
    torch.cuda.synchronize()
    finite = bool(torch.isfinite(c).all().item())
    rel = float(((c.float() - ref).norm() / ref.norm()).item()) if finite else float("nan")
    return finite, rel


def check_tuned_table(path: str | os.PathLike | None = None, tol: float = 2e-2) -> list:
    """Validate every GEMM row of a TunableOp results file on this GPU (see ``check_gemm_row``);
    loads the file (tuning off). Returns [(line, finite, rel_err, ok)] for every GEMM row."""
    p = str(path or RESULTS)
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    tun.read_file(p)
    out = []
    for ln in open(p).read().splitlines():
        parts = ln.split(",")
        if not parts[0].startswith("GemmTunableOp"):
            continue
        finite, rel = check_gemm_row(parts[0], parts[1])
        out.append((ln, finite, rel, finite and rel < tol))
    return out
