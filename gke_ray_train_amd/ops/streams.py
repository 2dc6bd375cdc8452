"""Side streams restricted to a subset of the MI355X's CUs.

A side stream that runs HBM-bound work (the overlapped AdamW, ``parallel/overlap.py``) beside the
compute stream's GEMMs otherwise dispatches its workgroups onto EVERY CU: its waves take the wave
slots, issue cycles, LDS and L2 of the CUs the GEMM tiles need, and the measured forward GEMMs
ran at 0.6-0.7 PF instead of ~1.5 PF while the update was in flight
(``profiles/r2_opt_cu_mask.md``). A CU mask (``hipExtStreamCreateWithCUMask``) confines the side
stream to ``n`` CUs: the GEMMs keep the rest at full speed and lose at most n/256 of the chip,
and n CUs with many loads in flight still stream HBM at a useful rate.

Patterns (which CUs, given HIP's linear CU numbering):
* ``spread``: every (256/n)-th CU;
* ``low``: the first n CUs.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch

_cache: Dict[Tuple[int, int, str], "torch.cuda.ExternalStream"] = {}


def cu_mask_words(n_cus: int, total: int, pattern: str = "spread") -> List[int]:
    """Bit mask (32 CUs per word) selecting ``n_cus`` of ``total`` CUs."""
    if not 0 < n_cus <= total:
        raise ValueError(f"n_cus must be in 1..{total}, got {n_cus}")
    if pattern == "spread":
        step = total / n_cus
        bits = sorted({int(i * step) for i in range(n_cus)})
    elif pattern == "low":
        bits = list(range(n_cus))
    else:
        raise ValueError(f"unknown CU mask pattern {pattern!r}")
    words = [0] * ((total + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    return words


def cu_masked_stream(n_cus: int, device=None, pattern: str = "spread") -> "torch.cuda.ExternalStream":
    """A (cached, process-lifetime) HIP stream on ``device`` limited to ``n_cus`` CUs."""
    d = torch.device("cuda") if device is None else torch.device(device)
    dev = torch.device("cuda", torch.cuda.current_device() if d.index is None else d.index)
    key = (dev.index, int(n_cus), pattern)
    s = _cache.get(key)
    if s is None:
        from .. import _native
        total = torch.cuda.get_device_properties(dev).multi_processor_count
        words = cu_mask_words(min(int(n_cus), total), total, pattern)
        ptr = _native.kernels().cu_masked_stream(words, dev.index)
        s = torch.cuda.ExternalStream(ptr, device=dev)
        _cache[key] = s
    return s
