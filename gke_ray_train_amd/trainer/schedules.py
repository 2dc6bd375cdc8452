"""Learning-rate schedules (HF ``get_scheduler`` names + the reference's warmup-cosine-with-floor).

Reference: BasicLLM's LambdaLR warmup + cosine to ``min_lr_ratio`` (ray-jobs/pytorch_llm_ray.py:
239-258) and SFT's ``lr_scheduler_type="cosine"`` with ``warmup_ratio=0.03``
(fine_tune_config.json:18,20).
"""
from __future__ import annotations

import math

import torch
from torch.optim.lr_scheduler import LambdaLR


def warmup_cosine_floor(total_steps: int, warmup_steps: int, min_lr_ratio: float = 0.0):
    decay = max(1, total_steps - warmup_steps)

    def f(step):
        if step < warmup_steps:
            return step / max(1, warmup_steps)
        if step < total_steps:
            p = (step - warmup_steps) / decay
            return min_lr_ratio + (1 - min_lr_ratio) * 0.5 * (1 + math.cos(math.pi * p))
        return min_lr_ratio
    return f


def get_scheduler(name: str, optimizer, num_warmup_steps: int, num_training_steps: int, min_lr_ratio: float = 0.0,
                  num_cycles: float = 0.5):
    name = (name or "linear").lower()
    W, T = num_warmup_steps, max(1, num_training_steps)
    if name == "constant":
        return LambdaLR(optimizer, lambda s: 1.0)
    if name == "constant_with_warmup":
        return LambdaLR(optimizer, lambda s: min(1.0, s / max(1, W)))
    if name == "linear":
        return LambdaLR(optimizer, lambda s: s / max(1, W) if s < W else max(0.0, (T - s) / max(1, T - W)))
    if name == "cosine":
        def f(s):
            if s < W:
                return s / max(1, W)
            p = (s - W) / max(1, T - W)
            return max(0.0, 0.5 * (1.0 + math.cos(math.pi * num_cycles * 2.0 * p)))
        return LambdaLR(optimizer, f)
    if name in ("cosine_with_min_lr", "warmup_cosine_floor"):
        return LambdaLR(optimizer, warmup_cosine_floor(T, W, min_lr_ratio))
    if name == "polynomial":
        return LambdaLR(optimizer, lambda s: s / max(1, W) if s < W else max(0.0, (1 - (s - W) / max(1, T - W))) ** 1.0)
    raise ValueError(f"unknown lr_scheduler_type {name!r}")
