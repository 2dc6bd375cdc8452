"""Run / scaling / checkpoint / failure configs with Ray Train's names and defaults.

Reference call sites: ScalingConfig(num_workers, use_gpu, resources_per_worker)
(ray-jobs/pytorch_llm_ray.py:346-350, fine_tune_llama_ray.py:445-449), RunConfig(name,
storage_path, checkpoint_config) and CheckpointConfig(num_to_keep=1,
checkpoint_score_attribute="loss", checkpoint_score_order="min") (pytorch_llm_ray.py:352-360).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class ScalingConfig:
    num_workers: int = 1
    use_gpu: bool = False
    resources_per_worker: Optional[Dict[str, float]] = None
    placement_strategy: str = "PACK"
    trainer_resources: Optional[Dict[str, float]] = None

    @property
    def gpus_per_worker(self) -> float:
        if not self.use_gpu:
            return 0.0
        return float((self.resources_per_worker or {}).get("GPU", 1.0))

    @property
    def cpus_per_worker(self) -> float:
        return float((self.resources_per_worker or {}).get("CPU", 0.0 if self.use_gpu else 1.0))


@dataclass
class CheckpointConfig:
    num_to_keep: Optional[int] = None
    checkpoint_score_attribute: Optional[str] = None
    checkpoint_score_order: str = "max"
    checkpoint_frequency: int = 0
    checkpoint_at_end: Optional[bool] = None

    def __post_init__(self):
        if self.checkpoint_score_order not in ("max", "min"):
            raise ValueError("checkpoint_score_order must be 'max' or 'min'")
        if self.num_to_keep is not None and self.num_to_keep <= 0:
            raise ValueError("num_to_keep must be a positive integer or None")


@dataclass
class FailureConfig:
    max_failures: int = 0
    fail_fast: bool = False


@dataclass
class RunConfig:
    name: Optional[str] = None
    storage_path: Optional[str] = None
    checkpoint_config: Optional[CheckpointConfig] = None
    failure_config: Optional[FailureConfig] = None
    verbose: int = 1
    log_to_file: bool = False
    stop: Optional[Dict[str, Any]] = None
    callbacks: Optional[list] = None

    def resolved_storage(self) -> str:
        return os.path.expanduser(self.storage_path or os.environ.get("GRT_STORAGE_PATH", "~/ray_results"))
