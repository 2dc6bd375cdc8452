"""Observability: ROCTX ranges, per-step metrics (tokens/s, MFU, phase breakdown, HBM), JSONL/CSV
and Prometheus export, and a torch.profiler helper (SURVEY §5.1 / §5.5 targets)."""
from . import roctx
from .metrics import MI355X_PEAK_BF16_DENSE, PrometheusExporter, StepMeter
from .profiler import profile_steps, rocprof_command

__all__ = ["roctx", "StepMeter", "PrometheusExporter", "MI355X_PEAK_BF16_DENSE", "profile_steps", "rocprof_command"]
