"""Per-step training metrics: throughput, MFU, phase breakdown, HBM use; JSONL / CSV / Prometheus.

Reference observability is print() on rank 0 plus Ray's result.json / progress.csv and the HF
Trainer's end-of-run ``train_samples_per_second`` (reference ray-jobs/fine_tune_llama_ray.py:334,
SURVEY §5.5) — it never measures tokens/s, MFU, or where step time goes. ``StepMeter`` does, without
stalling the GPU pipeline: phases are bracketed by HIP events recorded on the current stream, and
event times are only resolved when a step is logged (``log_every``), so no host synchronisation is
added to unlogged steps.

    meter = StepMeter(tokens_per_step=B*S*world, flops_per_token=cfg.flops_per_token(S), n_gpus=world,
                      jsonl="run/metrics.jsonl", rank=rank)
    for step in ...:
        with meter.step(step):
            with meter.phase("forward"): ...
            with meter.phase("backward"): ...
            with meter.phase("grad_sync"): ...
            with meter.phase("optimizer"): ...
        meter.log(step, loss=loss)           # rank 0 writes one JSON line every log_every steps
"""
from __future__ import annotations

import contextlib
import csv
import json
import os
import time
from collections import defaultdict
from typing import Dict, List, Optional

import torch

from . import roctx

MI355X_PEAK_BF16_DENSE = 2.5e15  # FLOP/s per GPU, dense (no 2:1 sparsity)
MI355X_PEAK_FP32_MFMA = 1.57e14


class _Timer:
    """Wall-clock on CPU tensors, HIP events on GPU (resolved lazily)."""

    def __init__(self, device):
        self.cuda = device is not None and torch.device(device).type == "cuda"
        self.a = self.b = None

    def start(self):
        if self.cuda:
            self.a = torch.cuda.Event(enable_timing=True)
            self.a.record()
        else:
            self.a = time.perf_counter()

    def stop(self):
        if self.cuda:
            self.b = torch.cuda.Event(enable_timing=True)
            self.b.record()
        else:
            self.b = time.perf_counter()

    def ms(self) -> float:
        if self.a is None or self.b is None:
            return 0.0
        if self.cuda:
            self.b.synchronize()
            return float(self.a.elapsed_time(self.b))
        return (self.b - self.a) * 1000.0


class StepMeter:
    def __init__(self, tokens_per_step: int, flops_per_token: float = 0.0, n_gpus: int = 1,
                 samples_per_step: Optional[int] = None, peak_flops: float = MI355X_PEAK_BF16_DENSE,
                 jsonl: Optional[str] = None, csv_path: Optional[str] = None, rank: int = 0, log_every: int = 1,
                 device=None, prometheus=None, annotate: bool = True):
        self.tokens_per_step = tokens_per_step
        self.samples_per_step = samples_per_step
        self.flops_per_token = flops_per_token
        self.n_gpus = max(1, n_gpus)
        self.peak = peak_flops
        self.rank = rank
        self.log_every = max(1, log_every)
        self.device = torch.device(device) if device is not None else (torch.device("cuda", torch.cuda.current_device())
                                                         if torch.cuda.device_count() and torch.cuda.is_initialized()
                                                         else torch.device("cpu"))
        self.jsonl = jsonl if rank == 0 else None
        self.csv_path = csv_path if rank == 0 else None
        self.prom = prometheus if rank == 0 else None
        self.annotate = annotate
        self._step_timer: Optional[_Timer] = None
        self._phases: Dict[str, List[_Timer]] = defaultdict(list)
        self._wall0 = None
        self.history: List[dict] = []
        self._t_start = time.perf_counter()
        self._steps = 0
        self._tokens = 0
        if self.jsonl:
            os.makedirs(os.path.dirname(os.path.abspath(self.jsonl)), exist_ok=True)

    @contextlib.contextmanager
    def step(self, idx: int):
        self._phases.clear()  # phases recorded outside a step (e.g. warmup) do not count
        t = _Timer(self.device)
        if self.annotate:
            roctx.push(f"step {idx}")
        t.start()
        self._wall0 = time.perf_counter()
        try:
            yield
        finally:
            t.stop()
            if self.annotate:
                roctx.pop()
            self._step_timer = t
            self._wall_ms = (time.perf_counter() - self._wall0) * 1000.0
            self._steps += 1
            self._tokens += self.tokens_per_step

    @contextlib.contextmanager
    def phase(self, name: str):
        t = _Timer(self.device)
        if self.annotate:
            roctx.push(name)
        t.start()
        try:
            yield
        finally:
            t.stop()
            if self.annotate:
                roctx.pop()
            self._phases[name].append(t)

    def memory(self) -> dict:
        if self.device.type != "cuda":
            return {}
        free, total = torch.cuda.mem_get_info(self.device)
        return {"hbm_allocated_gb": torch.cuda.memory_allocated(self.device) / 2 ** 30,
                "hbm_peak_gb": torch.cuda.max_memory_allocated(self.device) / 2 ** 30,
                "hbm_reserved_gb": torch.cuda.memory_reserved(self.device) / 2 ** 30,
                "hbm_used_gb": (total - free) / 2 ** 30, "hbm_total_gb": total / 2 ** 30}

    def log(self, step: int, loss=None, lr=None, force: bool = False, **extra) -> Optional[dict]:
        """Resolve this step's timings (syncs on the step-end event) and emit one record."""
        if not force and step % self.log_every != 0:
            self._phases.clear()
            return None
        ms = self._step_timer.ms() if self._step_timer is not None else 0.0
        ms = ms or getattr(self, "_wall_ms", 0.0)
        rec = {"step": step, "time": time.time(), "step_ms": round(ms, 3)}
        if ms > 0:
            tps = self.tokens_per_step / (ms / 1000.0)
            rec["tokens_per_sec"] = round(tps, 1)
            rec["tokens_per_sec_per_gpu"] = round(tps / self.n_gpus, 1)
            if self.samples_per_step:
                rec["samples_per_sec"] = round(self.samples_per_step / (ms / 1000.0), 3)
            if self.flops_per_token:
                rec["mfu"] = round(tps / self.n_gpus * self.flops_per_token / self.peak, 4)
        for name, timers in self._phases.items():
            rec[f"{name}_ms"] = round(sum(t.ms() for t in timers), 3)
        self._phases.clear()
        if loss is not None:
            rec["loss"] = float(loss.item() if isinstance(loss, torch.Tensor) else loss)
        if lr is not None:
            rec["learning_rate"] = float(lr)
        rec.update(self.memory())
        rec.update(extra)
        self.history.append(rec)
        self._emit(rec)
        return rec

    def _emit(self, rec):
        if self.jsonl:
            with open(self.jsonl, "a") as f:
                f.write(json.dumps(rec) + "\n")
        if self.csv_path:
            new = not os.path.exists(self.csv_path)
            with open(self.csv_path, "a", newline="") as f:
                w = csv.DictWriter(f, fieldnames=list(rec.keys()), extrasaction="ignore")
                if new:
                    w.writeheader()
                w.writerow(rec)
        if self.prom is not None:
            self.prom.update(rec)

    def summary(self) -> dict:
        """HF-Trainer-style end metrics (train_runtime, train_*_per_second, total_flos)."""
        rt = time.perf_counter() - self._t_start
        out = {"train_runtime": round(rt, 4), "train_steps_per_second": round(self._steps / rt, 3) if rt else 0.0,
               "train_tokens_per_second": round(self._tokens / rt, 1) if rt else 0.0,
               "total_flos": float(self._tokens * self.flops_per_token)}
        if self.samples_per_step:
            out["train_samples_per_second"] = round(self._steps * self.samples_per_step / rt, 3) if rt else 0.0
        return out


class PrometheusExporter:
    """Gauges for the latest step record, served at ``http://<host>:<port>/metrics`` (the Ray
    dashboard / GKE managed-Prometheus role of the reference, a3-mega/gke-ray-cluster-setup.sh:21-22)."""

    KEYS = ("step", "step_ms", "tokens_per_sec", "samples_per_sec", "mfu", "loss", "learning_rate",
            "hbm_allocated_gb", "hbm_peak_gb", "forward_ms", "backward_ms", "grad_sync_ms", "optimizer_ms")

    def __init__(self, port: int = 0, prefix: str = "grt_train", registry=None, start_server: bool = True):
        from prometheus_client import CollectorRegistry, Gauge, start_http_server
        self.registry = registry or CollectorRegistry()
        self.gauges = {k: Gauge(f"{prefix}_{k}", k.replace("_", " "), registry=self.registry) for k in self.KEYS}
        self.server = None
        if start_server:
            self.server = start_http_server(port, addr="127.0.0.1", registry=self.registry)

    def update(self, rec: dict):
        for k, g in self.gauges.items():
            if k in rec and isinstance(rec[k], (int, float)):
                g.set(rec[k])

    def text(self) -> str:
        from prometheus_client import generate_latest
        return generate_latest(self.registry).decode()
