"""Experiment / trial directory layout, result files and checkpoint retention.

Reproduces the on-disk layout of Ray Train V1 that the reference relies on:
``<storage_path>/<name>/`` holding the experiment state and one trial directory
``TorchTrainer_<id>_00000_0_<date>/`` with ``params.json``, ``result.json`` (one JSON object per
report), ``progress.csv`` and ``checkpoint_%06d/`` directories, pruned to ``num_to_keep`` by
``checkpoint_score_attribute`` / ``checkpoint_score_order`` (reference
ray-jobs/pytorch_llm_ray.py:352-360). The most recent checkpoint is never pruned (it is the
restart point for FailureConfig).
"""
from __future__ import annotations

import csv
import datetime as _dt
import json
import os
import shutil
import socket
import time
import uuid
from typing import Dict, List, Optional, Tuple

from ._checkpoint import Checkpoint
from ._config import CheckpointConfig, RunConfig


def _json_safe(v):
    try:
        json.dumps(v)
        return v
    except TypeError:
        if isinstance(v, dict):
            return {str(k): _json_safe(x) for k, x in v.items()}
        if isinstance(v, (list, tuple)):
            return [_json_safe(x) for x in v]
        return repr(v)


class RunStorage:
    def __init__(self, run_config: RunConfig, trainer_name: str, config: Optional[dict]):
        self.run_config = run_config
        self.ckpt_cfg = run_config.checkpoint_config or CheckpointConfig()
        date = _dt.datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
        self.storage_path = run_config.resolved_storage()
        self.experiment_name = run_config.name or f"{trainer_name}_{date}"
        self.exp_dir = os.path.join(self.storage_path, self.experiment_name)
        self.trial_id = uuid.uuid4().hex[:5]
        self.trial_name = f"{trainer_name}_{self.trial_id}_00000"
        self.trial_dir = os.path.join(self.exp_dir, f"{self.trial_name}_0_{date}")
        os.makedirs(self.trial_dir, exist_ok=True)
        self.config = _json_safe(config or {})
        with open(os.path.join(self.trial_dir, "params.json"), "w") as f:
            json.dump(self.config, f, indent=2, sort_keys=True)
        with open(os.path.join(self.exp_dir, f"experiment_state-{date}.json"), "w") as f:
            json.dump({"experiment_name": self.experiment_name, "trial_dirs": [self.trial_dir],
                       "trainer": trainer_name, "start_time": time.time()}, f, indent=2)
        self.iteration = 0
        self.ckpt_index = 0
        self.checkpoints: List[Tuple[Checkpoint, Dict]] = []
        self.latest_checkpoint: Optional[Checkpoint] = None
        self.last_metrics: Optional[Dict] = None
        self.t_start = time.time()
        self.t_last = self.t_start
        self._csv_cols: Optional[List[str]] = None
        self._rows: List[Dict] = []

    # ----------------------------------------------------------------- reports
    def record(self, metrics: Dict, ckpt_dirs: List[str]) -> Optional[str]:
        now = time.time()
        self.iteration += 1
        m = dict(metrics)
        persisted = None
        if ckpt_dirs:
            dst = os.path.join(self.trial_dir, f"checkpoint_{self.ckpt_index:06d}")
            os.makedirs(dst, exist_ok=True)
            for d in ckpt_dirs:  # Ray merges every rank's checkpoint files into one directory
                shutil.copytree(d, dst, dirs_exist_ok=True)
                shutil.rmtree(d, ignore_errors=True)
            self.ckpt_index += 1
            persisted = dst
            ck = Checkpoint(dst)
            self.latest_checkpoint = ck
            m["checkpoint_dir_name"] = os.path.basename(dst)
            self.checkpoints.append((ck, dict(metrics)))
            self._prune()
        else:
            m.setdefault("checkpoint_dir_name", None)
        m.update({
            "timestamp": int(now), "time_this_iter_s": now - self.t_last, "time_total_s": now - self.t_start,
            "training_iteration": self.iteration, "done": False, "trial_id": self.trial_id,
            "date": _dt.datetime.now().strftime("%Y-%m-%d_%H-%M-%S"), "hostname": socket.gethostname(),
            "node_ip": "127.0.0.1", "pid": os.getpid(),
        })
        self.t_last = now
        self.last_metrics = m
        row = dict(m)
        row["config"] = self.config
        with open(os.path.join(self.trial_dir, "result.json"), "a") as f:
            f.write(json.dumps(_json_safe(row)) + "\n")
        self._write_csv(m)
        return persisted

    def _write_csv(self, m):
        flat = {k: v for k, v in m.items() if not isinstance(v, (dict, list))}
        self._rows.append(flat)
        cols = list(self._csv_cols or [])
        new = [k for k in flat if k not in cols]
        path = os.path.join(self.trial_dir, "progress.csv")
        if new or self._csv_cols is None:
            cols += new
            self._csv_cols = cols
            with open(path, "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=cols)
                w.writeheader()
                for r in self._rows:
                    w.writerow(r)
        else:
            with open(path, "a", newline="") as f:
                csv.DictWriter(f, fieldnames=cols).writerow(flat)

    def _prune(self):
        k = self.ckpt_cfg.num_to_keep
        if k is None or len(self.checkpoints) <= k:
            return
        attr = self.ckpt_cfg.checkpoint_score_attribute
        latest = self.checkpoints[-1][0]
        if attr is None:
            keep = self.checkpoints[-k:]
        else:
            rev = self.ckpt_cfg.checkpoint_score_order == "max"
            scored = [c for c in self.checkpoints if attr in c[1]]
            unscored = [c for c in self.checkpoints if attr not in c[1]]
            scored.sort(key=lambda c: c[1][attr], reverse=rev)
            keep = (scored + unscored)[:k]
        keep_paths = {c[0].path for c in keep} | {latest.path}
        for c in list(self.checkpoints):
            if c[0].path not in keep_paths:
                shutil.rmtree(c[0].path, ignore_errors=True)
                self.checkpoints.remove(c)

    def best_checkpoints(self):
        return list(self.checkpoints)

    def finish(self):
        if self.last_metrics is not None:
            path = os.path.join(self.trial_dir, "result.json")
            with open(path) as f:
                lines = f.read().splitlines()
            if lines:
                last = json.loads(lines[-1])
                last["done"] = True
                lines[-1] = json.dumps(last)
                with open(path, "w") as f:
                    f.write("\n".join(lines) + "\n")
