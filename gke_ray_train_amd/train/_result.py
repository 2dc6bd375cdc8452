"""``Result`` of ``TorchTrainer.fit()`` (reference reads ``result.metrics``,
ray-jobs/fine_tune_llama_ray.py:459-463)."""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

from ._checkpoint import Checkpoint


@dataclass
class Result:
    metrics: Dict[str, Any]
    checkpoint: Optional[Checkpoint]
    path: str
    error: Optional[BaseException] = None
    best_checkpoints: List[Tuple[Checkpoint, Dict[str, Any]]] = field(default_factory=list)
    storage: Any = None

    @property
    def metrics_dataframe(self):
        import pandas as pd
        p = os.path.join(self.path, "result.json")
        if not os.path.exists(p):
            return pd.DataFrame()
        with open(p) as f:
            rows = [json.loads(l) for l in f if l.strip()]
        for r in rows:
            r.pop("config", None)
        return pd.DataFrame(rows)

    @property
    def config(self):
        p = os.path.join(self.path, "params.json")
        with open(p) as f:
            return json.load(f)

    def get_best_checkpoint(self, metric: str, mode: str = "max") -> Optional[Checkpoint]:
        c = [x for x in self.best_checkpoints if metric in x[1]]
        if not c:
            return None
        c.sort(key=lambda x: x[1][metric], reverse=(mode == "max"))
        return c[0][0]

    @classmethod
    def from_path(cls, path: str) -> "Result":
        rows = []
        p = os.path.join(path, "result.json")
        if os.path.exists(p):
            with open(p) as f:
                rows = [json.loads(l) for l in f if l.strip()]
        ckpts = sorted(d for d in os.listdir(path) if d.startswith("checkpoint_"))
        latest = Checkpoint(os.path.join(path, ckpts[-1])) if ckpts else None
        return cls(metrics=rows[-1] if rows else {}, checkpoint=latest, path=path)
