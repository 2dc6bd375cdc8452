"""Directory-backed Checkpoint handle (``Checkpoint.from_directory`` at
reference ray-jobs/pytorch_llm_ray.py:305)."""
from __future__ import annotations

import contextlib
import json
import os
import shutil
import tempfile
from typing import Any, Dict


class Checkpoint:
    _META = ".metadata.json"

    def __init__(self, path: str, filesystem=None):
        self.path = os.path.abspath(os.fspath(path))
        self.filesystem = filesystem

    @classmethod
    def from_directory(cls, path) -> "Checkpoint":
        return cls(path)

    @classmethod
    def from_dict(cls, data: Dict[str, Any]) -> "Checkpoint":
        import torch
        d = tempfile.mkdtemp(prefix="grt_ckpt_")
        torch.save(data, os.path.join(d, "dict_checkpoint.pt"))
        return cls(d)

    def to_dict(self) -> Dict[str, Any]:
        import torch
        return torch.load(os.path.join(self.path, "dict_checkpoint.pt"), weights_only=False)

    def to_directory(self, path=None) -> str:
        dst = path or tempfile.mkdtemp(prefix="grt_ckpt_")
        os.makedirs(dst, exist_ok=True)
        shutil.copytree(self.path, dst, dirs_exist_ok=True)
        return dst

    @contextlib.contextmanager
    def as_directory(self):
        yield self.path

    def get_metadata(self) -> Dict[str, Any]:
        p = os.path.join(self.path, self._META)
        if os.path.exists(p):
            with open(p) as f:
                return json.load(f)
        return {}

    def set_metadata(self, metadata: Dict[str, Any]):
        with open(os.path.join(self.path, self._META), "w") as f:
            json.dump(metadata, f)

    def update_metadata(self, metadata: Dict[str, Any]):
        m = self.get_metadata()
        m.update(metadata)
        self.set_metadata(m)

    def __repr__(self):
        return f"Checkpoint(filesystem=local, path={self.path})"

    def __eq__(self, o):
        return isinstance(o, Checkpoint) and o.path == self.path

    def __hash__(self):
        return hash(self.path)
