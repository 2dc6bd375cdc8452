"""``train.torch`` utilities: device, model / data-loader preparation, TorchConfig, TorchTrainer.

Reference: ``train.torch.get_device()`` (ray-jobs/pytorch_llm_ray.py:128), ``prepare_model``
(:230), ``prepare_data_loader`` (:216), ``TorchConfig(backend="nccl")`` (:362-364).
Differences by design:
* ``prepare_model`` ALWAYS wraps (also at world size 1), so the reference's
  ``model.module.state_dict()`` works on one GPU; the wrapper is the flat-buffer RCCL DDP of
  ``parallel/ddp.py`` (or FSDP with ``parallel_strategy="fsdp"``);
* ``prepare_data_loader`` re-shards with a DistributedSampler (shuffle preserved) and moves
  batches to the GPU from pinned memory on a side stream, one batch ahead.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist
from torch.utils.data import DataLoader, DistributedSampler, RandomSampler

from ._session import get_context
from ._trainer import TorchTrainer  # noqa: F401  (ray.train.torch.TorchTrainer)


@dataclass
class TorchConfig:
    backend: Optional[str] = None
    init_method: str = "env"
    timeout_s: int = 1800


def get_device() -> torch.device:
    if torch.cuda.is_available():
        lr = int(os.environ.get("LOCAL_RANK", get_context().get_local_rank()))
        return torch.device("cuda", lr % max(1, torch.cuda.device_count()))
    return torch.device("cpu")


def get_devices():
    return [get_device()]


def enable_reproducibility(seed: int = 0):
    import random
    import numpy as np
    torch.manual_seed(seed)
    random.seed(seed)
    np.random.seed(seed)


def prepare_model(model: torch.nn.Module, move_to_device=True, parallel_strategy: str = "ddp",
                  parallel_strategy_kwargs: Optional[dict] = None, **_):
    dev = get_device()
    if move_to_device:
        model = model.to(dev)
    kw = dict(parallel_strategy_kwargs or {})
    if parallel_strategy == "fsdp":
        from ..parallel.fsdp import FullyShardedDataParallel
        return FullyShardedDataParallel(model, **kw)
    if parallel_strategy in (None, "none"):
        return model
    from ..parallel.ddp import DistributedDataParallel
    return DistributedDataParallel(model, **kw)


class _DeviceLoader:
    """Iterates a DataLoader and moves each batch to ``device`` one batch ahead on a side stream."""

    def __init__(self, loader: DataLoader, device: torch.device):
        self.loader = loader
        self.device = device
        self.sampler = loader.sampler
        self.batch_size = loader.batch_size
        self.dataset = loader.dataset

    def __len__(self):
        return len(self.loader)

    def _move(self, b):
        if isinstance(b, torch.Tensor):
            if self.device.type == "cuda":
                if not b.is_pinned():
                    b = b.pin_memory()
                return b.to(self.device, non_blocking=True)
            return b.to(self.device)
        if isinstance(b, (list, tuple)):
            return type(b)(self._move(x) for x in b)
        if isinstance(b, dict):
            return {k: self._move(v) for k, v in b.items()}
        return b

    def __iter__(self):
        it = iter(self.loader)
        if self.device.type != "cuda":
            for b in it:
                yield self._move(b)
            return
        stream = torch.cuda.Stream(self.device)
        nxt = None
        try:
            first = next(it)
        except StopIteration:
            return
        with torch.cuda.stream(stream):
            nxt = self._move(first)
        compute = torch.cuda.current_stream(self.device)
        for b in it:
            compute.wait_stream(stream)
            cur = nxt
            _record_stream(cur, compute)
            with torch.cuda.stream(stream):
                nxt = self._move(b)
            yield cur
        compute.wait_stream(stream)
        _record_stream(nxt, compute)
        yield nxt


def _record_stream(b, stream):
    """Batches are allocated on the copy stream but read on the compute stream: tell the caching
    allocator, so a dropped batch's memory is not handed to the next H2D copy while compute
    kernels queued on ``stream`` still read it."""
    if isinstance(b, torch.Tensor):
        if b.is_cuda:
            b.record_stream(stream)
    elif isinstance(b, (list, tuple)):
        for x in b:
            _record_stream(x, stream)
    elif isinstance(b, dict):
        for x in b.values():
            _record_stream(x, stream)


def prepare_data_loader(data_loader: DataLoader, add_dist_sampler: bool = True, move_to_device: bool = True,
                        auto_transfer: bool = True):
    world = dist.get_world_size() if dist.is_initialized() else 1
    loader = data_loader
    if add_dist_sampler and world > 1 and not isinstance(loader.sampler, DistributedSampler):
        shuffle = isinstance(loader.sampler, RandomSampler)
        sampler = DistributedSampler(loader.dataset, num_replicas=world, rank=dist.get_rank(), shuffle=shuffle)
        loader = DataLoader(loader.dataset, batch_size=loader.batch_size, sampler=sampler,
                            num_workers=loader.num_workers, collate_fn=loader.collate_fn,
                            pin_memory=loader.pin_memory, drop_last=loader.drop_last,
                            persistent_workers=loader.persistent_workers if loader.num_workers > 0 else False)
    if move_to_device:
        return _DeviceLoader(loader, get_device())
    return loader


def backward(tensor):
    tensor.backward()
