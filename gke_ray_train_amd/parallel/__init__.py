"""Parallelism engines: flat-buffer DDP (RCCL all-reduce) and FSDP full-shard (+CPU offload)."""
from .comm import Topology, default_backend, plan_bucket_bytes, ring_allreduce_seconds, topology
from .ddp import DistributedDataParallel

__all__ = ["DistributedDataParallel", "Topology", "default_backend", "plan_bucket_bytes",
           "ring_allreduce_seconds", "topology"]
