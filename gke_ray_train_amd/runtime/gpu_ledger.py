"""Node-wide GPU lease ledger: one ``flock``-ed file per GPU.

Ray keeps one resource ledger per cluster, so two jobs attached with ``ray.init(address='auto')``
(reference ray-jobs/prepare_wikitext2_ray_job.py:95-109) can never both hold GPU 3. This runtime
starts a scheduler per driver, so the ledger has to live outside any one process: GPU ``i`` is
leased by taking an exclusive, non-blocking ``flock`` on ``<dir>/gpu<i>.lock``. The kernel drops
the lock when the holder closes it or dies, so a crashed driver never leaks a GPU, and no daemon
or cleanup pass is needed. ``GRT_GPU_LEASES=0`` keeps the lease table in-process only.
"""
from __future__ import annotations

import fcntl
import os
import threading
from typing import Dict, List, Optional


def _lease_dir() -> str:
    d = os.environ.get("GRT_GPU_LEASE_DIR")
    if not d:
        from ..cluster.head import grt_tmpdir
        d = os.path.join(grt_tmpdir(), "gpu_leases")
    return d


class GpuLedger:
    def __init__(self, num_gpus: int, directory: Optional[str] = None, shared: bool = True):
        self.n = int(num_gpus)
        self.shared = shared and self.n > 0
        self.dir = directory
        self._fds: Dict[int, int] = {}   # GPU index -> locked fd (shared) / -1 (in-process)
        self._lock = threading.Lock()
        if self.shared:
            os.makedirs(self.dir, exist_ok=True)

    @classmethod
    def for_node(cls, num_gpus: int) -> "GpuLedger":
        shared = os.environ.get("GRT_GPU_LEASES", "1") != "0"
        return cls(num_gpus, _lease_dir() if shared else None, shared=shared)

    def _try_lock(self, i: int) -> Optional[int]:
        if not self.shared:
            return -1
        fd = os.open(os.path.join(self.dir, f"gpu{i}.lock"), os.O_RDWR | os.O_CREAT, 0o666)
        try:
            fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
        except OSError:
            os.close(fd)
            return None
        os.ftruncate(fd, 0)
        os.write(fd, f"{os.getpid()}\n".encode())
        return fd

    def _unlock(self, fd: int):
        if fd >= 0:
            try:
                fcntl.flock(fd, fcntl.LOCK_UN)
            finally:
                os.close(fd)

    def try_acquire(self, k: int) -> Optional[List[int]]:
        """Lease ``k`` GPUs (lowest free indices) or return None without holding any."""
        k = int(k)
        if k <= 0:
            return []
        with self._lock:
            got: List[int] = []
            for i in range(self.n):
                if len(got) == k:
                    break
                if i in self._fds:
                    continue
                fd = self._try_lock(i)
                if fd is not None:
                    self._fds[i] = fd
                    got.append(i)
            if len(got) < k:
                for i in got:
                    self._unlock(self._fds.pop(i))
                return None
            return got

    def release(self, ids) -> None:
        with self._lock:
            for i in ids or []:
                fd = self._fds.pop(i, None)
                if fd is not None:
                    self._unlock(fd)

    def num_free(self) -> int:
        """GPUs neither leased here nor by another process (probed, not reserved)."""
        with self._lock:
            free = 0
            for i in range(self.n):
                if i in self._fds:
                    continue
                fd = self._try_lock(i)
                if fd is not None:
                    free += 1
                    self._unlock(fd)
            return free

    def held(self) -> List[int]:
        with self._lock:
            return sorted(self._fds)

    def describe(self) -> str:
        return f"{self.n} GPUs, held by this driver {self.held()}, free {self.num_free()}"

    def close(self):
        self.release(list(self._fds))
