"""Job submission client (``ray.job_submission.JobSubmissionClient`` surface) for the head daemon.

Reference usage: ``ray job submit --address http://localhost:8265 --runtime-env-json {...} --
python ray-jobs/fine_tune_llama_ray.py`` (a3-mega/gke-ray-cluster-setup.sh:71-91). The CLI in
``gke_ray_train_amd.cli`` is a thin layer over this client.
"""
from __future__ import annotations

import enum
import json
import time
import urllib.error
import urllib.request
from typing import Dict, Iterator, List, Optional

from .head import read_current_cluster


class JobStatus(str, enum.Enum):
    PENDING = "PENDING"
    RUNNING = "RUNNING"
    STOPPED = "STOPPED"
    SUCCEEDED = "SUCCEEDED"
    FAILED = "FAILED"

    def is_terminal(self) -> bool:
        return self in (JobStatus.STOPPED, JobStatus.SUCCEEDED, JobStatus.FAILED)

    def __str__(self):
        return self.value


def resolve_head_address(address: Optional[str]) -> str:
    if address in (None, "", "auto"):
        cur = read_current_cluster()
        if cur is None:
            raise ConnectionError("no running grt head found (start one with `grt start --head`)")
        return cur["address"]
    if not address.startswith("http"):
        address = "http://" + address
    return address.rstrip("/")


class JobSubmissionClient:
    def __init__(self, address: Optional[str] = None, timeout: float = 30.0):
        self.address = resolve_head_address(address)
        self.timeout = timeout
        self._req("GET", "/api/version")  # fail fast when nothing listens

    def _req(self, method, path, body=None):
        data = json.dumps(body).encode() if body is not None else None
        r = urllib.request.Request(self.address + path, data=data, method=method,
                                   headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(r, timeout=self.timeout) as resp:
                return json.loads(resp.read() or b"null")
        except urllib.error.HTTPError as e:
            msg = e.read().decode(errors="replace")
            try:
                msg = json.loads(msg).get("error", msg)
            except ValueError:
                pass
            if e.code == 404:
                raise RuntimeError(f"not found: {msg}") from None
            raise RuntimeError(f"job server error {e.code}: {msg}") from None

    def submit_job(self, *, entrypoint: str, runtime_env: Optional[dict] = None, submission_id: Optional[str] = None,
                   metadata: Optional[Dict[str, str]] = None, entrypoint_num_gpus: float = 0,
                   entrypoint_num_cpus: float = 0, job_id: Optional[str] = None) -> str:
        body = {"entrypoint": entrypoint, "runtime_env": runtime_env or {}, "submission_id": submission_id or job_id,
                "metadata": metadata or {}, "entrypoint_num_gpus": entrypoint_num_gpus,
                "entrypoint_num_cpus": entrypoint_num_cpus}
        return self._req("POST", "/api/jobs/", body)["submission_id"]

    def get_job_info(self, job_id: str) -> dict:
        return self._req("GET", f"/api/jobs/{job_id}")

    def get_job_status(self, job_id: str) -> JobStatus:
        return JobStatus(self.get_job_info(job_id)["status"])

    def get_job_logs(self, job_id: str) -> str:
        return self._req("GET", f"/api/jobs/{job_id}/logs")["logs"]

    def tail_job_logs(self, job_id: str, poll: float = 0.5) -> Iterator[str]:
        """Yield new log text until the job reaches a terminal state."""
        seen = 0
        while True:
            status = self.get_job_status(job_id)
            logs = self.get_job_logs(job_id)
            if len(logs) > seen:
                yield logs[seen:]
                seen = len(logs)
            if status.is_terminal():
                logs = self.get_job_logs(job_id)
                if len(logs) > seen:
                    yield logs[seen:]
                return
            time.sleep(poll)

    def wait(self, job_id: str, timeout: Optional[float] = None, poll: float = 0.5) -> JobStatus:
        t0 = time.time()
        while True:
            st = self.get_job_status(job_id)
            if st.is_terminal():
                return st
            if timeout is not None and time.time() - t0 > timeout:
                raise TimeoutError(f"job {job_id} still {st} after {timeout}s")
            time.sleep(poll)

    def stop_job(self, job_id: str) -> bool:
        return bool(self._req("POST", f"/api/jobs/{job_id}/stop", {})["stopped"])

    def delete_job(self, job_id: str) -> bool:
        return bool(self._req("DELETE", f"/api/jobs/{job_id}")["deleted"])

    def list_jobs(self) -> List[dict]:
        return self._req("GET", "/api/jobs/")

    def cluster_status(self) -> dict:
        return self._req("GET", "/api/cluster_status")

    def shutdown_cluster(self):
        return self._req("POST", "/api/shutdown", {})
