"""Single-node cluster bring-up (replaces the reference's GKE/KubeRay scripts and RayCluster CRs):
cluster spec (``spec.py``), head daemon / job server (``head.py``), job client (``jobs.py``)."""
from .config import resolve_address
from .head import read_current_cluster
from .jobs import JobStatus, JobSubmissionClient
from .spec import ClusterSpec, envsubst

__all__ = ["ClusterSpec", "JobStatus", "JobSubmissionClient", "envsubst", "read_current_cluster", "resolve_address"]
