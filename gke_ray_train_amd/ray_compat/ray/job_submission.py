"""``ray.job_submission`` shim: the job client of the node-local head daemon."""
from gke_ray_train_amd.cluster.jobs import JobStatus, JobSubmissionClient

__all__ = ["JobStatus", "JobSubmissionClient"]
