"""``RayTrainReportCallback`` / ``prepare_trainer`` for the framework's SFT trainer (imported but unused by
the reference, ray-jobs/fine_tune_llama_ray.py:8)."""
from gke_ray_train_amd.trainer.callbacks import RayTrainReportCallback, prepare_trainer  # noqa: F401
