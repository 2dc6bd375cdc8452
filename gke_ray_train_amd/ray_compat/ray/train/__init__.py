from gke_ray_train_amd.train import *  # noqa: F401,F403
from gke_ray_train_amd.train import (Checkpoint, CheckpointConfig, FailureConfig, Result, RunConfig, ScalingConfig,
                                     get_checkpoint, get_context, get_dataset_shard, report)
from . import torch  # noqa: F401
