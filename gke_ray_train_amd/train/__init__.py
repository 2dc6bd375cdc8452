"""Ray-Train-compatible API (``from gke_ray_train_amd import train`` ~ ``from ray import train``)."""
from . import torch  # noqa: F401  (train.torch.get_device / prepare_model / prepare_data_loader)
from ._checkpoint import Checkpoint
from ._config import CheckpointConfig, FailureConfig, RunConfig, ScalingConfig
from ._result import Result
from ._session import TrainContext, get_checkpoint, get_context, get_dataset_shard, report
from ._trainer import DataParallelTrainer, TorchTrainer
from ..runtime.errors import TrainingFailedError

__all__ = ["Checkpoint", "CheckpointConfig", "FailureConfig", "RunConfig", "ScalingConfig", "Result",
           "TrainContext", "get_checkpoint", "get_context", "get_dataset_shard", "report", "DataParallelTrainer",
           "TorchTrainer", "TrainingFailedError", "torch"]
