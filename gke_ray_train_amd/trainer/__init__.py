"""Trainers: SFT (HF-Trainer / TRL semantics), LR schedules, callbacks, TensorBoard writer."""
from .callbacks import RayTrainReportCallback, prepare_trainer
from .schedules import get_scheduler, warmup_cosine_floor
from .sft import SFTConfig, SFTTrainer, TrainOutput
from .sft_data import (SYSTEM_PROMPT, LengthGroupedSampler, PadCollator, format_chat_sample, pack_sequences,
                       synthetic_text_to_sql)

__all__ = ["RayTrainReportCallback", "prepare_trainer", "get_scheduler", "warmup_cosine_floor", "SFTConfig",
           "SFTTrainer", "TrainOutput", "SYSTEM_PROMPT", "LengthGroupedSampler", "PadCollator", "format_chat_sample",
           "pack_sequences", "synthetic_text_to_sql"]
