"""Typed configuration layer: the reference's JSON / dict configs with validation and overrides.

The reference has no flag parser: the SFT job reads 35 keys from ray-jobs/fine_tune_config.json by
a working-dir-relative path (ray-jobs/fine_tune_llama_ray.py:428-436), the BasicLLM job builds a
19-key dict literal (ray-jobs/pytorch_llm_ray.py:324-344), and worker counts come from
NUM_NODES / NUM_GPUS_PER_NODE env vars (:439-442) — SURVEY §5.6. Several keys are read but never
used (§2.8). This module keeps the SAME key names and JSON files, and adds:

* a dataclass per job with the reference defaults and types (coercion of JSON/CLI strings);
* unknown keys -> warning (typos are no longer silently ignored), keys the reference reads but
  never uses are accepted and listed in ``UNUSED_BY_REFERENCE``;
* ``--set KEY=VALUE`` overrides (values parsed as JSON, falling back to strings);
* ``num_workers_from_env()``: NUM_NODES x NUM_GPUS_PER_NODE with the node's MI355X count as the
  default instead of the reference's 1 x 1.
"""
from __future__ import annotations

import dataclasses
import json
import os
import warnings
from dataclasses import asdict, dataclass, field, fields
from typing import Any, Dict, Iterable, List, Optional


@dataclass
class FineTuneConfig:
    """ray-jobs/fine_tune_config.json (all 35 keys) + framework extensions (bottom)."""
    MODEL_ID: str = "meta-llama/Meta-Llama-3.1-8B-Instruct"
    DATASET_NAME: str = "gretelai/synthetic_text_to_sql"
    OUTPUT_DIR_BASE: str = "pvc/finetuned_llama3_1_8b_gretel_sql"
    USE_QLORA: bool = True
    LORA_ALPHA: int = 16
    LORA_DROPOUT: float = 0.1
    LORA_R: int = 64
    BNB_4BIT_COMPUTE_DTYPE: str = "bfloat16"
    BNB_4BIT_QUANT_TYPE: str = "nf4"
    USE_NESTED_QUANT: bool = False
    NUM_TRAIN_EPOCHS: float = 1
    PER_DEVICE_TRAIN_BATCH_SIZE: int = 2
    GRADIENT_ACCUMULATION_STEPS: int = 4
    LEARNING_RATE: float = 2e-4
    WEIGHT_DECAY: float = 0.001
    OPTIM: str = "paged_adamw_32bit"
    LR_SCHEDULER_TYPE: str = "cosine"
    MAX_GRAD_NORM: float = 0.3
    WARMUP_RATIO: float = 0.03
    LOGGING_STEPS: int = 10
    SAVE_STRATEGY: str = "steps"
    SAVE_STEPS_SFT: int = 50
    EVALUATION_STRATEGY_SFT: str = "steps"
    EVAL_STEPS_SFT: int = 50
    REPORT_TO: str = "tensorboard"
    MAX_SEQ_LENGTH: int = 1024
    PACKING: bool = False
    GROUP_BY_LENGTH: bool = True
    LLAMA_TARGET_MODULES: List[str] = field(default_factory=lambda: ["q_proj", "k_proj", "v_proj", "o_proj",
                                                                     "gate_proj", "up_proj", "down_proj"])
    NUM_EVAL_SAMPLES_INFERENCE: int = 2
    MAX_NEW_GENERATION_TOKENS_INFERENCE: int = 300
    SFT_SUBDIR_NAME: str = "sft_model_output_sql_gretel"
    MERGED_MODEL_SUBDIR_NAME: str = "final_merged_model_on_gcs"
    FULL_FT_MODEL_SUBDIR_NAME: str = "final_model_on_gcs"
    INFERENCE: bool = False
    # ---- extensions (not in the reference file)
    NUM_TRAIN_SAMPLES: int = 1000       # the reference hard-codes select(<=1000) (:288)
    NUM_EVAL_SAMPLES: int = 200         # ... and select(<=200)
    MAX_STEPS: int = -1
    GRADIENT_CHECKPOINTING: bool = False
    USE_LORA_BF16: bool = False         # BASELINE config #4: LoRA on an unquantized bf16 base
    SEED: int = 0


# keys the reference reads but never uses: accepted, flagged in the docs
UNUSED_BY_REFERENCE = {"FineTuneConfig": ["DATASET_NAME", "NUM_EVAL_SAMPLES_INFERENCE"],
                       "BasicLLMTrainConfig": ["train_report_frequency_steps", "storage_path_base_on_fuse",
                                               "experiment_name_for_tb"]}


@dataclass
class BasicLLMTrainConfig:
    """train_loop_config of ray-jobs/pytorch_llm_ray.py:324-344 (19 keys, same names/defaults)."""
    lr: float = 3e-4
    batch_size_per_worker: int = 16
    num_epochs: int = 1
    embed_dim: int = 2048
    num_layers: int = 24
    num_heads: int = 16
    hidden_dim: int = 2048 * 4
    model_max_seq_len: int = 1024
    dataset_seq_len: int = 256
    dataloader_num_workers: int = 0
    log_frequency_batches: int = 20
    train_report_frequency_steps: int = 20
    warmup_steps_ratio: float = 0.05
    min_lr_ratio: float = 0.01
    raw_data_path: str = "/mnt/pvc/datasets/wikitext-2-raw/wiki.train.tokens"
    processed_data_dir: str = "/mnt/pvc/datasets/wikitext-2-processed/"
    storage_path_base_on_fuse: str = "/mnt/pvc/ray_llm_training_runs"
    experiment_name_for_tb: str = "wikitext2_manualTB_v1"
    test_run: bool = True


def _coerce(value: Any, typ) -> Any:
    """JSON/CLI value -> the dataclass field type (bool/int/float/str/list)."""
    origin = getattr(typ, "__origin__", None)
    if isinstance(typ, str):  # postponed annotations
        typ = {"bool": bool, "int": int, "float": float, "str": str}.get(typ, None) or typ
    if typ is bool or typ == "bool":
        if isinstance(value, str):
            v = value.strip().lower()
            if v in ("1", "true", "yes", "on"):
                return True
            if v in ("0", "false", "no", "off"):
                return False
            raise ValueError(f"not a boolean: {value!r}")
        return bool(value)
    if typ in (int, "int"):
        if isinstance(value, bool):
            raise ValueError("boolean given for an integer key")
        f = float(value)
        if f != int(f):
            raise ValueError(f"not an integer: {value!r}")
        return int(f)
    if typ in (float, "float"):
        return float(value)
    if typ in (str, "str"):
        return str(value)
    if origin in (list, List) or (isinstance(typ, str) and typ.startswith("List")):
        if isinstance(value, str):
            value = json.loads(value) if value.strip().startswith("[") else [x for x in value.split(",") if x]
        return list(value)
    return value


def from_dict(cls, d: Dict[str, Any], strict: bool = False):
    """Build ``cls`` from a dict; unknown keys warn (or raise with ``strict``)."""
    names = {f.name: f for f in fields(cls)}
    unknown = [k for k in d if k not in names]
    if unknown:
        msg = f"{cls.__name__}: unknown config keys {sorted(unknown)}"
        if strict:
            raise KeyError(msg)
        warnings.warn(msg)
    kw = {}
    for k, v in d.items():
        if k in names:
            try:
                kw[k] = _coerce(v, names[k].type)
            except (TypeError, ValueError) as e:
                raise ValueError(f"{cls.__name__}.{k}: {e}") from None
    return cls(**kw)


def parse_overrides(items: Optional[Iterable[str]]) -> Dict[str, Any]:
    """``["LEARNING_RATE=1e-4", "USE_QLORA=false", 'LLAMA_TARGET_MODULES=["q_proj"]']`` -> dict."""
    out = {}
    for it in items or []:
        if "=" not in it:
            raise ValueError(f"override {it!r} is not KEY=VALUE")
        k, v = it.split("=", 1)
        try:
            out[k.strip()] = json.loads(v)
        except json.JSONDecodeError:
            out[k.strip()] = v
    return out


def load_json_config(cls, path: Optional[str] = None, overrides: Optional[Dict[str, Any]] = None,
                     strict: bool = False):
    d: Dict[str, Any] = {}
    if path:
        with open(path) as f:
            d.update(json.load(f))
    d.update(overrides or {})
    return from_dict(cls, d, strict=strict)


def to_dict(cfg) -> Dict[str, Any]:
    return asdict(cfg)


def num_workers_from_env(default_gpus: Optional[int] = None) -> int:
    """NUM_NODES x NUM_GPUS_PER_NODE; GPUs per node default to the visible MI355X count."""
    nodes = int(os.environ.get("NUM_NODES", "1"))
    if "NUM_GPUS_PER_NODE" in os.environ:
        per = int(os.environ["NUM_GPUS_PER_NODE"])
    else:
        if default_gpus is None:
            try:
                import torch
                default_gpus = torch.cuda.device_count()  # does not initialise HIP
            except Exception:
                default_gpus = 0
        per = max(1, default_gpus)
    return nodes * per


__all__ = ["FineTuneConfig", "BasicLLMTrainConfig", "UNUSED_BY_REFERENCE", "from_dict", "parse_overrides",
           "load_json_config", "to_dict", "num_workers_from_env", "dataclasses"]
