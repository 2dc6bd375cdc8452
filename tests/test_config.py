"""Typed config layer: reference JSON keys, coercion, unknown-key warnings, CLI
overrides, env-var worker scaling."""
import json
import os
import warnings

import pytest

from gke_ray_train_amd.utils.config import (BasicLLMTrainConfig, FineTuneConfig, from_dict, load_json_config,
                                            num_workers_from_env, parse_overrides)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_json_loads_with_all_35_keys():
    path = os.path.join(ROOT, "jobs", "fine_tune_config.json")
    raw = json.load(open(path))
    assert len(raw) == 35
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        cfg = load_json_config(FineTuneConfig, path)
    assert cfg.USE_QLORA is True and cfg.LORA_R == 64 and cfg.OPTIM == "paged_adamw_32bit"
    assert cfg.LLAMA_TARGET_MODULES[-1] == "down_proj" and cfg.MAX_GRAD_NORM == 0.3


def test_overrides_coercion_and_unknown_keys():
    ov = parse_overrides(["LEARNING_RATE=1e-5", "USE_QLORA=false", 'LLAMA_TARGET_MODULES=["q_proj","v_proj"]',
                          "OPTIM=adamw_torch", "PER_DEVICE_TRAIN_BATCH_SIZE=8"])
    cfg = from_dict(FineTuneConfig, ov)
    assert cfg.LEARNING_RATE == 1e-5 and cfg.USE_QLORA is False and cfg.PER_DEVICE_TRAIN_BATCH_SIZE == 8
    assert cfg.LLAMA_TARGET_MODULES == ["q_proj", "v_proj"]
    assert from_dict(FineTuneConfig, {"USE_QLORA": "yes", "LORA_R": "16"}).LORA_R == 16
    with pytest.warns(UserWarning, match="LERNING_RATE"):
        from_dict(FineTuneConfig, {"LERNING_RATE": 1.0})
    with pytest.raises(KeyError):
        from_dict(FineTuneConfig, {"LERNING_RATE": 1.0}, strict=True)
    with pytest.raises(ValueError):
        from_dict(FineTuneConfig, {"LORA_R": 2.5})
    with pytest.raises(ValueError):
        parse_overrides(["NOEQUALS"])
    assert from_dict(BasicLLMTrainConfig, {"test_run": "false"}).test_run is False


def test_num_workers_from_env(monkeypatch):
    monkeypatch.setenv("NUM_NODES", "1")
    monkeypatch.setenv("NUM_GPUS_PER_NODE", "8")
    assert num_workers_from_env() == 8
    monkeypatch.delenv("NUM_GPUS_PER_NODE")
    assert num_workers_from_env(default_gpus=4) == 4
    assert num_workers_from_env(default_gpus=0) == 1
