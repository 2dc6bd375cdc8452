"""The SFT job (fine_tune_llama_ray.py path) end to end on 2 CPU workers: QLoRA + LoRA r on 7 targets,
grad accumulation, eval/save steps, TensorBoard events, checkpoint-<step> layout, merge + save,
inference comparison JSON; plus a full-FT run and trainer resume."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jobs"))


@pytest.fixture(autouse=True)
def _rt(monkeypatch, tmp_path):
    from gke_ray_train_amd import runtime as rt
    monkeypatch.setenv("GRT_STORAGE_PATH", str(tmp_path / "ray_results"))
    rt.init(num_cpus=4, num_gpus=0, ignore_reinit_error=True)
    yield
    rt.shutdown()


def _cfg(tmp_path, **kw):
    import fine_tune_llama_ray as job
    over = {"MODEL_ID": "llama-tiny-gqa", "OUTPUT_DIR_BASE": str(tmp_path / "out"), "MAX_SEQ_LENGTH": 96,
            "LORA_R": 4, "LORA_ALPHA": 8, "NUM_TRAIN_SAMPLES": 48, "NUM_EVAL_SAMPLES": 16, "LOGGING_STEPS": 2,
            "SAVE_STEPS_SFT": 3, "EVAL_STEPS_SFT": 3, "GRADIENT_ACCUMULATION_STEPS": 2, "INFERENCE": True,
            "MAX_NEW_GENERATION_TOKENS_INFERENCE": 8, "NUM_TRAIN_EPOCHS": 1}
    over.update(kw)
    return job.load_config(overrides=over)


def test_qlora_sft_job(tmp_path):
    import fine_tune_llama_ray as job
    cfg = _cfg(tmp_path)
    res = job.main(cfg, num_workers=2, use_gpu=False)
    m = res.metrics
    for k in ("train_runtime", "train_samples_per_second", "train_steps_per_second", "train_loss"):
        assert k in m, k
    sft = tmp_path / "out" / "sft_model_output_sql_gretel"
    ck = sorted(d for d in os.listdir(sft) if d.startswith("checkpoint-"))
    assert ck and ck[0] == "checkpoint-3"
    files = set(os.listdir(sft / ck[0]))
    for f in ("adapter_model.safetensors", "adapter_config.json", "optimizer.pt", "scheduler.pt",
              "trainer_state.json", "training_args.bin", "rng_state_0.pth", "rng_state_1.pth"):
        assert f in files, f
    st = json.load(open(sft / ck[0] / "trainer_state.json"))
    assert st["global_step"] == 3 and any("eval_loss" in r for r in st["log_history"])
    runs = list((sft / "runs").rglob("events.out.tfevents.*"))
    assert runs
    from gke_ray_train_amd.trainer.tb import read_scalars
    tags = {t for t, _, _ in read_scalars(str(runs[0]))}
    assert "train/loss" in tags and "eval/loss" in tags
    merged = tmp_path / "out" / "final_merged_model_on_gcs"
    assert {"config.json", "model.safetensors", "tokenizer_config.json"} <= set(os.listdir(merged))
    inf = json.load(open(tmp_path / "out" / "inference_comparison_results.json"))
    assert inf and {"ground_truth_sql", "original_model_sql_response", "fine_tuned_model_sql_response"} <= set(inf[0])


def test_full_ft_job_and_resume(tmp_path):
    import fine_tune_llama_ray as job
    cfg = _cfg(tmp_path, USE_QLORA=False, INFERENCE=False, NUM_TRAIN_SAMPLES=24, SAVE_STEPS_SFT=2)
    res = job.main(cfg, num_workers=1, use_gpu=False)
    assert os.path.exists(tmp_path / "out" / "final_model_on_gcs" / "model.safetensors")
    # resume a trainer from the saved full-model checkpoint
    import torch
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.trainer import SFTConfig, SFTTrainer
    sft = tmp_path / "out" / "sft_model_output_sql_gretel"
    ck = sorted((d for d in os.listdir(sft) if d.startswith("checkpoint-")), key=lambda d: int(d.split("-")[1]))[0]
    m = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32)
    rows = [{"text": "hello world " * 5}] * 24
    tr = SFTTrainer(m, SFTConfig(output_dir=str(tmp_path / "r"), per_device_train_batch_size=2,
                                 gradient_accumulation_steps=2, max_steps=4, logging_steps=1, save_steps=100),
                    train_dataset=rows)
    out = tr.train(resume_from_checkpoint=str(sft / ck))
    assert out.global_step == 4
