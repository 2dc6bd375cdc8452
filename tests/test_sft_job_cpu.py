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


def _fused_vs_unfused(tmp_path, fuse, padding_free=None):
    import torch
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.trainer import SFTConfig, SFTTrainer
    torch.manual_seed(0)
    m = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32)
    # varied lengths so micro-batches pad differently and carry different valid-token counts
    rows = [{"text": "select * from t where x = %d " % i * (1 + i % 4)} for i in range(16)]
    tr = SFTTrainer(m, SFTConfig(output_dir=str(tmp_path / f"{fuse}_{padding_free}"), per_device_train_batch_size=2,
                                 gradient_accumulation_steps=4, max_steps=2, logging_steps=1, save_strategy="no",
                                 learning_rate=1e-3, max_grad_norm=1e9, fuse_accumulation=fuse, fuse_max_tokens=10 ** 6,
                                 padding_free=padding_free),
                    train_dataset=rows)
    out = tr.train()
    return out, {k: v.detach().clone() for k, v in m.state_dict().items()}


@pytest.mark.parametrize("padding_free", [False, True])
def test_fused_grad_accumulation_matches_unfused(tmp_path, padding_free):
    """One batch per optimizer step with per-micro-batch loss weights == HF-style accumulation of
    per-micro-batch means (same loss, same updated parameters) — padded, or padding-free packed
    (sequences on one token axis, ops.Varlen)."""
    import torch
    a, pa = _fused_vs_unfused(tmp_path, False)
    b, pb = _fused_vs_unfused(tmp_path, True, padding_free)
    assert abs(a.training_loss - b.training_loss) < 1e-4 * max(1.0, abs(a.training_loss))
    # AdamW's first steps are ~lr * sign(g): elements whose gradient is ~0 may flip under fp32
    # summation-order changes, so allow a handful of such elements (bounded by 2 steps x lr)
    for k in pa:
        d = (pa[k] - pb[k]).abs()
        assert float(d.max()) <= 2e-3, k
        assert int((d > 1e-5).sum()) <= max(2, pa[k].numel() // 10000), k


def test_step_chunks_respect_token_cap(tmp_path):
    import torch
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.trainer import SFTConfig, SFTTrainer
    m = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32)
    rows = [{"text": "abc " * (3 + i)} for i in range(8)]
    tr = SFTTrainer(m, SFTConfig(output_dir=str(tmp_path), per_device_train_batch_size=2, gradient_accumulation_steps=4,
                                 fuse_accumulation=True, fuse_max_tokens=2 * 48, padding_free=False), train_dataset=rows)
    batches = tr._batches(tr.train_seqs, 2, 0, shuffle=False)
    chunks = tr._step_chunks(batches, list(range(4)), True)
    assert 1 < len(chunks) <= 4
    tot_w = 0.0
    for cb, w in chunks:
        assert cb["input_ids"].numel() <= 2 * 48 or cb["input_ids"].shape[0] == 2
        assert w.shape == cb["input_ids"].shape
        valid = (cb["labels"][:, 1:] != -100) & (cb["attention_mask"][:, 1:] != 0)
        tot_w += float((w[:, :-1] * valid).sum())
    assert abs(tot_w - 1.0) < 1e-6  # 4 micro-batches x (n_m * 1 / (n_m * 4))


def test_lm_head_row_weights_cpu():
    import torch
    import torch.nn.functional as F
    from gke_ray_train_amd.ops.fused import lm_head_cross_entropy
    torch.manual_seed(0)
    h = torch.randn(10, 16, requires_grad=True)
    w = torch.randn(32, 16, requires_grad=True)
    lab = torch.randint(0, 32, (10,))
    lab[3] = -100
    rw = torch.rand(10)
    loss = lm_head_cross_entropy(h, w, lab, row_weights=rw)
    ref = (F.cross_entropy(h @ w.t(), lab, reduction="none") * rw * (lab != -100)).sum()
    torch.testing.assert_close(loss, ref)
    loss.backward()
    assert h.grad is not None and torch.isfinite(h.grad).all()


def test_padding_free_pack_layout(tmp_path):
    """Packed step: real tokens only (plus one masked filler segment up to the pad multiple), per-token
    weights summing to 1 over the valid next-token targets, sequence lengths for ops.Varlen."""
    import torch
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.trainer import SFTConfig, SFTTrainer
    m = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32)
    rows = [{"text": "abc " * (3 + i)} for i in range(8)]
    tr = SFTTrainer(m, SFTConfig(output_dir=str(tmp_path), per_device_train_batch_size=2, gradient_accumulation_steps=4,
                                 fuse_accumulation=True, pack_multiple=64, padding_free=True), train_dataset=rows)
    batches = tr._batches(tr.train_seqs, 2, 0, shuffle=False)
    (cb, w), = tr._step_chunks(batches, list(range(4)), True)
    real = sum(len(s) for s in tr.train_seqs)
    assert cb["input_ids"].shape == (1, sum(cb["lengths"])) and cb["input_ids"].shape[1] % 64 == 0
    assert int(cb["attention_mask"].sum()) == real and sum(cb["lengths"][:8]) == real
    bounds = torch.tensor(cb["lengths"]).cumsum(0)
    valid = torch.zeros(cb["input_ids"].shape[1], dtype=torch.bool)
    for a, b in zip([0] + bounds.tolist()[:-1], bounds.tolist()):
        valid[a:b - 1] = cb["labels"][0, a + 1:b] != -100  # targets inside each sequence only
    assert abs(float((w[0] * valid).sum()) - 1.0) < 1e-6


def test_padding_free_groups_by_real_tokens(tmp_path):
    """Packed rows hold whole micro-batches while their real tokens fit pack_max_tokens; the
    weights over all rows of the step still sum to 1."""
    import torch
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.trainer import SFTConfig, SFTTrainer
    m = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32)
    rows = [{"text": "abc " * (3 + i)} for i in range(8)]
    tr = SFTTrainer(m, SFTConfig(output_dir=str(tmp_path), per_device_train_batch_size=2, gradient_accumulation_steps=4,
                                 max_seq_length=64, fuse_accumulation=True, pack_multiple=16, pack_max_tokens=70,
                                 padding_free=True), train_dataset=rows)
    batches = tr._batches(tr.train_seqs, 2, 0, shuffle=False)
    chunks = tr._step_chunks(batches, list(range(4)), True)
    assert len(chunks) > 1
    tot = 0.0
    for cb, w in chunks:
        real = int(cb["attention_mask"].sum())
        assert real <= 70 or len(cb["lengths"]) <= 3      # one micro-batch (2 rows + filler) may exceed
        assert cb["input_ids"].shape[1] % 16 == 0
        bounds = torch.tensor(cb["lengths"]).cumsum(0).tolist()
        valid = torch.zeros(cb["input_ids"].shape[1], dtype=torch.bool)
        for a, b in zip([0] + bounds[:-1], bounds):
            valid[a:b - 1] = cb["labels"][0, a + 1:b] != -100
        tot += float((w[0] * valid).sum())
    assert abs(tot - 1.0) < 1e-5


def test_padding_free_eval_matches_padded(tmp_path):
    """evaluate() on padding-free packed batches (the default on GPU) gives the padded token-weighted
    eval_loss: same sequences, attention confined to each sequence by ops.Varlen."""
    import torch
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.trainer import SFTConfig, SFTTrainer
    torch.manual_seed(0)
    m = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32)
    rows = [{"text": "select * from t where x = %d " % i * (1 + i % 4)} for i in range(12)]
    losses = []
    for pf in (False, True):
        tr = SFTTrainer(m, SFTConfig(output_dir=str(tmp_path / f"e{pf}"), per_device_train_batch_size=2,
                                     per_device_eval_batch_size=3, gradient_accumulation_steps=2,
                                     fuse_accumulation=True, eval_padding_free=pf, pack_multiple=16),
                        train_dataset=rows, eval_dataset=rows)
        losses.append(tr.evaluate()["eval_loss"])
    assert abs(losses[0] - losses[1]) < 1e-5 * max(1.0, abs(losses[0])), losses


def test_padding_free_pack_selects_tokens_by_mask_for_left_padding(tmp_path, monkeypatch):
    """A user collator that LEFT-pads: the packed row must hold each sequence's real tokens (chosen
    by the attention mask), not its first L positions (pads); and GRT_SFT_EVAL_PADDING_FREE=0 turns
    packed evaluation off."""
    import torch
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.trainer import SFTConfig, SFTTrainer
    m = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32)
    rows = [{"text": "abc " * (3 + i)} for i in range(4)]
    tr = SFTTrainer(m, SFTConfig(output_dir=str(tmp_path), per_device_train_batch_size=2, gradient_accumulation_steps=1,
                                 fuse_accumulation=True, pack_multiple=1, padding_free=True), train_dataset=rows)
    pad = tr.pad_id
    ids = torch.tensor([[pad, pad, 5, 6, 7], [8, 9, 10, 11, 12]])
    mask = torch.tensor([[0, 0, 1, 1, 1], [1, 1, 1, 1, 1]])
    labels = ids.masked_fill(mask == 0, -100)
    out, w = tr._pack([{"input_ids": ids, "labels": labels, "attention_mask": mask}], 1, True)
    assert out["input_ids"][0].tolist() == [5, 6, 7, 8, 9, 10, 11, 12]
    assert out["lengths"] == [3, 5] and out["ntarget"] == 2 + 4
    monkeypatch.setenv("GRT_SFT_EVAL_PADDING_FREE", "0")
    assert tr._eval_padding_free() is False
