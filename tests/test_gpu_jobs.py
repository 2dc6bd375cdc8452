"""GPU end-to-end: the reference jobs through TorchTrainer on one MI355X worker (RCCL backend),
QLoRA on the HIP NF4 path, KV-cache generation vs full recompute, bf16 BasicLLM."""
import json
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jobs"))


@pytest.fixture
def _rt(monkeypatch, tmp_path):
    from gke_ray_train_amd import runtime as rt
    monkeypatch.setenv("GRT_STORAGE_PATH", str(tmp_path / "ray_results"))
    rt.init(num_cpus=8, ignore_reinit_error=True)
    yield
    rt.shutdown()


def test_generation_cache_matches_recompute():
    from gke_ray_train_amd.models import build_llama
    m = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=0)
    g = torch.Generator(device="cuda").manual_seed(0)
    ids = torch.randint(0, 512, (2, 40), device="cuda", generator=g)
    P, T = ids.shape[1], 8
    out = m.generate(ids, max_new_tokens=T)
    assert out.shape == (2, P + T) and torch.equal(out[:, :P], ids)
    # Teacher-forced check on the cached path's own trajectory (a free-running comparison lets one
    # bf16 near-tie flip every later token): the full-recompute logits on the same prefix must pick
    # each generated token, or rank it within bf16 rounding of the maximum (a tie).
    lg = m(out[:, :-1], return_logits=True)["logits"][:, P - 1:].float()   # predicts out[:, P:]
    gen = out[:, P:]
    best = lg.max(-1).values
    got = lg.gather(-1, gen.unsqueeze(-1)).squeeze(-1)
    tol = 0.02 + 0.01 * best.abs()
    assert bool((got >= best - tol).all()), (best - got).max().item()
    assert (lg.argmax(-1) == gen).float().mean().item() > 0.8  # ties are rare


def test_qlora_gpu_step():
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.peft import BitsAndBytesConfig, LoraConfig, get_peft_model, quantize_model_
    m = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=0)
    ids = torch.randint(0, 512, (2, 128), device="cuda")
    ref = m(ids, labels=ids)["loss"].item()
    quantize_model_(m, BitsAndBytesConfig())
    pm = get_peft_model(m, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.1))
    loss = pm(ids, labels=ids)["loss"]
    assert abs(loss.item() - ref) < 0.5
    loss.backward()
    assert all(p.grad is not None for p in pm.parameters() if p.requires_grad)


def test_fused_accumulation_loss_weights_match_micro_batches_on_gpu():
    """The SFT trainer's fused step (one padded batch, per-micro-batch loss weights) on the HIP
    path (row-weighted LM-head CE, NF4 dequant cache) gives the gradient of HF-style accumulation."""
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.peft import BitsAndBytesConfig, LoraConfig, get_peft_model, quantize_model_
    from gke_ray_train_amd.peft.quant import set_dequant_cache
    torch.manual_seed(0)
    m = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=0)
    quantize_model_(m, BitsAndBytesConfig())
    assert set_dequant_cache(m, "1")
    pm = get_peft_model(m, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.0))
    for n, p in pm.named_parameters():  # non-zero B so every adapter gradient is exercised
        if "lora_B" in n:
            p.data.normal_(0, 0.02)
    lens = [(2, 100), (2, 64), (2, 128), (2, 40)]
    micro = []
    for B, L in lens:
        ids = torch.randint(0, 512, (B, L), device="cuda")
        mask = torch.ones_like(ids)
        mask[0, L - 7:] = 0  # a padded row
        lab = ids.masked_fill(mask == 0, -100)
        micro.append((ids, mask, lab))
    accum = len(micro)
    params = [p for p in pm.parameters() if p.requires_grad]
    for ids, mask, lab in micro:
        (pm(ids, labels=lab, attention_mask=mask)["loss"] / accum).backward()
    ref = [p.grad.float().clone() for p in params]
    for p in params:
        p.grad = None
    Lm = 128
    pad = lambda t, v: torch.nn.functional.pad(t, (0, Lm - t.shape[1]), value=v)
    ids = torch.cat([pad(i, 0) for i, _, _ in micro])
    mask = torch.cat([pad(k, 0) for _, k, _ in micro])
    lab = torch.cat([pad(l, -100) for _, _, l in micro])
    w = torch.cat([torch.full((i.shape[0], Lm), 1.0 / (int(((l[:, 1:] != -100) & (k[:, 1:] != 0)).sum()) * accum),
                              device="cuda") for i, k, l in micro])
    pm(ids, labels=lab, attention_mask=mask, loss_weights=w)["loss"].backward()
    for p, r in zip(params, ref):
        g = p.grad.float()
        assert (g - r).norm() <= 2e-2 * r.norm() + 1e-6


def test_sft_job_on_gpu(_rt, tmp_path):
    import fine_tune_llama_ray as job
    cfg = job.load_config(overrides={"MODEL_ID": "llama-tiny-gqa", "OUTPUT_DIR_BASE": str(tmp_path / "out"),
                                     "MAX_SEQ_LENGTH": 256, "NUM_TRAIN_SAMPLES": 64, "NUM_EVAL_SAMPLES": 16,
                                     "SAVE_STEPS_SFT": 4, "EVAL_STEPS_SFT": 4, "LOGGING_STEPS": 2, "INFERENCE": True,
                                     "MAX_NEW_GENERATION_TOKENS_INFERENCE": 16})
    res = job.main(cfg, num_workers=1, use_gpu=True)
    assert res.metrics["train_loss"] > 0
    assert os.path.exists(tmp_path / "out" / "final_merged_model_on_gcs" / "model.safetensors")
    assert json.load(open(tmp_path / "out" / "inference_comparison_results.json"))
    # checkpoints written from the pinned snapshot: each file holds its own tensors, finite values
    from safetensors.torch import load_file
    ck = sorted((tmp_path / "out").glob("**/checkpoint-*"))
    assert ck
    ad = load_file(str(ck[-1] / "adapter_model.safetensors"))
    assert ad and all(torch.isfinite(t.float()).all() for t in ad.values())
    opt = torch.load(ck[-1] / "optimizer.pt", weights_only=True)
    st = [v for s in opt["state"].values() for v in s.values() if isinstance(v, torch.Tensor) and v.dim()]
    assert st and all(t.untyped_storage().nbytes() == t.numel() * t.element_size() for t in st)


def test_host_snapshot_copies_every_tensor_once():
    """The SFT checkpoint snapshot: one pinned buffer, mixed dtypes / shapes / strides, CPU leaves
    copied, and materialize() gives tensors that own their storage."""
    from gke_ray_train_amd.trainer.sft import _HostSnapshot
    dev = torch.device("cuda", 0)
    a = torch.randn(33, 7, device=dev)
    b = torch.randn(64, 48, device=dev, dtype=torch.bfloat16).t()   # non-contiguous
    c = torch.tensor(5.0, device=dev)                                # 0-dim
    d = torch.arange(10)                                             # CPU leaf
    obj = {"x": [a, (b, c)], "y": {"z": d, "n": 3}}
    snap = _HostSnapshot()
    a0 = a.clone()
    h = snap.take(obj)
    a.add_(1.0)  # the snapshot must not alias the device tensors
    assert torch.equal(h["x"][0], a0.cpu()) and torch.equal(h["x"][1][0], b.cpu())
    assert h["x"][1][1].item() == 5.0 and h["x"][1][1].dim() == 0 and h["y"]["n"] == 3
    assert torch.equal(h["y"]["z"], d) and h["y"]["z"].data_ptr() != d.data_ptr()
    assert h["x"][0].is_pinned()
    m = _HostSnapshot.materialize(h)
    for t in (m["x"][0], m["x"][1][0]):
        assert t.untyped_storage().nbytes() == t.numel() * t.element_size()
    buf = snap.buf
    snap.take(obj)
    assert snap.buf is buf  # reused across saves


def test_basic_llm_job_on_gpu(_rt, tmp_path):
    import pytorch_llm_ray as job
    res = job.main(["--workers", "1", "--preset", "tiny", "--batch", "8", "--seq", "128", "--data-scale", "0.01",
                    "--pvc", str(tmp_path), "--dtype", "bf16", "--max-windows", "2048"])
    assert res.metrics["loss"] < 5.0
    assert os.path.exists(os.path.join(res.checkpoint.path, "model.pth"))


def test_graph_decode_matches_eager_decode():
    """HIP-graph decode (one captured step replayed per token, device-side positions and KV
    lengths) produces the same tokens as the eager cached decode, incl. EOS trimming."""
    from gke_ray_train_amd.models import build_llama
    m = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=0)
    g = torch.Generator(device="cuda").manual_seed(4)
    ids = torch.randint(0, 512, (2, 37), device="cuda", generator=g)
    eager = m.generate(ids, max_new_tokens=40, use_graph=False)
    graph = m.generate(ids, max_new_tokens=40, use_graph=True)
    assert eager.shape == graph.shape == (2, 77)
    assert (eager == graph).float().mean().item() > 0.98, (eager[:, 37:], graph[:, 37:])
    eos = int(eager[0, 37 + 5])  # a token row 0 emits early: HF stops once every row has finished
    e2 = m.generate(ids, max_new_tokens=40, use_graph=False, eos_token_id=eos, pad_token_id=0)
    g2 = m.generate(ids, max_new_tokens=40, use_graph=True, eos_token_id=eos, pad_token_id=0, sync_every=7)
    assert e2.shape == g2.shape and (e2 == g2).float().mean().item() > 0.98


def test_sft_full_ft_overlapped_engine_matches_plain_path(tmp_path, monkeypatch):
    """Full fine-tuning through SFTTrainer on the bench's engine (AdamW per module on a side stream,
    overlapped with the next forward and writing W^T for the TN dX GEMMs; early per-bucket grad
    norm) gives the losses and parameters of the plain serial update (GRT_SFT_OVERLAP_OPT=0) to
    bf16 rounding, and the checkpoint layout is unchanged."""
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.parallel.overlap import OverlappedOptimizer
    from gke_ray_train_amd.trainer import SFTConfig, SFTTrainer
    rows = [{"text": "select a, b from t%d where c > %d order by b" % (i, 3 * i)} for i in range(48)]
    runs = []
    for overlap in ("1", "0"):
        monkeypatch.setenv("GRT_SFT_OVERLAP_OPT", overlap)
        torch.manual_seed(0)
        m = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=3)
        out = tmp_path / f"o{overlap}"
        tr = SFTTrainer(m, SFTConfig(output_dir=str(out), per_device_train_batch_size=2, gradient_accumulation_steps=2,
                                     learning_rate=1e-3, max_steps=6, logging_steps=2, save_steps=3,
                                     save_strategy="steps", max_seq_length=64, optim="adamw_torch",
                                     report_to="none", seed=1), train_dataset=rows)
        assert isinstance(tr.optimizer, OverlappedOptimizer) == (overlap == "1")
        res = tr.train()
        torch.cuda.synchronize()
        losses = [h["loss"] for h in tr.state["log_history"] if "loss" in h]
        runs.append((losses, {k: v.float().clone() for k, v in m.state_dict().items()}, res))
        ck = sorted(p.name for p in out.glob("checkpoint-*"))
        assert ck == ["checkpoint-3", "checkpoint-6"]
        assert {"optimizer.pt", "scheduler.pt", "trainer_state.json", "model.safetensors"} <= \
            {p.name for p in (out / "checkpoint-6").iterdir()}
    for a, b in zip(runs[0][0], runs[1][0]):
        assert abs(a - b) <= 2e-2 * abs(b), (runs[0][0], runs[1][0])
    for k, v in runs[1][1].items():
        d = (runs[0][1][k] - v).abs().max().item()
        assert d < 3e-2 * max(1.0, v.abs().max().item()), (k, d)
    assert runs[0][2].metrics["train_tokens_per_second"] > 0


def test_sft_full_ft_resume_on_gpu_matches_uninterrupted(tmp_path, monkeypatch):
    """Full fine-tuning on the overlapped engine, resumed from checkpoint-3 (per-parameter
    optimizer.pt loaded through load_portable_optimizer_state_dict into the device state) in a fresh
    trainer: steps 4-6 end at the parameters of the uninterrupted 6-step run to bf16 rounding (the
    stochastic-rounding bits and the first post-resume dX GEMM, NN until an update of this process
    registers W^T, differ), and far closer than a resume that drops the optimizer state (control)."""
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.parallel import DistributedDataParallel
    from gke_ray_train_amd.trainer import SFTConfig, SFTTrainer
    rows = [{"text": "select a, b from t%d where c > %d order by b" % (i, 3 * i)} for i in range(48)]

    def make(out):
        torch.manual_seed(0)
        m = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=3)
        tr = SFTTrainer(m, SFTConfig(output_dir=str(out), per_device_train_batch_size=2, gradient_accumulation_steps=2,
                                     learning_rate=1e-3, max_steps=6, logging_steps=2, save_steps=3,
                                     save_strategy="steps", max_seq_length=64, optim="adamw_torch",
                                     report_to="none", seed=1), train_dataset=rows)
        return m, tr

    ma, ta = make(tmp_path / "a")
    ta.train()
    torch.cuda.synchronize()
    ref = {k: v.float().clone() for k, v in ma.state_dict().items()}

    def resumed(out):
        m, tr = make(out)
        tr.train(resume_from_checkpoint=str(tmp_path / "a" / "checkpoint-3"))
        torch.cuda.synchronize()
        assert tr.state["global_step"] == 6
        return max((v.float() - ref[k]).abs().max().item() / max(1e-3, ref[k].abs().max().item())
                   for k, v in m.state_dict().items())

    worst = resumed(tmp_path / "b")
    monkeypatch.setattr(DistributedDataParallel, "load_portable_optimizer_state_dict", lambda self, opt, sd: None)
    worst_dropped = resumed(tmp_path / "c")
    assert worst <= 1e-2 and worst_dropped >= 4 * worst, (worst, worst_dropped)
