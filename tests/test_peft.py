"""LoRA / QLoRA on the fused-projection Llama: trainable-parameter count (reference r=64 on 7
targets -> 167,772,160 for Llama-3.1-8B), zero-init equivalence, merge_and_unload equivalence,
adapter save/load with PEFT names, NF4 quantisation (CPU reference path)."""
import torch

from gke_ray_train_amd.models import build_llama, get_config
from gke_ray_train_amd.peft import BitsAndBytesConfig, LoraConfig, get_peft_model, quantize_model_

TARGETS = ["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"]


def _count_expected(cfg, r):
    d, f, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    q, kv = cfg.num_attention_heads * hd, cfg.num_key_value_heads * hd
    per = r * ((d + q) + 2 * (d + kv) + (q + d) + 2 * (d + f) + (f + d))
    return per * cfg.num_hidden_layers


def test_reference_trainable_param_count():
    # SURVEY/BASELINE: 167,772,160 LoRA params for Llama-3.1-8B at r=64 on all 7 projections
    assert _count_expected(get_config("llama3.1-8b"), 64) == 167_772_160


def test_lora_zero_init_merge_and_roundtrip(tmp_path):
    torch.manual_seed(0)
    m = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32, seed=1)
    ids = torch.randint(0, 512, (2, 24))
    ref = m(ids)["logits"].detach()
    pm = get_peft_model(m, LoraConfig(r=8, lora_alpha=16, lora_dropout=0.0, target_modules=TARGETS))
    t, _ = pm.print_trainable_parameters()
    assert t == _count_expected(m.config, 8)
    assert torch.allclose(pm(ids)["logits"], ref, atol=1e-5)  # B = 0 at init
    with torch.no_grad():
        for lm in pm.lora_modules.values():
            for p in lm.lora_B.values():
                p.normal_(0, 0.02)
    out = pm(ids)["logits"].detach()
    assert not torch.allclose(out, ref, atol=1e-4)
    # training signal reaches only the adapters
    loss = pm(ids, labels=ids)["loss"]
    loss.backward()
    assert all((p.grad is not None) == p.requires_grad for p in pm.parameters())
    pm.save_pretrained(str(tmp_path / "adapter"))
    keys = set(pm.adapter_state_dict())
    assert "base_model.model.model.layers.0.self_attn.q_proj.lora_A.weight" in keys
    assert "base_model.model.model.layers.1.mlp.down_proj.lora_B.weight" in keys
    m2 = build_llama("llama-tiny-gqa", device="cpu", dtype=torch.float32, seed=1)
    pm2 = get_peft_model(m2, LoraConfig(r=8, lora_alpha=16, target_modules=TARGETS))
    pm2.load_adapter(str(tmp_path / "adapter"))
    assert torch.allclose(pm2(ids)["logits"], out, atol=1e-5)
    merged = pm.merge_and_unload()
    assert torch.allclose(merged(ids)["logits"], out, atol=1e-4)
    assert not any("lora" in n for n in merged.state_dict())
    hf = merged.hf_state_dict()
    assert "model.layers.0.self_attn.q_proj.weight" in hf and "model.layers.0.mlp.up_proj.weight" in hf


def test_qlora_nf4_cpu():
    torch.manual_seed(0)
    m = build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=2)
    ids = torch.randint(0, 512, (2, 16))
    ref = m(ids)["logits"].detach()
    quantize_model_(m, BitsAndBytesConfig(bnb_4bit_compute_dtype=torch.float32))
    q = m(ids)["logits"].detach()
    rel = (q - ref).norm() / ref.norm()
    assert rel < 0.2, rel
    pm = get_peft_model(m, LoraConfig(r=4, lora_alpha=8, target_modules=TARGETS))
    loss = pm(ids, labels=ids)["loss"]
    loss.backward()
    n_grads = sum(1 for p in pm.parameters() if p.grad is not None)
    assert n_grads == sum(1 for p in pm.parameters() if p.requires_grad) > 0
    merged = pm.merge_and_unload()
    assert torch.allclose(merged(ids)["logits"], pm(ids)["logits"], atol=1e-4)


def test_double_quant_close_to_single():
    torch.manual_seed(0)
    m1 = build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=3)
    m2 = build_llama("llama-tiny", device="cpu", dtype=torch.float32, seed=3)
    quantize_model_(m1, BitsAndBytesConfig(bnb_4bit_compute_dtype=torch.float32))
    quantize_model_(m2, BitsAndBytesConfig(bnb_4bit_compute_dtype=torch.float32, bnb_4bit_use_double_quant=True))
    ids = torch.randint(0, 512, (1, 16))
    a, b = m1(ids)["logits"], m2(ids)["logits"]
    assert (a - b).norm() / a.norm() < 0.02


def test_attention_dropout_reference_mask_statistics():
    """CPU reference of the kernel's counter-hash dropout: keep-rate ~ 1-p, deterministic in the
    seed, different across seeds, and the expectation of dropped attention equals no dropout."""
    import torch
    from gke_ray_train_amd.ops import _ref
    keep = _ref.attn_dropout_keep(7, 2, 3, 64, 64, 0.25)
    assert abs(keep.float().mean().item() - 0.75) < 0.02
    assert torch.equal(keep, _ref.attn_dropout_keep(7, 2, 3, 64, 64, 0.25))
    assert not torch.equal(keep, _ref.attn_dropout_keep(8, 2, 3, 64, 64, 0.25))
    q = torch.randn(1, 32, 2, 16)
    k = torch.randn(1, 32, 2, 16)
    v = torch.randn(1, 32, 2, 16)
    base = _ref.attention(q, k, v, causal=True)
    avg = torch.stack([_ref.attention(q, k, v, causal=True, dropout_p=0.2, seed=s) for s in range(400)]).mean(0)
    assert (avg - base).abs().max().item() < 0.15


def test_nf4_dequant_cache_cpu():
    import torch
    import torch.nn as nn
    from gke_ray_train_amd.peft import BitsAndBytesConfig
    from gke_ray_train_amd.peft.quant import NF4Linear, set_dequant_cache
    torch.manual_seed(0)
    lin = nn.Linear(128, 64, bias=False)
    q = NF4Linear.from_linear(lin, BitsAndBytesConfig(bnb_4bit_compute_dtype=torch.float32))
    model = nn.Sequential(q)
    assert set_dequant_cache(model, "auto") is False  # CPU: auto keeps the transient path
    w0 = q.dequantize()
    assert set_dequant_cache(model, "1") is True
    w1 = q.dequantize()
    assert q.dequantize() is w1  # resident
    torch.testing.assert_close(w0, w1, rtol=0, atol=0)
    dy = torch.randn(3, 64)
    torch.testing.assert_close(q.input_grad(dy), dy @ w0)
    q.qweight.add_(0)  # packed weights rewritten -> cache invalidated
    assert q.dequantize() is not w1
    assert q.weight is not q.dequantize()  # the public view is a copy
    set_dequant_cache(model, "0")
    assert q._w_cache is None
