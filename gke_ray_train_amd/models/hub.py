"""HF-layout ``save_pretrained`` / ``from_pretrained`` for the Llama family (safetensors shards +
index, config.json, generation_config.json).

Reference: ``merged_model.save_pretrained(...)`` / ``model_to_save.save_pretrained(...)`` and
``AutoModelForCausalLM.from_pretrained(path, torch_dtype=bfloat16)``
(ray-jobs/fine_tune_llama_ray.py:54-60,353-355,373). Tensors are written with HF parameter names
(the fused q/k/v and gate/up projections are split at this boundary), so directories written here
load in HF transformers and real HF checkpoints load here.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch

from .llama import LlamaConfig, LlamaForCausalLM, get_config


def save_pretrained(model: LlamaForCausalLM, path: str, max_shard_bytes: int = 5 * 2 ** 30, dtype=None):
    from safetensors.torch import save_file
    os.makedirs(path, exist_ok=True)
    sd = {k: (v.to(dtype) if dtype else v).detach().contiguous().cpu() for k, v in model.hf_state_dict().items()}
    shards, cur, size = [], {}, 0
    for k in sorted(sd):
        nb = sd[k].numel() * sd[k].element_size()
        if cur and size + nb > max_shard_bytes:
            shards.append(cur)
            cur, size = {}, 0
        cur[k] = sd[k]
        size += nb
    if cur:
        shards.append(cur)
    weight_map = {}
    if len(shards) == 1:
        save_file(shards[0], os.path.join(path, "model.safetensors"), metadata={"format": "pt"})
    else:
        for i, sh in enumerate(shards):
            name = f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors"
            save_file(sh, os.path.join(path, name), metadata={"format": "pt"})
            for k in sh:
                weight_map[k] = name
        total = sum(v.numel() * v.element_size() for v in sd.values())
        with open(os.path.join(path, "model.safetensors.index.json"), "w") as f:
            json.dump({"metadata": {"total_size": total}, "weight_map": weight_map}, f, indent=2)
    cfg = model.config.to_hf_dict()
    if dtype is not None:
        cfg["torch_dtype"] = str(dtype).replace("torch.", "")
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(cfg, f, indent=2)
    with open(os.path.join(path, "generation_config.json"), "w") as f:
        json.dump({"bos_token_id": model.config.bos_token_id, "eos_token_id": model.config.eos_token_id,
                   "do_sample": False}, f, indent=2)


def config_from_hf_dict(d: dict, name: Optional[str] = None) -> LlamaConfig:
    fields = LlamaConfig.__dataclass_fields__
    kw = {k: v for k, v in d.items() if k in fields}
    if name is not None:
        kw["name"] = name
    return LlamaConfig(**kw)


def load_config(path: str) -> LlamaConfig:
    with open(os.path.join(path, "config.json")) as f:
        d = json.load(f)
    return config_from_hf_dict(d, os.path.basename(os.path.normpath(path)))


def from_pretrained(name_or_path: str, device=None, torch_dtype=torch.bfloat16, random_init_seed: Optional[int] = 0,
                    **overrides) -> LlamaForCausalLM:
    """Load an HF-layout directory; a known model id without local files gives the same
    architecture with random-init weights (no network on this machine)."""
    if os.path.isdir(name_or_path) and os.path.exists(os.path.join(name_or_path, "config.json")):
        from safetensors.torch import load_file
        cfg = load_config(name_or_path)
        for k, v in overrides.items():
            setattr(cfg, k, v)
        model = LlamaForCausalLM(cfg, device=device, dtype=torch_dtype)
        files = [f for f in os.listdir(name_or_path) if f.endswith(".safetensors")]
        sd = {}
        for fn in sorted(files):
            sd.update(load_file(os.path.join(name_or_path, fn)))
        model.load_hf_state_dict({k: v.to(torch_dtype) for k, v in sd.items()}, strict=True)
        return model
    cfg = get_config(name_or_path, **overrides)
    model = LlamaForCausalLM(cfg, device=device, dtype=torch_dtype)
    model.init_weights(random_init_seed)
    return model
