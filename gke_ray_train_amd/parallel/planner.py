"""Per-rank HBM / host memory preflight for a training configuration.

Not in the reference (its 16 x H100 jobs never size anything); required so BASELINE.json config #5
(Llama-3-70B FSDP full-shard + CPU offload on 8 x MI355X) either fits
by construction or is refused up front with the numbers, instead of dying mid-step with an
allocator error or the host OOM killer.

The plan mirrors what the engines actually allocate:
* DDP (``parallel/ddp.py``): flat bf16 parameters + flat gradient buffer on every rank; ZeRO adds
  a 1/world gradient shard and shrinks the fp32 AdamW moments to 1/world; the one-GPU overlapped
  optimizer keeps W^T of every projection (``adamw_t``);
* FSDP (``parallel/fsdp.py``): the 1/world parameter + gradient shard stores, the root unit's
  gathered parameters and gradients (alive for the whole step), ONE prefetched decoder unit beside
  the running one, and ``1 + GRT_FSDP_RS_INFLIGHT`` full-unit gradient buffers; the partition is
  computed by ``fsdp.partition_units`` on a meta-device model, so unit sizes are exact;
* ``offload``: the fp32 moments (8 B / parameter of the shard) move to pinned host memory — the
  whole node needs ``world x`` that in RAM — and HBM keeps 3 staging chunks;
* activations: the tensors the Llama layer saves for backward (7h + 3 kv + 3 F bf16 values per
  token per layer: block input, normed inputs, fused qkv output, rotated q/k, attention output,
  mid residual, fused gate/up output, SwiGLU output); with activation checkpointing only the
  block inputs plus one recomputed layer;
* a fixed reserve for RCCL channels, hipBLASLt workspaces and allocator fragmentation.
"""
from __future__ import annotations

import math
import os
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional

GiB = float(1 << 30)
MI355X_HBM_BYTES = 288 * 10 ** 9  # 288 GB HBM3E per GPU
RESERVE_BYTES = 6 * (1 << 30)      # RCCL buffers, BLAS workspaces, allocator slack


@dataclass
class MemoryPlan:
    model: str
    world: int
    parallel: str
    offload: bool
    peft: str
    hbm_per_rank: Dict[str, float] = field(default_factory=dict)   # bytes by component
    host_per_rank: Dict[str, float] = field(default_factory=dict)
    hbm_capacity: float = MI355X_HBM_BYTES
    host_capacity: Optional[float] = None                          # node RAM available (bytes)
    units: Optional[Dict[str, float]] = None                       # FSDP partition facts
    # ranks whose host memory THIS machine holds for the run at hand: world on a real node, 1 for a
    # one-process proxy of rank 0 (bench.py --proxy-world); host_total_node always covers every rank
    host_ranks_here: Optional[int] = None

    @property
    def hbm_total(self) -> float:
        return sum(self.hbm_per_rank.values())

    @property
    def host_total_node(self) -> float:
        return sum(self.host_per_rank.values()) * self.world

    def problems(self) -> List[str]:
        out = []
        if self.hbm_total > self.hbm_capacity:
            out.append(f"HBM: needs {self.hbm_total / GiB:.1f} GiB per rank, the GPU has "
                       f"{self.hbm_capacity / GiB:.1f} GiB ({self._top(self.hbm_per_rank)})")
        here = self.host_ranks_here if self.host_ranks_here is not None else self.world
        need = sum(self.host_per_rank.values()) * here
        if self.host_capacity is not None and need > self.host_capacity:
            out.append(f"host RAM: needs {need / GiB:.1f} GiB pinned across {here} ranks, "
                       f"{self.host_capacity / GiB:.1f} GiB available ({self._top(self.host_per_rank)} per rank)")
        return out

    @property
    def fits(self) -> bool:
        return not self.problems()

    @staticmethod
    def _top(d):
        return ", ".join(f"{k} {v / GiB:.1f}" for k, v in sorted(d.items(), key=lambda kv: -kv[1])[:4])

    def to_dict(self) -> dict:
        d = asdict(self)
        d["hbm_total_gib"] = round(self.hbm_total / GiB, 2)
        d["host_total_node_gib"] = round(self.host_total_node / GiB, 2)  # every rank of the job
        d["host_per_rank_gib"] = round(sum(self.host_per_rank.values()) / GiB, 2)
        d["host_capacity_gib"] = None if self.host_capacity is None else round(self.host_capacity / GiB, 1)
        d["host_fits_full_node"] = self.host_capacity is None or self.host_total_node <= self.host_capacity
        d["fits"] = self.fits
        d["problems"] = self.problems()
        return d


def host_available_bytes() -> Optional[float]:
    """MemAvailable, or ``GRT_HOST_MEM_GB`` when the job's share of the node is capped below it."""
    cap = os.environ.get("GRT_HOST_MEM_GB")
    if cap:
        return float(cap) * GiB
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    return float(line.split()[1]) * 1024
    except OSError:
        pass
    return None


def hbm_capacity_bytes(device_index: int = 0) -> float:
    try:
        import torch
        if torch.cuda.is_available():
            return float(torch.cuda.get_device_properties(device_index).total_memory)
    except Exception:
        pass
    return float(MI355X_HBM_BYTES)


def activation_bytes(cfg, tokens: int, checkpointing: bool, dtype_bytes: int = 2) -> float:
    h, f, L = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers
    kv = cfg.num_key_value_heads * cfg.head_dim
    per_layer_tok = (7 * h + 3 * kv + 3 * f) * dtype_bytes
    if checkpointing:
        return tokens * (L * h * dtype_bytes + per_layer_tok)
    # + the final norm input / LM-head chunk of the fused cross-entropy (bounded chunk)
    return tokens * (L * per_layer_tok + 2 * h * dtype_bytes) + min(tokens, 4096) * cfg.vocab_size * dtype_bytes


def plan_memory(cfg, world: int, parallel: str = "ddp", offload: bool = False, peft: str = "none",
                micro_batch: int = 8, seq: int = 1024, zero: Optional[bool] = None, checkpointing: bool = False,
                lora_r: int = 64, overlap_opt: Optional[bool] = None, hbm_capacity: Optional[float] = None,
                host_capacity: Optional[float] = None, offload_chunk_elems: int = 1 << 26,
                lora_dropout: float = 0.1, lora_kcat: Optional[bool] = None) -> MemoryPlan:
    """Per-rank memory plan for ``cfg`` (a ``LlamaConfig``) at ``world`` ranks."""
    P = float(cfg.num_params())
    B = 2.0  # bf16 parameters / gradients
    plan = MemoryPlan(cfg.name, world, parallel, offload, peft,
                      hbm_capacity=hbm_capacity if hbm_capacity is not None else hbm_capacity_bytes(),
                      host_capacity=host_capacity if host_capacity is not None else host_available_bytes())
    hbm, host = plan.hbm_per_rank, plan.host_per_rank
    tokens = micro_batch * seq
    hbm["activations"] = activation_bytes(cfg, tokens, checkpointing)
    hbm["reserve"] = RESERVE_BYTES
    if parallel == "fsdp":
        from ..models.llama import LlamaForCausalLM
        from .fsdp import partition_units
        import torch
        meta = LlamaForCausalLM(cfg, device="meta", dtype=torch.bfloat16)
        units, replicated = partition_units(meta, world)
        root = [u for u in units if u.module is meta]
        blocks = [u for u in units if u.module is not meta]
        big = max((u.total for u in blocks), default=0)
        root_total = sum(u.total for u in root)
        shard = sum(u.shard_numel for u in units)
        rep = sum(p.numel() for _, p in replicated)
        inflight = int(os.environ.get("GRT_FSDP_RS_INFLIGHT", "2"))
        comm = world > 1
        hbm["param_shards"] = shard * B + rep * B
        hbm["grad_shards"] = shard * B + rep * B
        hbm["gathered_params"] = (2 * big + root_total) * B if comm else 0.0
        hbm["unit_grad_buffers"] = ((1 + inflight) * big + root_total) * B
        opt = 8.0 * (shard + rep)
        if offload:
            host["adam_moments_fp32"] = 8.0 * shard
            hbm["adam_moments_fp32"] = 8.0 * rep + 2 * 3 * min(offload_chunk_elems, shard) * 4.0
        else:
            hbm["adam_moments_fp32"] = opt
        plan.units = {"decoder_units": len(blocks), "root_units": len(root),
                      "block_params": float(blocks[0].total if blocks else 0),
                      "block_shard_params": float(blocks[0].shard_numel if blocks else 0),
                      "root_params": float(root_total), "replicated_params": float(rep),
                      "peak_gathered_bytes": (2 * big + root_total) * B}
        return plan
    # DDP (replicated parameters)
    if peft in ("lora", "qlora"):
        h, f = cfg.hidden_size, cfg.intermediate_size
        kvd = cfg.num_key_value_heads * cfg.head_dim
        L, r = cfg.num_hidden_layers, lora_r
        t = L * r * (  # A [r, in] + B [out, r] for q, k, v, o, gate, up, down
            (h + h) * 2 + (h + kvd) * 2 + (h + f) * 3)
        lin = L * (h * (h * 2 + 2 * kvd) + 3 * h * f)
        # adapted modules per layer (peft/lora.py LoraLinear on the fused projections):
        # (out_features, R = r x targets): qkv, o, gate_up, down
        mods = [(h + 2 * kvd, 3 * r), (h, r), (2 * f, 2 * r), (h, r)]
        kcat = (r % 64 == 0 and h % 128 == 0 and f % 128 == 0 and os.environ.get("GRT_LORA_KCAT", "1") != "0") \
            if lora_kcat is None else lora_kcat
        tails = L * sum(o * R for o, R in mods)
        cached = True
        if peft == "qlora":  # NF4 codes (0.5 B) + fp32 absmax per 64
            hbm["frozen_nf4_codes"] = lin * (0.5 + 4.0 / 64)
            # peft/quant.py set_dequant_cache: the resident bf16 W / W^T exist only when the cache is
            # on ("auto": 4 B per base parameter within 15 % of the device's HBM — 8B yes, 70B no).
            # Without it each projection is dequantised per use: into a transient K-concatenated W'
            # (peft/lora.py _kcat_weight_streamed) in the forward, as W^T in the backward
            mode = os.environ.get("GRT_NF4_CACHE", "auto")
            cap = plan.hbm_capacity if math.isfinite(plan.hbm_capacity) else float(MI355X_HBM_BYTES)
            cached = (4.0 * lin <= 0.15 * cap) if mode == "auto" else mode not in ("0", "off", "false")
            kcat = kcat and (cached or os.environ.get("GRT_NF4_STREAM_KCAT", "1") != "0")
        hbm["frozen_unadapted"] = (P - lin) * B  # embeddings, LM head, norms
        if not cached:
            # transient per-use dequantisation: the largest projection's W' (forward) and W^T (backward)
            hbm["nf4_dequant_scratch"] = 2 * h * max(2 * f, h + 2 * kvd) * B
            if kcat and r == 64:
                hbm["lora_bt"] = tails * B
        elif kcat:
            # K-concatenated W' = [W | B blocks] (bf16; for LoRA the base weight is a view of it, for
            # QLoRA it replaces the dequant cache) + the B^T buffer of the adapter-gradient kernel
            hbm["frozen_kcat_weight"] = (lin + tails) * B
            hbm["lora_bt"] = tails * B if r == 64 else 0.0
        else:
            hbm["frozen_base"] = lin * B  # bf16 weight, or the resident NF4 dequant cache
        if cached:
            hbm["frozen_base_transposed"] = lin * B  # cached W^T of the TN dX GEMMs (both peft kinds)
        hbm["adapters"] = t * B
        hbm["adapter_grads"] = t * B
        hbm["adam_moments_fp32"] = 8.0 * t
        # adapter activations: the h' tails of the [x | h'] rows. The dropped inputs x_d kept for dA
        # take the place of the adapted projections' inputs, which the frozen base no longer saves
        # for weight gradients (both are in `activations`)
        hbm["adapter_activations"] = tokens * L * sum(R for _, R in mods) * B
        return plan
    zero = (world > 1) if zero is None else zero
    hbm["params"] = P * B
    hbm["grads"] = P * B
    if zero:
        hbm["grad_shard"] = P * B / world
        hbm["param_shard"] = P * B / world  # the contiguous shard the sharded AdamW updates
        opt = 8.0 * P / world
    else:
        opt = 8.0 * P
    if offload:
        host["adam_moments_fp32"] = opt
        hbm["adam_moments_fp32"] = 2 * 3 * offload_chunk_elems * 4.0
    else:
        hbm["adam_moments_fp32"] = opt
    overlap = (world == 1 and not zero) if overlap_opt is None else overlap_opt
    if overlap or zero:  # W^T of the projection weights (adamw_t, or the ZeRO forward transposes)
        hbm["weight_transposes"] = (P - 2 * cfg.vocab_size * cfg.hidden_size) * B
    return plan


def preflight(plan: MemoryPlan) -> None:
    """Raise a clear error when the plan does not fit."""
    probs = plan.problems()
    if probs:
        raise MemoryError(f"{plan.model} {plan.parallel} world={plan.world} offload={plan.offload} does not fit: "
                          + "; ".join(probs))
