"""Distributed checkpointing: per-rank FSDP shards, offline consolidation to HF safetensors,
resharding on load, sharded optimizer state, and asynchronous (overlapped) snapshots.

Reference: rank 0 saves ``model.module.state_dict()`` / optimizer / scheduler ``.pth`` files into a
temp dir and reports ``Checkpoint.from_directory`` (ray-jobs/pytorch_llm_ray.py:296-305); the SFT
trainer writes ``checkpoint-<step>`` and ``save_pretrained`` at the end
(ray-jobs/fine_tune_llama_ray.py:315,354,373). SURVEY §5.4 targets for the rebuild: FSDP sharded
checkpoints (per-rank shard files + rank-0 consolidation to HF-style safetensors) for 7B / 70B and
async device->host copies so the hot loop is not blocked.

Layout of a sharded directory::

    fsdp_layout.json                         world, dtype, per-unit flat layout, model config
    shard-00000-of-00008.safetensors         rank 0: its slice of every unit + replicated 1-D params
    ...
    optim-00000-of-00008.safetensors         (optional) rank-local optimizer state (FusedAdamW)

Everything is safetensors / JSON: loading executes nothing from the files.
"""
from __future__ import annotations

import json
import os
import threading
from typing import Dict, Optional

import torch
import torch.distributed as dist

LAYOUT = "fsdp_layout.json"


def _shard_name(rank: int, world: int, kind: str = "shard") -> str:
    return f"{kind}-{rank:05d}-of-{world:05d}.safetensors"


def _atomic_save(tensors: Dict[str, torch.Tensor], path: str, metadata: Optional[dict] = None):
    from safetensors.torch import save_file
    tmp = path + ".tmp"
    save_file({k: v.contiguous() for k, v in tensors.items()}, tmp, metadata=metadata or {"format": "pt"})
    os.replace(tmp, path)


class AsyncCheckpointer:
    """Snapshot tensors to pinned host memory on a side HIP stream and write them from a thread.

    ``save()`` returns as soon as the copies are queued: the device->host transfer overlaps the
    following forward/backward (which only READ the parameters). Call ``fence()`` before anything
    that modifies the snapshotted tensors (the optimizer step): it makes the compute stream wait for
    the copies on the device, without a host sync. ``wait()`` joins the file write.
    """

    def __init__(self):
        self._thread: Optional[threading.Thread] = None
        self._pinned: Dict[str, torch.Tensor] = {}
        self._stream = None
        self._done = None
        self.error: Optional[BaseException] = None

    def save(self, tensors: Dict[str, torch.Tensor], path: str, metadata: Optional[dict] = None):
        self.wait()
        host = {}
        cuda = any(t.is_cuda for t in tensors.values())
        if cuda:
            if self._stream is None:
                self._stream = torch.cuda.Stream()
            snap = torch.cuda.Event()
            snap.record()
            self._stream.wait_event(snap)
            with torch.cuda.stream(self._stream):
                for k, t in tensors.items():
                    buf = self._pinned.get(k)
                    if buf is None or buf.shape != t.shape or buf.dtype != t.dtype:
                        buf = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                        self._pinned[k] = buf
                    buf.copy_(t.detach(), non_blocking=True)
                    host[k] = buf
            self._done = torch.cuda.Event()
            self._done.record(self._stream)
        else:
            host = {k: t.detach().clone() for k, t in tensors.items()}
            self._done = None
        done = self._done

        def work():
            try:
                if done is not None:
                    done.synchronize()
                _atomic_save(host, path, metadata)
            except BaseException as e:  # surfaced by wait()
                self.error = e
        self._thread = threading.Thread(target=work, daemon=True, name="grt-async-ckpt")
        self._thread.start()

    def fence(self):
        if self._done is not None:
            torch.cuda.current_stream().wait_event(self._done)

    def wait(self):
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self.error is not None:
            e, self.error = self.error, None
            raise e


# ------------------------------------------------------------------------------------- FSDP
def fsdp_layout(fsdp) -> dict:
    units = [{"names": u.names, "shapes": [list(s) for s in u.shapes], "offsets": u.offsets, "numels": u.numels,
              "shard_numel": u.shard_numel, "total": u.total} for u in fsdp.units]
    rep, off = [], 0
    for n, p in fsdp.replicated:
        rep.append({"name": n, "shape": list(p.shape), "offset": off})
        off += p.numel()
    cfg = getattr(fsdp.module, "config", None)
    cfg_d = cfg.to_hf_dict() if hasattr(cfg, "to_hf_dict") else None
    return {"world": fsdp.world, "dtype": str(fsdp.dtype).replace("torch.", ""), "units": units, "replicated": rep,
            "model_config": cfg_d, "format": "grt-fsdp-v1"}


def save_fsdp_sharded(fsdp, path: str, optimizer=None, async_ckpt: Optional[AsyncCheckpointer] = None):
    """Every rank writes its own shard file (1/world of the parameters); rank 0 writes the layout."""
    os.makedirs(path, exist_ok=True)
    tensors = {"shard_store": fsdp.shard_store, "rep_flat": fsdp.rep_flat}
    name = os.path.join(path, _shard_name(fsdp.rank, fsdp.world))
    if async_ckpt is not None:
        async_ckpt.save(tensors, name)
    else:
        _atomic_save({k: v.detach().cpu() for k, v in tensors.items()}, name)
    if optimizer is not None:
        save_optimizer_state(optimizer, os.path.join(path, _shard_name(fsdp.rank, fsdp.world, "optim")))
    if fsdp.rank == 0:
        tmp = os.path.join(path, LAYOUT + ".tmp")
        with open(tmp, "w") as f:
            json.dump(fsdp_layout(fsdp), f)
        os.replace(tmp, os.path.join(path, LAYOUT))
    if async_ckpt is not None:
        async_ckpt.wait()
    if fsdp.world > 1:
        dist.barrier(group=fsdp.pg)


def _read_layout(path: str) -> dict:
    with open(os.path.join(path, LAYOUT)) as f:
        return json.load(f)


def _read_shards(path: str, layout: dict):
    from safetensors.torch import load_file
    W = layout["world"]
    return [load_file(os.path.join(path, _shard_name(r, W))) for r in range(W)]


def consolidate_fsdp_checkpoint(path: str) -> Dict[str, torch.Tensor]:
    """Full (unsharded) state dict with module parameter names, on CPU, from a sharded directory —
    offline, no process group needed."""
    layout = _read_layout(path)
    shards = _read_shards(path, layout)
    out, base = {}, 0
    for u in layout["units"]:
        per = u["shard_numel"]
        full = torch.cat([sh["shard_store"][base:base + per] for sh in shards])
        for n, shp, o, k in zip(u["names"], u["shapes"], u["offsets"], u["numels"]):
            out[n] = full[o:o + k].view(shp).clone()
        base += per
    rep = shards[0]["rep_flat"]
    for r in layout["replicated"]:
        k = 1
        for s in r["shape"]:
            k *= s
        out[r["name"]] = rep[r["offset"]:r["offset"] + k].view(r["shape"]).clone()
    return out


def load_fsdp_sharded(fsdp, path: str, optimizer=None):
    """Load a sharded directory into ``fsdp``. Same world size: each rank reads only its file;
    different world size: the units are reassembled and re-sliced (resharding)."""
    from safetensors.torch import load_file
    layout = _read_layout(path)
    if layout["world"] == fsdp.world and [u.names for u in fsdp.units] == [u["names"] for u in layout["units"]]:
        sd = load_file(os.path.join(path, _shard_name(fsdp.rank, fsdp.world)))
        with torch.no_grad():
            fsdp.shard_store.copy_(sd["shard_store"])
            fsdp.rep_flat[:sd["rep_flat"].numel()].copy_(sd["rep_flat"])
        if optimizer is not None:
            opt_file = os.path.join(path, _shard_name(fsdp.rank, fsdp.world, "optim"))
            if os.path.exists(opt_file):
                load_optimizer_state(optimizer, opt_file)
    else:
        fsdp.load_full_state_dict(consolidate_fsdp_checkpoint(path))


def export_hf(path: str, out_dir: str, dtype=torch.bfloat16):
    """Consolidate a sharded Llama checkpoint and write it as an HF ``save_pretrained`` directory."""
    from ..models.hub import save_pretrained
    from ..models.llama import LlamaConfig, LlamaForCausalLM
    layout = _read_layout(path)
    cfg_d = layout.get("model_config")
    if not cfg_d:
        raise ValueError("checkpoint has no model config: cannot build the HF layout")
    from ..models.hub import config_from_hf_dict
    cfg: LlamaConfig = config_from_hf_dict(cfg_d)
    sd = consolidate_fsdp_checkpoint(path)
    model = LlamaForCausalLM(cfg, device="meta", dtype=dtype)
    model.load_state_dict({k: v.to(dtype) for k, v in sd.items() if not k.endswith("inv_freq")}, strict=False,
                          assign=True)
    save_pretrained(model, out_dir, dtype=dtype)
    return out_dir


# ------------------------------------------------------------------------------------- optimizer
def save_optimizer_state(optimizer, path: str):
    """Rank-local optimizer state (FusedAdamW / torch AdamW layout) -> safetensors + scalars."""
    tensors, meta = {}, {"groups": []}
    for gi, g in enumerate(optimizer.param_groups):
        meta["groups"].append({k: v for k, v in g.items() if k != "params" and isinstance(v, (int, float, tuple, list))})
        for pi, p in enumerate(g["params"]):
            st = optimizer.state.get(p, {})
            for k, v in st.items():
                if isinstance(v, torch.Tensor):
                    tensors[f"{gi}.{pi}.{k}"] = v.detach().cpu() if v.dim() > 0 else v.detach().cpu().reshape(1)
    _atomic_save(tensors, path, metadata={"format": "pt", "grt_optim": json.dumps(meta)})


def load_optimizer_state(optimizer, path: str):
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        meta = json.loads(f.metadata().get("grt_optim", "{}"))
        keys = list(f.keys())
        for key in keys:
            gi, pi, name = key.split(".", 2)
            p = optimizer.param_groups[int(gi)]["params"][int(pi)]
            t = f.get_tensor(key)
            st = optimizer.state.setdefault(p, {})
            if name == "step":
                st[name] = t.reshape(())
            elif name in ("exp_avg", "exp_avg_sq") and getattr(optimizer, "_host_states", False):
                st[name] = t.pin_memory() if torch.cuda.is_available() else t
            else:
                st[name] = t.to(p.device)
    for g, gm in zip(optimizer.param_groups, meta.get("groups", [])):
        for k, v in gm.items():
            g[k] = tuple(v) if isinstance(g.get(k), tuple) else v
