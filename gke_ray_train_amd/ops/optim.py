"""Fused AdamW + device-side gradient clipping on the gfx950 kernels.

``FusedAdamW`` is a drop-in ``torch.optim.Optimizer`` (state_dict layout compatible with
``torch.optim.AdamW``: ``exp_avg`` / ``exp_avg_sq`` / ``step`` per parameter). On GPU every
parameter tensor is updated by ONE HIP kernel pass; the data-parallel engines hand it a single
flat parameter per dtype/decay group, so a whole 7B model updates in one launch.

Gradient clipping never synchronises with the host: ``clip_grad_norm_`` leaves the global
norm and the clip coefficient in a device buffer that the AdamW kernel reads directly
(reference ``clip_grad_norm_(…, 1.0)``/``max_grad_norm``: ray-jobs/pytorch_llm_ray.py:277,
ray-jobs/fine_tune_config.json:19).
"""
from __future__ import annotations

import math
import os
from typing import Iterable, Optional

import torch

from .. import _native
from . import _ref


class GradClipState:
    """Device scalars produced by clip_grad_norm_: buf[0] = global norm, buf[1] = grad scale."""

    def __init__(self, device):
        self.buf = torch.ones(2, device=device, dtype=torch.float32)

    @property
    def norm(self) -> torch.Tensor:
        return self.buf[0]


_ws_cache: dict = {}


def clip_grad_norm_(params_or_grads: Iterable, max_norm: float, prescale: float = 1.0,
                    state: Optional[GradClipState] = None, apply: bool = False) -> GradClipState:
    """Global L2 norm of all grads (times ``prescale``) and clip coefficient, on device.

    With ``apply=False`` (the fused path) grads are left untouched and the coefficient is
    consumed by ``FusedAdamW.step(grad_scale=state)``; ``apply=True`` scales grads in place
    (torch semantics) for optimizers that are not fused.
    """
    grads = []
    for t in params_or_grads:
        g = t.grad if isinstance(t, torch.nn.Parameter) or (isinstance(t, torch.Tensor) and t.grad is not None) else t
        if g is not None:
            grads.append(g)
    if not grads:
        dev = torch.device("cpu")
        st = state or GradClipState(dev)
        st.buf.fill_(1.0)
        st.buf[0] = 0.0
        return st
    dev = grads[0].device
    st = state or GradClipState(dev)
    if dev.type == "cuda":
        C = _native.kernels()
        nb = C.sumsq_blocks()
        key = (dev, len(grads))
        ws = _ws_cache.get(key)
        if ws is None:
            ws = torch.empty(len(grads) * nb, device=dev, dtype=torch.float32)
            _ws_cache[key] = ws
        for i, g in enumerate(grads):
            C.sumsq(g.contiguous() if not g.is_contiguous() else g, ws, i)
        C.clip_finalize(ws, len(grads) * nb, float(max_norm), float(prescale), st.buf)
        if apply:
            for g in grads:
                C.scale_(g, 1.0, st.buf[1:2])
    else:
        total = torch.stack([g.float().pow(2).sum() for g in grads]).sum().sqrt() * prescale
        coef = torch.clamp(max_norm / (total + 1e-6), max=1.0) if max_norm > 0 else torch.ones(())
        st.buf[0] = total
        st.buf[1] = coef * prescale
        if apply:
            for g in grads:
                g.mul_(st.buf[1].to(g.dtype))
    return st


# Hyper-parameter uploads (lr, betas, bias corrections, ...) go through a small ring of pinned host
# buffers: a pageable torch.tensor(...) -> device copy is a blocking hipMemcpy that waits for the
# stream, i.e. a host-device sync inside every optimizer step. A ring slot is reused only after the
# event of its previous copy completed (normally long before).
_PINNED_HYPER: dict = {}


def upload_hyper(hb: torch.Tensor, values) -> None:
    """hb (10 fp32 on the device) <- values, asynchronously on the current stream."""
    if hb.device.type != "cuda":
        hb.copy_(torch.tensor(values, dtype=torch.float32))
        return
    values = [float(v) for v in values]
    key = (hb.data_ptr(), hb.device.index)
    ring = _PINNED_HYPER.get(key)
    if ring is None:
        ring = _PINNED_HYPER[key] = [[torch.empty(hb.numel(), dtype=torch.float32, pin_memory=True), None]
                                     for _ in range(4)] + [0]
    if getattr(hb, "_grt_hyper", None) == values:  # this buffer already holds them (one upload per step)
        return
    hb._grt_hyper = values
    i = ring[-1]
    ring[-1] = (i + 1) % 4
    buf, ev = ring[i]
    if ev is not None:
        ev.synchronize()
    buf.numpy()[:] = values
    hb.copy_(buf, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    ring[i][1] = ev


# Bumped by every framework optimizer step. The fused kernels write parameters through raw device
# pointers, which does not advance a tensor's autograd version counter, so caches derived from
# trainable parameters (peft/lora.py's K-concatenated W' tail) key on this as well as on _version.
_PARAM_GENERATION = 0


def param_generation() -> int:
    return _PARAM_GENERATION


def bump_param_generation() -> None:
    global _PARAM_GENERATION
    _PARAM_GENERATION += 1


class FusedAdamW(torch.optim.Optimizer):
    """AdamW with fp32 moments; bf16 or fp32 params (optionally with an fp32 master copy).

    ``name`` aliases accepted by the trainer: ``adamw_torch``, ``adamw_32bit``,
    ``paged_adamw_32bit`` (the reference's OPTIM, ray-jobs/fine_tune_config.json:17 — paging is
    unnecessary with 288 GB of HBM, the states simply stay resident).
    """

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                 master_weights: bool = False, stochastic_rounding: Optional[bool] = None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.master_weights = master_weights
        # bf16 params without a master copy (the reference's paged_adamw_32bit on a bf16 model):
        # stochastic rounding of the update by default (GRT_ADAMW_SR=0 -> round to nearest)
        if stochastic_rounding is None:
            stochastic_rounding = os.environ.get("GRT_ADAMW_SR", "1") != "0"
        self.stochastic_rounding = bool(stochastic_rounding)
        self._hyper = {}

    def _hyper_buf(self, dev, key):
        hb = self._hyper.get((dev, key))
        if hb is None:
            hb = torch.empty(10, dtype=torch.float32, device=dev)
            self._hyper[(dev, key)] = hb
        return hb

    def _sr(self) -> float:
        return 1.0 if self.stochastic_rounding and not self.master_weights else 0.0

    _host_states = False  # OffloadedAdamW: moments live in pinned host memory

    def _state_tensor(self, v: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
        """A loaded moment / master copy in the layout the fused kernels take: fp32, contiguous,
        on the parameter's device (pinned host memory for the offloaded optimizers)."""
        v = v.detach().to(torch.float32, copy=True)  # never alias the state dict's tensors
        if self._host_states:
            v = v.cpu().contiguous()
            return v.pin_memory() if torch.cuda.is_available() else v
        return v.to(p.device).contiguous()

    def load_state_dict(self, state_dict):
        """torch.optim.Optimizer.load_state_dict casts floating state to the parameter's dtype and
        device — bf16 on the GPU for a bf16 model — which would drop the moments to bf16 (and put
        an offloaded optimizer's host state in HBM). Restore them from the checkpoint's own tensors
        in fp32 after the base class has mapped the parameters."""
        super().load_state_dict(state_dict)
        idmap = {}
        for g, sg in zip(self.param_groups, state_dict["param_groups"]):
            for p, pid in zip(g["params"], sg["params"]):
                idmap[pid] = p
        for pid, sst in state_dict["state"].items():
            p = idmap.get(pid)
            if p is None:
                continue
            st = self.state[p]
            for k in ("exp_avg", "exp_avg_sq", "master"):
                v = sst.get(k)
                if isinstance(v, torch.Tensor):
                    st[k] = self._state_tensor(v, p)
            if isinstance(st.get("step"), torch.Tensor):
                st["step"] = st["step"].detach().to("cpu", torch.float32, copy=True).reshape(())

    def _init_state(self, p):
        st = self.state[p]
        if len(st) == 0:
            st["step"] = torch.tensor(0.0)
            st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
            st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
            if self.master_weights and p.dtype != torch.float32:
                st["master"] = p.detach().float().contiguous()
        return st

    @torch.no_grad()
    def prepare_gpu_step(self):
        """Bump the step counters and upload each group's hyper-parameters (current stream);
        returns [(p, grad, exp_avg, exp_avg_sq, master, hyper)] for the caller to launch the
        update kernels on (views of) these tensors — used by the overlapped optimizer."""
        out = []
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None or not p.is_cuda:
                    continue
                st = self._init_state(p)
                st["step"] += 1
                step = float(st["step"])
                hb = self._hyper_buf(p.device, (gi,))
                upload_hyper(hb, [group["lr"], b1, b2, group["eps"], group["weight_decay"], 1.0 - b1 ** step,
                                  1.0 - b2 ** step, 1.0, self._sr(), step])
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                out.append((p, g, st["exp_avg"], st["exp_avg_sq"], st.get("master"), hb))
        return out

    @torch.no_grad()
    def step(self, closure=None, grad_scale: Optional[GradClipState] = None):
        bump_param_generation()
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            lr = group["lr"]
            b1, b2 = group["betas"]
            eps, wd = group["eps"], group["weight_decay"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self._init_state(p)
                st["step"] += 1
                step = float(st["step"].item()) if st["step"].device.type == "cpu" else float(st["step"])
                bc1 = 1.0 - b1 ** step
                bc2 = 1.0 - b2 ** step
                master = st.get("master")
                if p.is_cuda:
                    hb = self._hyper_buf(p.device, (gi,))
                    upload_hyper(hb, [lr, b1, b2, eps, wd, bc1, bc2, 1.0, self._sr(), step])
                    g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                    _native.kernels().adamw(p.data, g, st["exp_avg"], st["exp_avg_sq"], master, hb,
                                            None if grad_scale is None else grad_scale.buf)
                else:
                    gs = 1.0 if grad_scale is None else float(grad_scale.buf[1])
                    _ref.adamw_(p.data, p.grad, st["exp_avg"], st["exp_avg_sq"], step, lr, b1, b2, eps, wd,
                                grad_scale=gs, master=master)
        return loss


class OffloadedAdamW(FusedAdamW):
    """AdamW whose fp32 moments live in pinned HOST memory and stream through the GPU kernel.

    For FSDP + CPU offload (BASELINE config #5): per step each chunk of (m, v) is copied H2D on a
    side stream, updated by the same fused HIP AdamW kernel together with the HBM-resident
    parameter / gradient shard, and copied back D2H, with chunk i+1's upload and chunk i-1's
    download overlapping chunk i's update (two device staging slots). HBM holds only
    2 x chunk x 8 bytes of optimizer state instead of 8 bytes per parameter.
    """

    _host_states = True  # checkpoint loaders keep exp_avg / exp_avg_sq in pinned host memory

    def __init__(self, params, chunk_elems: int = 1 << 26, **kw):
        super().__init__(params, **kw)
        self.chunk = max(64, int(chunk_elems) // 64 * 64)  # aligned chunks (vector kernel, SR stream)
        self._stage = None
        self._copy_stream = None

    @torch.no_grad()
    def step(self, closure=None, grad_scale: Optional[GradClipState] = None):
        bump_param_generation()
        for gi, group in enumerate(self.param_groups):
            lr = group["lr"]
            b1, b2 = group["betas"]
            eps, wd = group["eps"], group["weight_decay"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not p.is_cuda:
                    raise RuntimeError("OffloadedAdamW streams states to a GPU parameter")
                st = self.state[p]
                n = p.numel()
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros(n, dtype=torch.float32).pin_memory()
                    st["exp_avg_sq"] = torch.zeros(n, dtype=torch.float32).pin_memory()
                st["step"] += 1
                step = float(st["step"])
                hb = self._hyper_buf(p.device, (gi,))
                upload_hyper(hb, [lr, b1, b2, eps, wd, 1.0 - b1 ** step, 1.0 - b2 ** step, 1.0, self._sr(), step])
                self._stream_update(p, st, hb, grad_scale)

    NSLOT = 3

    def _stream_update(self, p, st, hb, grad_scale):
        """H2D on one stream, D2H on another (the host link is full duplex), the update on the
        compute stream; NSLOT device staging slots so chunk i+1 uploads and chunk i-1 downloads
        while chunk i is updated."""
        C = _native.kernels()
        dev = p.device
        if self._copy_stream is None:
            self._copy_stream = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
            self._stage = [(torch.empty(self.chunk, device=dev), torch.empty(self.chunk, device=dev))
                           for _ in range(self.NSLOT)]
        up, down = self._copy_stream
        comp = torch.cuda.current_stream(dev)
        pf, gf = p.data.view(-1), p.grad.view(-1)
        m_h, v_h = st["exp_avg"], st["exp_avg_sq"]
        n = pf.numel()
        chunks = [(s, min(n, s + self.chunk)) for s in range(0, n, self.chunk)]
        up_done = [torch.cuda.Event() for _ in chunks]
        upd_done = [torch.cuda.Event() for _ in chunks]
        down_done = [torch.cuda.Event() for _ in chunks]
        entry = torch.cuda.Event()
        entry.record(comp)  # grads / params of this step are ready

        def upload(i):
            s, e = chunks[i]
            mb, vb = self._stage[i % self.NSLOT]
            with torch.cuda.stream(up):
                up.wait_event(entry)
                if i >= self.NSLOT:
                    up.wait_event(down_done[i - self.NSLOT])  # slot free: its previous chunk is home
                mb[: e - s].copy_(m_h[s:e], non_blocking=True)
                vb[: e - s].copy_(v_h[s:e], non_blocking=True)
                up_done[i].record(up)

        for i in range(min(self.NSLOT - 1, len(chunks))):
            upload(i)
        for i, (s, e) in enumerate(chunks):
            if i + self.NSLOT - 1 < len(chunks):
                upload(i + self.NSLOT - 1)
            comp.wait_event(up_done[i])
            mb, vb = self._stage[i % self.NSLOT]
            C.adamw(pf[s:e], gf[s:e], mb[: e - s], vb[: e - s], None, hb,
                    None if grad_scale is None else grad_scale.buf, 0, s)
            upd_done[i].record(comp)
            with torch.cuda.stream(down):
                down.wait_event(upd_done[i])
                m_h[s:e].copy_(mb[: e - s], non_blocking=True)
                v_h[s:e].copy_(vb[: e - s], non_blocking=True)
                down_done[i].record(down)
        comp.wait_stream(down)  # host states complete before the next step reads them
        comp.wait_stream(up)


_EIGHT_BIT = ("paged_adamw_8bit", "adamw_8bit", "adamw_bnb_8bit", "paged_adamw8bit", "adamw8bit")


def make_optimizer(name: str, params, lr: float, weight_decay: float, betas=(0.9, 0.999), eps=1e-8,
                   master_weights=False, offload: bool = False):
    """Optimizer by HF ``optim`` name. ``offload=True`` keeps AdamW moments in pinned host memory
    (OffloadedAdamW) — only worthwhile when HBM cannot hold them (e.g. 70B on one node)."""
    name = (name or "adamw_torch").lower()
    if name in _EIGHT_BIT:
        # bitsandbytes' 8-bit AdamW keeps block-quantized moments: a different algorithm and memory
        # footprint. Substituting 32-bit states silently would change both, so refuse loudly.
        raise ValueError(f"optimizer {name!r} (8-bit block-quantized AdamW states) is not implemented; use "
                         "'paged_adamw_32bit' / 'adamw_torch' (fp32 states, the reference config's choice)")
    if offload and name.startswith(("adamw", "paged_adamw", "fused_adamw")):
        return OffloadedAdamW(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
    if name in ("adamw", "adamw_torch", "adamw_hf", "adamw_32bit", "paged_adamw_32bit", "adamw_torch_fused",
                "fused_adamw"):
        return FusedAdamW(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                          master_weights=master_weights)
    if name == "sgd":
        return torch.optim.SGD(params, lr=lr, weight_decay=weight_decay)
    raise ValueError(f"unknown optimizer {name!r}")
