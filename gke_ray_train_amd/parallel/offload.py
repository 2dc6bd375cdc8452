"""Offloaded AdamW for FSDP, overlapped with the next forward (BASELINE config #5).

Not in the reference (SURVEY §2.4 CPU offload, §7.4 item 5). ``ops.optim.OffloadedAdamW`` streams
every chunk of the fp32 moments host -> HBM -> host AFTER backward, serially with compute; at 8 B of
moments per parameter each way that exposes the whole host-link transfer every step.

MI355X design:
* the update is split by FSDP unit and issued at ``step()`` time on side streams in FORWARD order
  (root unit — embeddings / LM head — first, then the decoder blocks): uploads on one stream,
  the fused AdamW kernel on another, downloads on a third, so chunk i+1's H2D and chunk i-1's D2H
  overlap chunk i's update (the host link is full duplex) and the whole pipeline runs under the
  next forward. Each unit records an event; FSDP waits for it right before the unit's next
  all-gather (issued from a gather stream, so the compute stream never blocks on a later unit's
  update) or, at world 1, before the unit's forward;
* the global clip stays exact: the coefficient computed at the end of backward is on the compute
  stream before the entry event every update stream waits for;
* RESIDENCY: the offload is a capacity valve, not an end in itself. 288 GB of HBM holds the moments
  of most units even at 70B / 8 ranks, so the first ``resident_units`` units in forward order keep
  their moments in HBM (updated with no host traffic; they are the units needed soonest) and only
  the rest stream. ``resident_fraction`` (bench.py ``--offload-resident auto``) is derived from the
  memory planner: the share of the moments that fits beside everything else;
* gradient shards of a unit are zeroed on the update stream right after its update (FSDP's
  ``zero_grad`` would otherwise memset them on the compute stream while updates still read them);
* PREFETCH into the backward window: the first ``prefetch_slots`` streamed chunks (forward order:
  the units the next forward needs first) own one device slot each; the remaining chunks share a
  ring of NSLOT slots. When the last decoder unit's forward starts, the uploads of the owned slots
  are issued, so they cross the host link during the backward, when it is otherwise idle;
  ``step()`` then updates those chunks at once and only the remaining chunks upload under the next
  forward. The owned slots' write-backs are deferred to the next forward tail, just before their
  next uploads, so both directions of the owned chunks use the backward window and the forward
  window carries only the ring chunks' traffic.
  A slot is reused only after the download of its previous chunk (event per slot), which also
  orders every upload after the previous step's download of the same host range;
* WRITE-BACK ENGINE (``GRT_OFFLOAD_D2H``): ``blit`` (default) copies with ``Tensor.copy_``, which
  ROCclr runs as blit kernels on the CUs; ``sdma`` hands each write-back to an SDMA engine of its own
  through the HSA runtime (``sdma_d2h``, csrc/bindings/sdma_copy.cpp), ordered on the download
  stream like a stream copy, so no write-back occupies the CUs; a failed SDMA copy raises at the next
  ``step()`` / ``synchronize()`` (profiles/r6_offload_link.md).
"""
from __future__ import annotations

import os

from typing import Dict, List, Optional

import torch

from .. import _native
from ..ops.optim import GradClipState, OffloadedAdamW, bump_param_generation, upload_hyper


class OverlappedOffloadAdamW(OffloadedAdamW):
    NSLOT = 3

    def __init__(self, fsdp, chunk_elems: int = 1 << 26, resident_fraction: float = 0.0, prefetch_slots: int = 0,
                 **kw):
        groups = fsdp.optimizer_param_groups(kw.pop("weight_decay", 0.0))
        super().__init__(groups, chunk_elems=chunk_elems, **kw)
        self.fsdp = fsdp
        root = [u for u in fsdp.units if u.module is fsdp.module]
        blocks = [u for u in fsdp.units if u.module is not fsdp.module]
        off, ranges = 0, {}
        for u in fsdp.units:  # shard store layout order
            ranges[id(u)] = (off, off + u.shard_numel)
            off += u.shard_numel
        self.segments = [(u,) + ranges[id(u)] for u in root + blocks]  # forward order
        total = sum(hi - lo for _, lo, hi in self.segments)
        budget = float(resident_fraction) * total
        self.resident = set()
        acc = 0
        for u, lo, hi in self.segments:
            if acc + (hi - lo) > budget:
                break
            self.resident.add(id(u))
            acc += hi - lo
        self._dev_m: Dict[int, torch.Tensor] = {}
        self._dev_v: Dict[int, torch.Tensor] = {}
        self._streams = None
        # streamed chunks in forward order: (unit, start, end) of the flat shard
        self.chunks = [(u, s, min(hi, s + self.chunk)) for u, lo, hi in self.segments if id(u) not in self.resident
                       for s in range(lo, hi, self.chunk)]
        # slots 0 .. P-1 belong to the prefetched chunks 0 .. P-1 (one each: the next step's upload of
        # chunk i waits only for this step's download of chunk i, among the first to finish); the
        # remaining chunks share a ring of NSLOT slots behind them
        self.prefetch_slots = min(int(prefetch_slots), len(self.chunks))
        self.nslot = self.prefetch_slots + self.NSLOT
        self._slot_free: List[Optional[torch.cuda.Event]] = [None] * self.nslot
        self._landed: Dict[int, torch.cuda.Event] = {}  # chunk index -> upload done (prefetched)
        self._pending_down: List[tuple] = []  # (chunk index, update done) of deferred write-backs
        self.defer_writeback = os.environ.get("GRT_OFFLOAD_DEFER_WRITEBACK", "1") != "0"
        mode = os.environ.get("GRT_OFFLOAD_D2H", "blit")
        if mode not in ("blit", "sdma"):
            raise ValueError(f"GRT_OFFLOAD_D2H={mode!r}: expected 'blit' or 'sdma'")
        self.d2h_engine = mode if fsdp.device.type == "cuda" else "blit"
        fsdp._grad_zero_by_optimizer = True
        if self.prefetch_slots > 0:
            fsdp.add_forward_tail_hook(self.prefetch)

    @property
    def resident_units(self) -> int:
        return len(self.resident)

    def _state(self, p):
        st = self.state[p]
        if len(st) == 0:
            n = p.numel()
            st["step"] = torch.tensor(0.0)
            st["exp_avg"] = torch.zeros(n, dtype=torch.float32).pin_memory()
            st["exp_avg_sq"] = torch.zeros(n, dtype=torch.float32).pin_memory()
        return st

    @torch.no_grad()
    def step(self, closure=None, grad_scale: Optional[GradClipState] = None):
        fs = self.fsdp
        dev = fs.device
        if dev.type != "cuda":
            return super().step(closure, grad_scale)
        bump_param_generation()
        fs._grads_consumed = True  # every unit's gradients are zeroed on the update stream below
        C = _native.kernels()
        self._ensure_streams(dev)
        up, upd, down = self._streams
        comp = torch.cuda.current_stream(dev)
        fs.wait_updates()  # the previous step's updates all landed (normally long done)
        self._check_d2h()
        self._flush_downloads()  # no forward tail since the last step (prefetch() did not run)
        hbs, work = [], []
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            for p in group["params"]:
                st = self._state(p)
                st["step"] += 1
                step = float(st["step"])
                hb = self._hyper_buf(p.device, (gi,))
                upload_hyper(hb, [group["lr"], b1, b2, group["eps"], group["weight_decay"], 1.0 - b1 ** step,
                                  1.0 - b2 ** step, 1.0, self._sr(), step])
                work.append((p, st, hb))
        entry = torch.cuda.Event()
        entry.record(comp)  # gradients, clip coefficient and hyper-parameters of this step
        gs = None if grad_scale is None else grad_scale.buf
        if gs is not None:
            # the clip state is read by every unit's update on the update stream, which runs under
            # the next forward: a caller that drops it right after step() (a fresh GradClipState per
            # step) must not let the allocator hand its memory to that forward before the updates ran
            # (the flaky loss mismatch of tests/test_parallel_gpu.py's overlapped-offload test)
            gs.record_stream(upd)
        (sp, sst, shb), (rp, rst, rhb) = work[0], work[1]
        for s in (upd, down):
            s.wait_event(entry)
        # uploads need no gradient: they only wait for their slot (and so for the previous step's
        # download of the same host range, issued earlier on the in-order download stream)
        # replicated 1-D parameters (norm weights): tiny, device moments, first on the update stream
        with torch.cuda.stream(upd):
            if "dev_m" not in rst:
                rst["dev_m"] = rst["exp_avg"].to(dev)
                rst["dev_v"] = rst["exp_avg_sq"].to(dev)
            C.adamw(rp.data, rp.grad, rst["dev_m"], rst["dev_v"], None, rhb, gs, 0, 0)
            rp.grad.zero_()
        pf, gf = sp.data.view(-1), sp.grad.view(-1)
        m_h, v_h = sst["exp_avg"], sst["exp_avg_sq"]
        events = {}
        ci = 0
        for u, lo, hi in self.segments:
            if id(u) in self.resident:
                with torch.cuda.stream(upd):
                    if id(u) not in self._dev_m:
                        self._dev_m[id(u)] = m_h[lo:hi].to(dev)
                        self._dev_v[id(u)] = v_h[lo:hi].to(dev)
                    C.adamw(pf[lo:hi], gf[lo:hi], self._dev_m[id(u)], self._dev_v[id(u)], None, shb, gs, 0, lo)
                    gf[lo:hi].zero_()
            else:
                while ci < len(self.chunks) and self.chunks[ci][0] is u:
                    _, s, e = self.chunks[ci]
                    slot = self._slot(ci)
                    mb, vb = self._stage[slot]
                    landed = self._landed.pop(ci, None) or self._upload(ci)
                    with torch.cuda.stream(upd):
                        upd.wait_event(landed)
                        C.adamw(pf[s:e], gf[s:e], mb[:e - s], vb[:e - s], None, shb, gs, 0, s)
                        gf[s:e].zero_()
                        done = torch.cuda.Event()
                        done.record(upd)
                    if ci < self.prefetch_slots and self.defer_writeback:
                        # an owned slot: its write-back is deferred to the backward window (the slot
                        # holds the only current copy until then; see _flush_downloads)
                        self._pending_down.append((ci, done))
                    else:
                        self._download(ci, done)
                    ci += 1
            ev = torch.cuda.Event()
            ev.record(upd)
            events[u] = ev
        self._landed.clear()
        fs.set_update_events(events)

    def _download(self, ci: int, done: torch.cuda.Event):
        """Device -> pinned host write-back of chunk ``ci`` after its update (``done``), on the
        in-order download stream; the event it records frees the chunk's slot."""
        down = self._streams[2]
        _, s, e = self.chunks[ci]
        slot = self._slot(ci)
        mb, vb = self._stage[slot]
        sst = self.state[self.param_groups[0]["params"][0]]
        with torch.cuda.stream(down):
            down.wait_event(done)
            if self.d2h_engine == "sdma":
                # the copy waits for the update stream itself (the producer of mb / vb)
                C = _native.kernels()
                upd = self._streams[1].cuda_stream
                C.sdma_d2h(sst["exp_avg"][s:e], mb[:e - s], upd)
                C.sdma_d2h(sst["exp_avg_sq"][s:e], vb[:e - s], upd)
            else:
                sst["exp_avg"][s:e].copy_(mb[:e - s], non_blocking=True)
                sst["exp_avg_sq"][s:e].copy_(vb[:e - s], non_blocking=True)
            free = torch.cuda.Event()
            free.record(down)
        self._slot_free[slot] = free

    def _flush_downloads(self):
        """Issue the deferred write-backs of the owned (prefetch) slots."""
        pend, self._pending_down = self._pending_down, []
        for ci, done in pend:
            self._download(ci, done)

    def _ensure_streams(self, dev):
        if self._streams is None:
            self._streams = tuple(torch.cuda.Stream(dev) for _ in range(3))  # up, update, down
            self._stage = [(torch.empty(self.chunk, device=dev), torch.empty(self.chunk, device=dev))
                           for _ in range(self.nslot)]

    def _slot(self, ci: int) -> int:
        P = self.prefetch_slots
        return ci if ci < P else P + (ci - P) % self.NSLOT

    def _upload(self, ci: int) -> torch.cuda.Event:
        """Host -> device copy of streamed chunk ``ci`` into its slot on the upload stream, after the
        slot's previous download."""
        up = self._streams[0]
        _, s, e = self.chunks[ci]
        slot = self._slot(ci)
        mb, vb = self._stage[slot]
        sst = self.state[self.param_groups[0]["params"][0]]
        with torch.cuda.stream(up):
            if self._slot_free[slot] is not None:
                up.wait_event(self._slot_free[slot])
            mb[:e - s].copy_(sst["exp_avg"][s:e], non_blocking=True)
            vb[:e - s].copy_(sst["exp_avg_sq"][s:e], non_blocking=True)
            landed = torch.cuda.Event()
            landed.record(up)
        return landed

    @torch.no_grad()
    def prefetch(self):
        """Upload the first ``prefetch_slots`` streamed chunks for the coming ``step()`` (called by
        FSDP when the last decoder unit's training forward starts: the uploads cross the host link
        during the backward)."""
        fs = self.fsdp
        if fs.device.type != "cuda" or self._landed or not self.chunks:
            return
        self._state(self.param_groups[0]["params"][0])
        self._ensure_streams(fs.device)
        # the owned slots' write-backs of the last step go first (their uploads wait for them): both
        # directions of the owned slots cross the link in the backward window, leaving the forward
        # window to the ring chunks
        self._flush_downloads()
        for ci in range(self.prefetch_slots):
            self._landed[ci] = self._upload(ci)

    def synchronize(self):
        """Current stream waits for every pending unit update and the moment downloads."""
        self.fsdp.wait_updates()
        if self._streams is not None:
            self._flush_downloads()
            torch.cuda.current_stream(self.fsdp.device).wait_stream(self._streams[2])
            self._check_d2h()

    def _check_d2h(self):
        """Raise if an SDMA write-back failed or timed out since the last check (its host range
        then holds stale moments; the copy released the stream instead of hanging it)."""
        if self.d2h_engine != "sdma" or self._streams is None:
            return
        C = _native.kernels()
        dev = self.fsdp.device.index if self.fsdp.device.index is not None else torch.cuda.current_device()
        err = C.sdma_stats(dev)["error"]
        if err:
            C.sdma_clear_error(dev)
            raise RuntimeError(f"offloaded AdamW: SDMA moment write-back failed: {err}")

    def state_dict(self):
        """Moments of resident units are copied into the host tensors, so the layout is the plain
        OffloadedAdamW one (full-size host exp_avg / exp_avg_sq)."""
        self.synchronize()
        torch.cuda.synchronize(self.fsdp.device)
        if self._dev_m:
            sp = self.param_groups[0]["params"][0]
            st = self.state[sp]
            for u, lo, hi in self.segments:
                if id(u) in self._dev_m:
                    st["exp_avg"][lo:hi].copy_(self._dev_m[id(u)])
                    st["exp_avg_sq"][lo:hi].copy_(self._dev_v[id(u)])
        rp = self.param_groups[1]["params"][0]
        rst = self.state.get(rp, {})
        if "dev_m" in rst:
            rst["exp_avg"].copy_(rst["dev_m"])
            rst["exp_avg_sq"].copy_(rst["dev_v"])
        sd = super().state_dict()
        for s in sd["state"].values():  # device mirrors are not part of the checkpoint
            s.pop("dev_m", None)
            s.pop("dev_v", None)
        return sd

    def load_state_dict(self, sd):
        self.synchronize()
        # the host waits for every in-flight write-back: the load replaces the host moment tensors,
        # and a device -> host copy landing after that (into memory the host allocator may already
        # have handed out again: SDMA copies are not tracked by it) would corrupt it
        torch.cuda.synchronize(self.fsdp.device)
        super().load_state_dict(sd)
        # slots uploaded ahead (prefetch()) hold the moments from before the load: drop them so the
        # next step uploads the loaded ones (and nothing stale is written back over them)
        self._landed.clear()
        self._pending_down = []
        self._dev_m.clear()
        self._dev_v.clear()
        for st in self.state.values():
            st.pop("dev_m", None)
            st.pop("dev_v", None)


# largest automatic prefetch ring (bench --offload-prefetch-gib auto; the HBM room beside the plan
# and the reserve bounds it further). Full-depth 70B, proxy rank 0 of 8, moments streamed: 32 / 48 /
# 64 GiB ring = 0.80 / 0.82 / 0.91 x of the resident step (profiles/r6_offload_link.md)
PREFETCH_CAP_BYTES = 64 * (1 << 30)


def prefetch_slots_for(budget_bytes: float, chunk_elems: int) -> int:
    """Device chunk slots (m + v fp32, 8 B per element) that fit in ``budget_bytes``."""
    return max(0, int(budget_bytes // (8.0 * chunk_elems)))


def hbm_reserve_bytes() -> float:
    """HBM kept free by the automatic offload plan (``GRT_OFFLOAD_HBM_RESERVE_GIB``, default 8):
    raise it to make ``auto`` stream moments and leave the room to activations / a bigger batch."""
    return float(os.environ.get("GRT_OFFLOAD_HBM_RESERVE_GIB", "8")) * (1 << 30)


def resident_fraction_from_plan(plan_offload, plan_resident=None, margin_bytes: Optional[float] = None) -> float:
    """Share of the offloaded moments that fits in HBM: capacity minus the offload plan's total
    (which already holds the staging chunks) minus the reserve, over the moments the offload moved.
    Every moment byte kept in HBM is one the host link does not carry twice per step, so the plan
    keeps as many resident as the reserve allows; :func:`host_link_plan` says whether what is left
    to stream fits under the step."""
    moved = plan_offload.host_per_rank.get("adam_moments_fp32", 0.0)
    if moved <= 0:
        return 1.0
    margin = hbm_reserve_bytes() if margin_bytes is None else float(margin_bytes)
    room = plan_offload.hbm_capacity - plan_offload.hbm_total - margin
    return max(0.0, min(1.0, room / moved))


# Host link of one MI355X (PCIe Gen5 x16), per direction, measured by tools/hostlink_bench.py:
# SDMA uploads 57 GB/s; the device -> host write-backs run as ROCclr blit kernels at 30-57 GB/s
# depending on the box (profiles/r5_offload70.md, profiles/r6_offload_link.md).
HOST_LINK_GBPS = 57.0


def host_link_plan(plan_offload, resident_fraction: float, step_s: float, link_GBps: Optional[float] = None) -> dict:
    """Bytes the streamed share moves per step (each direction) against what the link carries in
    ``step_s``: ``bound`` means the step will run at the link's pace, not the compute's."""
    link = float(os.environ.get("GRT_HOST_LINK_GBPS", HOST_LINK_GBPS) if link_GBps is None else link_GBps)
    moved = plan_offload.host_per_rank.get("adam_moments_fp32", 0.0)
    streamed = max(0.0, 1.0 - float(resident_fraction)) * moved
    link_s = streamed / (link * 1e9) if link > 0 else float("inf")
    return {"streamed_gib_per_direction": round(streamed / (1 << 30), 2), "link_s": round(link_s, 3),
            "step_s": round(step_s, 3), "link_bound": link_s > step_s,
            # the resident share at which the streamed bytes just fit under the step
            "resident_fraction_for_link": round(max(0.0, min(1.0, 1.0 - link * 1e9 * step_s / moved)), 3)
            if moved > 0 else 1.0}
