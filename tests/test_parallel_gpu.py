"""GPU checks for the data-parallel engines on one MI355X: FSDP (world 1, meta init, HIP kernels,
direct-grad GEMM slots) produces the same update as DDP; OffloadedAdamW (pinned host moments
streamed through the HIP AdamW kernel) matches the resident FusedAdamW bit-for-bit."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(engine, opt, ids):
    loss = engine(ids, labels=ids)["loss"]
    loss.backward()
    engine.finish_gradient_sync()
    st = engine.clip_grad_norm_(1.0) if hasattr(engine, "units") else None
    if st is None:
        from gke_ray_train_amd.ops import clip_grad_norm_
        st = clip_grad_norm_(engine.grad_buffers(), 1.0)
    opt.step(grad_scale=st)
    engine.zero_grad()
    return loss.item(), float(st.buf[0])


def test_offloaded_adamw_matches_fused():
    from gke_ray_train_amd.ops import FusedAdamW
    from gke_ray_train_amd.ops.optim import OffloadedAdamW
    torch.manual_seed(0)
    n = 5_000_003
    p0 = torch.randn(n, device="cuda").bfloat16()
    pa = torch.nn.Parameter(p0.clone())
    pb = torch.nn.Parameter(p0.clone())
    a = FusedAdamW([pa], lr=1e-3, weight_decay=0.1)
    b = OffloadedAdamW([pb], chunk_elems=1 << 20, lr=1e-3, weight_decay=0.1)
    for _ in range(3):
        g = torch.randn(n, device="cuda").bfloat16()
        pa.grad = g.clone()
        pb.grad = g.clone()
        a.step()
        b.step()
    torch.cuda.synchronize()
    assert torch.equal(pa.data, pb.data)
    assert torch.equal(a.state[pa]["exp_avg"].cpu(), b.state[pb]["exp_avg"])
    assert torch.equal(a.state[pa]["exp_avg_sq"].cpu(), b.state[pb]["exp_avg_sq"])
    assert b.state[pb]["exp_avg"].is_pinned()


@pytest.mark.parametrize("offload", [False, True])
def test_fsdp_world1_matches_ddp_on_gpu(offload, monkeypatch):
    # the two engines lay parameters out differently; compare with round-to-nearest updates
    # (stochastic rounding draws its bits by flat-buffer index)
    monkeypatch.setenv("GRT_ADAMW_SR", "0")
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.models.llama import LlamaForCausalLM, RMSNorm, get_config
    from gke_ray_train_amd.ops import FusedAdamW
    from gke_ray_train_amd.parallel import DistributedDataParallel
    from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel
    cfg = get_config("llama-tiny-gqa")
    ref = build_llama(cfg, device="cuda", dtype=torch.bfloat16, seed=11)
    sd = {k: v.clone() for k, v in ref.state_dict().items()}
    ddp = DistributedDataParallel(ref)
    opt_d = FusedAdamW(ddp.optimizer_param_groups(0.0), lr=1e-3)

    m = LlamaForCausalLM(cfg, device="meta", dtype=torch.bfloat16)

    def init(mod):
        with torch.no_grad():
            if isinstance(mod, (torch.nn.Linear, torch.nn.Embedding)):
                mod.weight.normal_(0, 0.02)
            elif isinstance(mod, RMSNorm):
                mod.weight.fill_(1.0)
    f = FullyShardedDataParallel(m, param_init_fn=init, device="cuda", cpu_offload=offload,
                                 offload_chunk_elems=1 << 16)
    f.load_full_state_dict(sd)
    opt_f = f.build_optimizer(lr=1e-3)
    g = torch.Generator(device="cuda").manual_seed(3)
    for _ in range(3):
        ids = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=g)
        ld, nd = _step(ddp, opt_d, ids)
        lf, nf = _step(f, opt_f, ids)
        assert abs(ld - lf) < 2e-2 * max(1.0, abs(ld)), (ld, lf)
        assert abs(nd - nf) < 2e-2 * max(1.0, nd), (nd, nf)
    full = f.full_state_dict()
    for k, v in ref.state_dict().items():
        d = (full[k].float() - v.float()).abs().max().item()
        assert d < 5e-3, (k, d)


@pytest.mark.parametrize("transpose", ["0", "1"])
def test_overlapped_optimizer_matches_serial(transpose, monkeypatch):
    """Chunked AdamW on a side stream, released to each module's forward pre-hook, gives
    bit-identical parameters and losses to the serial end-of-step update. With the transposing
    update (W^T for the next backward's TN dX GEMM) the input gradients round differently, so
    losses / parameters agree to bf16 rounding instead of bit for bit."""
    monkeypatch.setenv("GRT_OPT_TRANSPOSE", transpose)
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.ops import FusedAdamW, clip_grad_norm_
    from gke_ray_train_amd.parallel import DistributedDataParallel
    from gke_ray_train_amd.parallel.overlap import OverlappedOptimizer
    runs = []
    for overlap in (False, True):
        m = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=5)
        ddp = DistributedDataParallel(m)
        opt = FusedAdamW(ddp.optimizer_param_groups(0.01), lr=1e-3)
        if overlap:
            opt = OverlappedOptimizer(ddp, opt)
            # embed, layers (GRT_OVERLAP_FINE=1: per layer its norms + 4 projections), final norm, head
            per = 5 if os.environ.get("GRT_OVERLAP_FINE", "0") == "1" else 1
            assert len(opt.chunks) == per * m.config.num_hidden_layers + 3
            assert bool(opt._wt) == (transpose == "1")
        g = torch.Generator(device="cuda").manual_seed(9)
        losses = []
        for _ in range(4):
            ids = torch.randint(0, m.config.vocab_size, (2, 128), device="cuda", generator=g)
            loss = ddp(ids, labels=ids)["loss"]
            loss.backward()
            ddp.finish_gradient_sync()
            st = clip_grad_norm_(ddp.grad_buffers(), 0.5)
            opt.step(grad_scale=st)
            ddp.zero_grad()
            losses.append(loss.item())
        if overlap:
            opt.synchronize()
        torch.cuda.synchronize()
        runs.append((losses, {k: v.clone() for k, v in m.state_dict().items()}))
    if transpose == "0":
        assert runs[0][0] == runs[1][0]
        for k, v in runs[0][1].items():
            assert torch.equal(v, runs[1][1][k]), k
    else:
        for a, b in zip(runs[0][0], runs[1][0]):
            assert abs(a - b) < 1e-3 * abs(a), (runs[0][0], runs[1][0])
        for k, v in runs[0][1].items():
            d = (v.float() - runs[1][1][k].float()).abs().max().item()
            assert d < 2e-2 * max(1.0, v.float().abs().max().item()), (k, d)


def test_overlapped_optimizer_lr_scheduler_sees_the_step():
    """An LR scheduler bound to the inner optimizer (trainer/sft.py) must not warn
    "lr_scheduler.step() before optimizer.step()": the overlapped step marks the inner optimizer."""
    import warnings
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.ops import FusedAdamW, clip_grad_norm_
    from gke_ray_train_amd.parallel import DistributedDataParallel
    from gke_ray_train_amd.parallel.overlap import OverlappedOptimizer
    m = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=5)
    ddp = DistributedDataParallel(m)
    inner = FusedAdamW(ddp.optimizer_param_groups(0.01), lr=1e-3)
    sched = torch.optim.lr_scheduler.LambdaLR(inner, lambda s: 1.0 / (1 + s))
    opt = OverlappedOptimizer(ddp, inner)
    ids = torch.randint(0, m.config.vocab_size, (2, 64), device="cuda")
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        for _ in range(2):
            ddp(ids, labels=ids)["loss"].backward()
            ddp.finish_gradient_sync()
            opt.step(grad_scale=clip_grad_norm_(ddp.grad_buffers(), 0.5))
            sched.step()
            ddp.zero_grad()
    opt.synchronize()
    assert abs(inner.param_groups[0]["lr"] - 1e-3 / 3) < 1e-9


def test_sequence_parallel_single_rank_matches_plain_on_gpu():
    """Ulysses path on the GPU (RoPE at absolute positions through the HIP kernel's position array,
    all-to-all degenerate at P=1, flash kernel) == the fused rope_attention path."""
    import os
    import torch.distributed as dist
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.parallel.sequence import enable_sequence_parallel, shard_sequence
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29671")
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        ids = torch.randint(0, 512, (2, 256), device="cuda", generator=torch.Generator(device="cuda").manual_seed(2))
        a = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=4)
        b = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=4)
        enable_sequence_parallel(b)
        la = a(ids, labels=ids)["loss"]
        la.backward()
        ids_l, lab_l, w = shard_sequence(ids)
        lb = b(ids_l, shifted_labels=lab_l)["loss"] * w
        lb.backward()
        assert abs(la.item() - lb.item()) < 1e-3 * max(1.0, la.item())
        for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
            rel = (pa.grad.float() - pb.grad.float()).norm() / pa.grad.float().norm().clamp_min(1e-12)
            assert rel < 2e-2, (n, float(rel))
    finally:
        dist.destroy_process_group()


def test_llama3_70b_shapes_fsdp_offload_step():
    """BASELINE config #5 shapes on one GPU: Llama-3-70B layer geometry (d 8192, GQA 64:8,
    FFN 28672, V 128256) with 2 of its 80 layers, FSDP meta init + CPU-offloaded AdamW, two steps
    through every HIP kernel at those shapes; loss finite and decreasing."""
    from gke_ray_train_amd.models.llama import LlamaForCausalLM, RMSNorm, get_config
    from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel
    cfg = get_config("llama3-70b", num_hidden_layers=2)
    m = LlamaForCausalLM(cfg, device="meta", dtype=torch.bfloat16)

    def init(mod):
        with torch.no_grad():
            if isinstance(mod, (torch.nn.Linear, torch.nn.Embedding)):
                mod.weight.normal_(0, 0.02)
            elif isinstance(mod, RMSNorm):
                mod.weight.fill_(1.0)
    f = FullyShardedDataParallel(m, param_init_fn=init, device="cuda", cpu_offload=True)
    opt = f.build_optimizer(lr=1e-4)
    ids = torch.randint(0, cfg.vocab_size, (2, 1024), device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
    losses = []
    for _ in range(3):
        loss, _ = _step(f, opt, ids)
        losses.append(loss)
    assert all(l == l and l < 20 for l in losses), losses
    assert losses[-1] < losses[0], losses


@pytest.mark.parametrize("accum,bucket_mb", [(1, 0.25), (2, 0.25), (1, None)])
def test_ddp_early_grad_norm_matches_full_norm(accum, bucket_mb):
    """One GPU: per-bucket sums of squares launched on a side stream as buckets finish during
    backward (parallel/ddp.py) give the same global norm / clip coefficient as the norm of the
    final gradient buffers computed after backward, over several steps (flags reset per step)."""
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.ops import clip_grad_norm_
    from gke_ray_train_amd.parallel import DistributedDataParallel
    m = build_llama("llama-tiny-gqa", device="cuda", dtype=torch.bfloat16, seed=3)
    ddp = DistributedDataParallel(m, bucket_cap_mb=bucket_mb)
    assert ddp._early_norm
    if bucket_mb:
        assert ddp.num_buckets() > 2
    g = torch.Generator(device="cuda").manual_seed(5)
    for step in range(3):
        for j in range(accum):
            ids = torch.randint(0, 512, (2, 128), device="cuda", generator=g)
            with ddp.no_sync(j < accum - 1):
                (ddp(ids, labels=ids)["loss"] / accum).backward()
        ddp.finish_gradient_sync()
        st = ddp.clip_grad_norm_(0.3)
        ref = clip_grad_norm_(ddp.grad_buffers(), 0.3)
        full = torch.sqrt(sum((b.float() ** 2).sum() for b in ddp.grad_buffers()))
        torch.cuda.synchronize()
        bad = [n for n, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
        assert not bad, (step, "non-finite gradients", bad)
        assert abs(float(st.buf[0]) - float(full)) <= 1e-3 * float(full), (step, float(st.buf[0]), float(full))
        assert abs(float(st.buf[1]) - float(ref.buf[1])) <= 1e-3 * float(ref.buf[1])
        ddp.zero_grad()


@pytest.mark.parametrize("resident,prefetch,proxy", [(0.0, 0, 0), (0.5, 0, 0), (0.0, 5, 0), (0.5, 4096, 0),
                                                   (0.0, 5, 4), (1.0, 0, 4)])
def test_fsdp_overlapped_offload_matches_serial_offload(resident, prefetch, proxy):
    """The per-unit offloaded AdamW issued on side streams at step() and waited for by each unit's
    next forward (parallel/offload.py), with part of the moments HBM-resident and the first
    ``prefetch`` streamed chunks uploaded during the backward (a ring smaller than the chunk count:
    slots reused within a step; larger: every chunk prefetched), gives the parameters, moments and
    losses of the serial after-backward stream (same kernel, same data). ``proxy``: rank 0 of a
    ``proxy``-rank job on one device, whose gathers of an updated unit run on a side stream (a
    missing wait there let the forward read a half-written gather buffer)."""
    from gke_ray_train_amd.models.llama import LlamaForCausalLM, RMSNorm, get_config
    from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel
    from gke_ray_train_amd.parallel.offload import OverlappedOffloadAdamW
    cfg = get_config("llama-tiny-gqa")

    def init(mod):
        with torch.no_grad():
            if isinstance(mod, (torch.nn.Linear, torch.nn.Embedding)):
                mod.weight.normal_(0, 0.02)
            elif isinstance(mod, RMSNorm):
                mod.weight.fill_(1.0)
    runs = []
    for overlap in (False, True):
        torch.manual_seed(0)
        m = LlamaForCausalLM(cfg, device="meta", dtype=torch.bfloat16)
        f = FullyShardedDataParallel(m, param_init_fn=init, device="cuda", cpu_offload=True,
                                     offload_chunk_elems=1 << 14, proxy_world=proxy)
        opt = f.build_optimizer(lr=1e-3, overlap=overlap, resident_fraction=resident,
                                prefetch_slots=prefetch if overlap else 0)
        assert isinstance(opt, OverlappedOffloadAdamW) == overlap
        if overlap:
            assert (opt.resident_units > 0) == (resident > 0)
            assert opt.resident_units < len(opt.segments) or resident == 1.0
            assert opt.prefetch_slots == min(prefetch, len(opt.chunks))
            assert prefetch == 0 or prefetch >= len(opt.chunks) or len(opt.chunks) > opt.nslot
        g = torch.Generator(device="cuda").manual_seed(4)
        losses = []
        for _ in range(4):
            ids = torch.randint(0, cfg.vocab_size, (2, 128), device="cuda", generator=g)
            loss, _ = _step(f, opt, ids)
            losses.append(loss)
        sd = opt.state_dict()
        torch.cuda.synchronize()
        st = [v for s in sd["state"].values() for k, v in s.items() if k in ("exp_avg", "exp_avg_sq")]
        runs.append((losses, f.shard_store.clone(), f.rep_flat.clone(), [t.clone() for t in st]))
    # same kernel on the same data: identical in every run so far (tools/offload_debug.py); compared
    # to bf16 rounding so that a reduction-order difference elsewhere in the step cannot flake it,
    # while a stale-parameter race (a unit running before its update) still fails by far
    for a, b in zip(runs[0][0], runs[1][0]):
        assert abs(a - b) <= 1e-3 * abs(a), (runs[0][0], runs[1][0])
    for a, b in ((runs[0][1], runs[1][1]), (runs[0][2], runs[1][2])):
        d = (a.float() - b.float()).abs().max().item()
        assert d <= 2e-2 * max(1.0, a.float().abs().max().item()), d
    for a, b in zip(runs[0][3], runs[1][3]):
        d = (a.cpu() - b.cpu()).abs().max().item()
        assert d <= 1e-2 * max(1e-6, a.abs().max().item()), d


@pytest.mark.parametrize("resident,prefetch", [(0.0, 3), (0.5, 0)])
def test_overlapped_offload_optimizer_resume_continues_identically(resident, prefetch):
    """Checkpoint / resume of the overlapped offloaded AdamW: after load_state_dict the
    moments are fp32 pinned host tensors again (resident units re-uploaded on first use), and two
    more steps give the parameters of the uninterrupted run."""
    from gke_ray_train_amd.models.llama import LlamaForCausalLM, RMSNorm, get_config
    from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel
    cfg = get_config("llama-tiny-gqa")

    def init(mod):
        with torch.no_grad():
            if isinstance(mod, (torch.nn.Linear, torch.nn.Embedding)):
                mod.weight.normal_(0, 0.02)
            elif isinstance(mod, RMSNorm):
                mod.weight.fill_(1.0)

    def build():
        torch.manual_seed(0)
        m = LlamaForCausalLM(cfg, device="meta", dtype=torch.bfloat16)
        f = FullyShardedDataParallel(m, param_init_fn=init, device="cuda", cpu_offload=True,
                                     offload_chunk_elems=1 << 14)
        return f, f.build_optimizer(lr=1e-3, overlap=True, resident_fraction=resident, prefetch_slots=prefetch)

    g = torch.Generator(device="cuda").manual_seed(11)
    batches = [torch.randint(0, cfg.vocab_size, (2, 64), device="cuda", generator=g) for _ in range(4)]
    f1, o1 = build()
    for ids in batches[:2]:
        _step(f1, o1, ids)
    import copy
    sd_opt = copy.deepcopy(o1.state_dict())  # as if saved: torch's state_dict aliases the live moments
    sd_par = {k: v.clone() for k, v in f1.sharded_state_dict().items()}
    for ids in batches[2:]:
        _step(f1, o1, ids)
    o1.synchronize()
    f2, o2 = build()
    f2.load_sharded_state_dict(sd_par)
    o2.load_state_dict(sd_opt)
    for st in o2.state.values():
        for k in ("exp_avg", "exp_avg_sq"):
            if k in st:
                assert st[k].dtype == torch.float32 and st[k].device.type == "cpu" and st[k].is_pinned(), k
    for ids in batches[2:]:
        _step(f2, o2, ids)
    o2.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(f1.shard_store, f2.shard_store)
    assert torch.equal(f1.rep_flat, f2.rep_flat)


def test_fsdp_forward_transpose_budget_uses_full_weight_sizes(monkeypatch):
    """FSDP's forward-time W^T copies persist (one full bf16 copy of the projection weights), so they
    are enabled only under GRT_FSDP_FWD_TRANSPOSE_MAX_GIB measured on the FULL weight sizes: the
    sharded module tensors no longer carry them (a 70B run once kept 130 GiB of copies)."""
    from gke_ray_train_amd.models.llama import LlamaForCausalLM, get_config
    from gke_ray_train_amd.ops.linear import Linear
    from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel
    cfg = get_config("llama-tiny-gqa")
    expect = None
    for limit, on in (("24", True), ("0.0001", False)):
        monkeypatch.setenv("GRT_FSDP_FWD_TRANSPOSE_MAX_GIB", limit)
        torch.manual_seed(0)
        m = LlamaForCausalLM(cfg, device="meta", dtype=torch.bfloat16)
        full = sum(mod.weight.numel() * 2 for blk in m.model.layers for mod in blk.modules() if isinstance(mod, Linear))
        f = FullyShardedDataParallel(m, param_init_fn=lambda mod: None, device="cuda", proxy_world=4)
        assert f.fwd_transpose_bytes == full, (f.fwd_transpose_bytes, full)
        flags = [getattr(mod.weight, "_grt_fsdp_fwd_transpose", False) for blk in m.model.layers
                 for mod in blk.modules() if isinstance(mod, Linear)]
        assert flags and all(x == on for x in flags), (limit, flags)
