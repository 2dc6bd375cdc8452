#!/usr/bin/env python3
"""Headline benchmark: Llama-2-7B bf16 fine-tune, tokens/s for the whole node.

BASELINE.json metric: "tokens/sec (whole node) Llama-2-7B fine-tune at 1/2/4/8 MI355X".
Default = config #2 "Llama-2 7B DDP bf16, 8 Ray workers on 8xMI355X (fine_tune_llama_ray.py path)":
* model: Llama-2-7B architecture (6.74 B params), random init, bf16 params + bf16 grads, fp32
  AdamW moments (the reference full-FT path: torch_dtype=bfloat16 + paged_adamw_32bit,
  reference ray-jobs/fine_tune_llama_ray.py:235-241, fine_tune_config.json:17);
* data: synthetic Wikitext-2-shaped token stream (Zipf ids) streamed by the framework's loader
  (native window gather -> pinned host ring -> async H2D), seq 1024 (MAX_SEQ_LENGTH), 8 sequences
  per GPU per optimizer step (= PER_DEVICE_TRAIN_BATCH_SIZE 2 x GRADIENT_ACCUMULATION_STEPS 4,
  fine_tune_config.json:13-14) — weak scaling;
* step: forward + backward + gradient sync (RCCL, bucketed, overlapped) + global grad-norm clip
  (MAX_GRAD_NORM 0.3) + fused AdamW. Nothing is skipped inside the timed region.
Other BASELINE configs: ``--parallel fsdp`` (#3), ``--peft lora|qlora`` (#4),
``--model llama3-70b --parallel fsdp --offload`` (#5).

Launch: ``python bench.py --gpus N``: for N > 1 (and no ``WORLD_SIZE`` in the environment) the
parent starts N rank processes through the framework's own ``TorchTrainer(num_workers=N,
use_gpu=True)`` — one worker actor per GPU, RCCL rendezvous, exactly the "8 Ray workers" of
BASELINE config #2 (reference ray-jobs/pytorch_llm_ray.py:346-350,368-376) — and never touches the
GPU itself. ``python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`` also works;
a ``WORLD_SIZE`` that disagrees with ``--gpus`` is an error. Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os

# kernel arguments in device memory (read by the HIP runtime at its first call; launch-time setting)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--batch", type=int, default=8, help="sequences per GPU per optimizer step")
    ap.add_argument("--micro-batch", type=int, default=0, help="micro-batch (grad accumulation); 0 = batch")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--parallel", default="ddp", choices=["ddp", "fsdp"])
    ap.add_argument("--sp", type=int, default=1, help="sequence-parallel degree (Ulysses all-to-all, "
                    "parallel/sequence.py): groups of --sp consecutive ranks share each sequence")
    ap.add_argument("--offload", action="store_true", help="FSDP: optimizer states in pinned host memory")
    ap.add_argument("--peft", default="none", choices=["none", "lora", "qlora"])
    ap.add_argument("--lora-r", type=int, default=64)
    ap.add_argument("--bucket-mb", type=float, default=0.0, help="DDP bucket size (0 = planner)")
    ap.add_argument("--zero", default="auto", choices=["auto", "on", "off"],
                    help="DDP sharded optimizer (reduce-scatter + 1/N AdamW + overlapped all-gather); "
                         "auto = on when world > 1")
    ap.add_argument("--max-grad-norm", type=float, default=0.3)
    ap.add_argument("--lr", type=float, default=2e-5)
    ap.add_argument("--checkpointing", action="store_true", help="activation checkpointing")
    ap.add_argument("--data", default="loader", choices=["loader", "pipeline", "static"],
                    help="loader: native window gather + pinned H2D; pipeline: the Ray-Data-like Dataset "
                         "(shuffle -> map_batches -> per-rank streaming shard -> iter_torch_batches, produced "
                         "in a separate process through the shared-memory ring); static: on-device batches")
    ap.add_argument("--profile-dir", default="", help="write a torch.profiler trace here")
    ap.add_argument("--heartbeat", type=float, default=0.0,
                    help="rank 0 prints its current phase to stderr every N seconds outside the timed region (long builds)")
    ap.add_argument("--metrics-jsonl", default="", help="per-step metrics (phase breakdown, MFU, HBM) -> JSONL; "
                    "adds one host sync per step, so it is off for the headline number")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--no-tuned-gemm", action="store_true", help="library-default GEMM solutions (A/B)")
    ap.add_argument("--overlap-opt", default="auto", choices=["auto", "on", "off"],
                    help="replicated DDP: run the AdamW update per module on a side stream, overlapped with the "
                         "next forward (parallel/overlap.py); auto = on unless ZeRO / FSDP")
    ap.add_argument("--ipc", action="store_true", help="latency-bound collectives (grad-norm all-reduce) over the "
                    "xGMI IPC one-shot kernel instead of RCCL (GRT_IPC_COLLECTIVES=1)")
    ap.add_argument("--backend", default="", help="process-group backend (default: nccl = RCCL on GPU, gloo on CPU)")
    ap.add_argument("--force-collectives", action="store_true",
                    help="run the multi-rank collective path even at world 1 (one-rank RCCL process group: "
                         "ZeRO reduce-scatter / all-gather, FSDP gathers) — one-GPU rehearsal of the 8-GPU data plane")
    ap.add_argument("--offload-resident", default="auto",
                    help="--offload: share of the AdamW moments kept in HBM (0..1), 'auto' = what the memory "
                         "planner says fits beside everything else (the rest streams over the host link, "
                         "overlapped with the next forward, parallel/offload.py)")
    ap.add_argument("--offload-prefetch-gib", default="auto",
                    help="--offload: device ring for the streamed moments, filled during the backward (GiB); "
                         "'auto' = min(streamed moments, 32 GiB, planner headroom)")
    ap.add_argument("--offload-overlap", default="on", choices=["on", "off"],
                    help="--offload: per-unit update overlapped with the next forward (on) or the serial "
                         "after-backward stream (off)")
    ap.add_argument("--proxy-world", type=int, default=0,
                    help="one-GPU rehearsal of rank 0 of an N-rank job: DDP/ZeRO buckets and the 1/N optimizer "
                         "shard, or (--parallel fsdp) 1/N parameter / gradient / optimizer shards with the full-unit "
                         "gather buffers of world N; collectives replaced by local copies of this rank's chunk "
                         "(xGMI time excluded; loss not meaningful). Reports the per-rank step with n_gpus 1 and "
                         "proxy_world N")
    ap.add_argument("--layers", type=int, default=0,
                    help="rehearsal only: keep the first N decoder layers of --model (the JSON names the model "
                         "'<model>[N/L layers]', so it is never mistaken for the full model's number)")
    ap.add_argument("--plan-only", action="store_true",
                    help="print the per-rank HBM / host memory plan (parallel/planner.py) for this config and exit")
    ap.add_argument("--launcher", default="", help=argparse.SUPPRESS)  # set by launch_workers
    return ap.parse_args()


def build(a, cfg, dev, dtype, world):
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.models.llama import LlamaForCausalLM, RMSNorm
    from gke_ray_train_amd.ops import FusedAdamW
    if a.parallel == "fsdp":
        from gke_ray_train_amd.parallel.fsdp import FullyShardedDataParallel
        std = cfg.initializer_range
        model = LlamaForCausalLM(cfg, device="meta", dtype=dtype)

        def init(m):
            with torch.no_grad():
                if isinstance(m, (torch.nn.Linear, torch.nn.Embedding)):
                    m.weight.normal_(0.0, std)
                elif isinstance(m, RMSNorm):
                    m.weight.fill_(1.0)
        if a.checkpointing:
            model.gradient_checkpointing_enable()
        proxy = a.proxy_world > 1 and world == 1  # rank 0 of an N-rank full-shard job on one device
        eng = FullyShardedDataParallel(model, param_init_fn=init, device=dev, cpu_offload=a.offload,
                                       proxy_world=a.proxy_world if proxy else 0)
        opt = eng.build_optimizer(lr=a.lr, overlap=a.offload_overlap == "on",
                                  resident_fraction=getattr(a, "resident_fraction", 0.0),
                                  prefetch_slots=getattr(a, "prefetch_slots", 0))
        return model, eng, eng, opt
    from gke_ray_train_amd.parallel import DistributedDataParallel
    model = build_llama(cfg, device=dev, dtype=dtype, seed=1234)
    if a.checkpointing:
        model.gradient_checkpointing_enable()
    if a.sp > 1:
        from gke_ray_train_amd.parallel.sequence import enable_sequence_parallel
        enable_sequence_parallel(model, a.sp_group)
    fwd = model
    if a.peft != "none":
        from gke_ray_train_amd.peft import BitsAndBytesConfig, LoraConfig, get_peft_model, quantize_model_
        if a.peft == "qlora":
            quantize_model_(model, BitsAndBytesConfig(bnb_4bit_compute_dtype=dtype))
        fwd = get_peft_model(model, LoraConfig(r=a.lora_r, lora_alpha=16, lora_dropout=0.1))
    proxy = a.proxy_world > 1 and world == 1
    zero = a.zero == "on" or (a.zero == "auto" and (world > 1 or a.force_collectives or proxy))
    eng = DistributedDataParallel(fwd, bucket_cap_mb=a.bucket_mb or None, shard_optimizer=zero,
                                  proxy_world=a.proxy_world if proxy else 0)
    opt = FusedAdamW(eng.optimizer_param_groups(weight_decay=0.0), lr=a.lr)
    if a.overlap_opt == "on" or (a.overlap_opt == "auto" and not zero and dev.type == "cuda"):
        from gke_ray_train_amd.parallel.overlap import OverlappedOptimizer
        opt = OverlappedOptimizer(eng, opt)
    return fwd, eng, fwd, opt


def _baseline_metric() -> str:
    """The headline metric exactly as BASELINE.json names it."""
    try:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "BASELINE.json")) as f:
            return json.load(f)["metric"]
    except (OSError, ValueError, KeyError):
        return "tokens/sec (whole node) Llama-2-7B fine-tune at 1/2/4/8 MI355X; samples/sec on Wikitext-2"


def _link_plan(plan, a, step_s):
    if a.parallel != "fsdp":
        return None
    from gke_ray_train_amd.parallel.offload import host_link_plan
    return host_link_plan(plan, a.resident_fraction, step_s)


def _bench_worker(cfg: dict):
    """TorchTrainer ``train_loop_per_worker``: the process group is already up (TrainWorker)."""
    run(argparse.Namespace(**cfg))


def launch_workers(a) -> int:
    """``--gpus N`` with no launcher: N TorchTrainer worker actors run :func:`run`; rank 0's JSON
    line reaches this process's stdout through the inherited descriptor. This process only counts
    devices (no HIP context), so the workers own the GPUs."""
    import shutil
    import tempfile
    from gke_ray_train_amd.runtime.errors import TrainingFailedError
    from gke_ray_train_amd.train import RunConfig, ScalingConfig, TorchTrainer
    from gke_ray_train_amd.train.torch import TorchConfig
    use_gpu = a.device != "cpu"
    if use_gpu and torch.cuda.device_count() < a.gpus:
        print(f"bench.py: --gpus {a.gpus} but only {torch.cuda.device_count()} GPU(s) visible", file=sys.stderr)
        return 2
    backend = a.backend or ("nccl" if use_gpu else "gloo")
    store = tempfile.mkdtemp(prefix="grt_bench_")
    os.environ.setdefault("GRT_NUM_GPUS", str(a.gpus if use_gpu else 0))
    try:
        cfg = dict(vars(a), launcher=f"TorchTrainer(num_workers={a.gpus})")
        TorchTrainer(_bench_worker, train_loop_config=cfg,
                     scaling_config=ScalingConfig(num_workers=a.gpus, use_gpu=use_gpu),
                     run_config=RunConfig(name="bench", storage_path=store, verbose=0),
                     torch_config=TorchConfig(backend=backend)).fit()
        return 0
    except TrainingFailedError as e:
        print(f"bench.py: a rank failed: {e}", file=sys.stderr)
        return 1
    finally:
        shutil.rmtree(store, ignore_errors=True)


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != a.gpus:
            print(f"bench.py: WORLD_SIZE={env_world} from the launcher but --gpus {a.gpus}; refusing to "
                  f"benchmark a different number of ranks than requested", file=sys.stderr)
            sys.exit(2)
    elif a.gpus > 1:
        sys.exit(launch_workers(a))
    a.launcher = a.launcher or ("torch.distributed.run" if env_world is not None else "in-process")
    run(a)


class _Progress:
    """Phase lines on stderr (rank 0) outside the timed region; with ``--heartbeat N`` also the current
    phase every N seconds from a daemon thread, for long runs (a 70B offload build) under a runner that
    treats a silent process as hung. Nothing is printed between the timing barriers."""

    def __init__(self, enabled: bool, every: float):
        import threading
        self.enabled, self.name, self.t0, self.quiet = enabled, "start", time.perf_counter(), False
        self._stop = threading.Event()
        if enabled and every > 0:
            def beat():
                while not self._stop.wait(every):
                    if not self.quiet:
                        print(f"bench.py: [{time.perf_counter() - self.t0:.0f} s] {self.name}", file=sys.stderr, flush=True)
            threading.Thread(target=beat, daemon=True).start()

    def phase(self, name: str):
        self.name = name
        if self.enabled:
            print(f"bench.py: [{time.perf_counter() - self.t0:.0f} s] {name}", file=sys.stderr, flush=True)

    def stop(self):
        self._stop.set()


def run(a):
    if a.ipc:
        os.environ["GRT_IPC_COLLECTIVES"] = "1"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    cpu = a.device == "cpu"
    if cpu:
        dev = torch.device("cpu")
    else:
        # one rank per GPU; ranks beyond the visible GPUs share them (rehearsal with --backend gloo)
        idx = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(idx)
        dev = torch.device("cuda", idx)
        if os.environ.get("GRT_COMPUTE_STREAM_PRIORITY", "normal") == "high":
            # the training step on a high-priority stream: the side streams (overlapped AdamW,
            # grad-norm partials, gathers) keep the default priority and yield to it
            torch.cuda.set_stream(torch.cuda.Stream(dev, priority=torch.cuda.Stream.priority_range()[1]))
    if a.force_collectives:
        os.environ["GRT_FORCE_COLLECTIVES"] = "1"
    if (world > 1 or a.force_collectives) and not dist.is_initialized():
        backend = a.backend or ("gloo" if cpu else "nccl")
        if world == 1:  # one-rank group for the forced-collective rehearsal
            import socket
            with socket.socket() as s_:
                s_.bind(("127.0.0.1", 0))
                port = s_.getsockname()[1]
            dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                    device_id=dev if backend == "nccl" else None)
        else:
            dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
    pg_world = dist.get_world_size() if dist.is_initialized() else 1
    if pg_world != world:
        raise SystemExit(f"bench.py: process group has {pg_world} ranks but WORLD_SIZE={world}")

    from gke_ray_train_amd.data import TokenBatchLoader, synthetic_tokens
    from gke_ray_train_amd.models import get_config

    a.sp_group = None
    if a.sp > 1:
        if world % a.sp or a.parallel != "ddp" or a.peft != "none":
            raise SystemExit("--sp needs world % sp == 0 and the DDP engine without PEFT")
        for g0 in range(0, world, a.sp):  # every rank creates every group (collective)
            grp = dist.new_group(list(range(g0, g0 + a.sp)))
            if g0 <= rank < g0 + a.sp:
                a.sp_group = grp
    dp_world, dp_rank = world // a.sp, rank // a.sp

    torch.manual_seed(1234)
    dtype = torch.float32 if cpu else torch.bfloat16
    tuned = False
    if not cpu and not a.no_tuned_gemm:
        from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms
        tuned = enable_tuned_gemms()
    cfg = get_config(a.model)
    if a.layers and a.layers < cfg.num_hidden_layers:
        full = cfg.num_hidden_layers
        cfg = get_config(a.model, num_hidden_layers=a.layers)
        cfg.name = f"{cfg.name}[{a.layers}/{full} layers]"
    from gke_ray_train_amd.parallel.planner import GiB, plan_memory
    plan_world = a.proxy_world if (a.proxy_world > 1 and world == 1) else world
    plan = plan_memory(cfg, plan_world, a.parallel, offload=a.offload, peft=a.peft, micro_batch=a.micro_batch or a.batch,
                       seq=a.seq, zero=(a.zero == "on" or (a.zero == "auto" and (plan_world > 1 or a.force_collectives))),
                       checkpointing=a.checkpointing, lora_r=a.lora_r,
                       hbm_capacity=None if not cpu else float("inf"))
    if a.proxy_world > 1 and world == 1:
        plan.host_ranks_here = 1  # this process holds rank 0's host state only
    a.resident_fraction = 0.0
    a.prefetch_slots = 0
    if a.offload and a.parallel == "fsdp":
        from gke_ray_train_amd.parallel.offload import (PREFETCH_CAP_BYTES, hbm_reserve_bytes, prefetch_slots_for,
                                                        resident_fraction_from_plan)
        if a.offload_resident == "auto":
            a.resident_fraction = resident_fraction_from_plan(plan, None)
        else:
            a.resident_fraction = float(a.offload_resident)
        moved = plan.host_per_rank.get("adam_moments_fp32", 0.0)
        streamed = (1.0 - a.resident_fraction) * moved
        room = max(0.0, plan.hbm_capacity - plan.hbm_total - a.resident_fraction * moved - hbm_reserve_bytes())
        budget = (min(streamed, PREFETCH_CAP_BYTES, room) if a.offload_prefetch_gib == "auto"
                  else float(a.offload_prefetch_gib) * GiB)
        a.prefetch_slots = prefetch_slots_for(budget, 1 << 26)
        plan.hbm_per_rank["offload_resident_moments"] = a.resident_fraction * moved
        plan.hbm_per_rank["offload_prefetch_ring"] = a.prefetch_slots * 8.0 * (1 << 26)
    if a.plan_only:
        if rank == 0:
            print(json.dumps({"memory_plan": plan.to_dict()}), flush=True)
        if dist.is_initialized():
            dist.destroy_process_group()
        return
    if not plan.fits:  # refuse up front with the numbers instead of an allocator error mid-step
        print(f"bench.py: memory preflight failed for {cfg.name} {a.parallel} world={world}: "
              + "; ".join(plan.problems()), file=sys.stderr, flush=True)
        sys.exit(3)
    t_build = time.perf_counter()
    progress = _Progress(rank == 0, a.heartbeat)
    progress.phase(f"building {cfg.name} ({a.parallel}, world {world})")
    model, eng, call, opt = build(a, cfg, dev, dtype, world)
    model.train()
    progress.phase(f"model and optimizer built in {time.perf_counter() - t_build:.1f} s; warm-up")

    mb = a.micro_batch or a.batch
    assert a.batch % mb == 0
    accum = a.batch // mb
    total_micro = (a.warmup + a.steps) * accum
    if a.data == "loader":
        toks = synthetic_tokens(max(total_micro * mb * a.seq * world + a.seq + 2, 1 << 20), cfg.vocab_size, seed=7)
        loader = TokenBatchLoader(toks, a.seq, mb, device=dev, rank=dp_rank, world=dp_world, shuffle=True, seed=3,
                                  stride=a.seq)
        it = iter(loader)

        def next_batch(_i):
            return next(it)[0]
    elif a.data == "pipeline":
        # Ray-Data streaming (BASELINE config #4): windowed shuffle -> map_batches, ONE execution in
        # a coordinator process (rank 0 hosts it) dealing equal row shares to the ranks, pinned-ring
        # H2D prefetch on a copy stream (data/pipeline.py)
        if a.sp > 1:
            raise SystemExit("--data pipeline deals one split per data-parallel rank; use it with --sp 1")
        from gke_ray_train_amd.data.pipeline import Dataset
        n_win = total_micro * mb * dp_world + 8 * dp_world
        toks = synthetic_tokens(n_win * a.seq, cfg.vocab_size, seed=7)
        ds = (Dataset.from_numpy({"input_ids": toks.reshape(n_win, a.seq)}, parallelism=max(16, 4 * dp_world))
              .random_shuffle(seed=3)
              .map_batches(lambda b: {"input_ids": b["input_ids"].astype(np.int64)}))
        split = ds.streaming_split_for_rank(dp_rank, dp_world)
        it = iter(split.iter_torch_batches(batch_size=mb, device=dev, drop_last=True, prefetch_batches=4))

        def next_batch(_i):
            return next(it)["input_ids"]
    else:
        g = torch.Generator(device=dev)
        g.manual_seed(dp_rank + 17)  # ranks of one SP group share their sequences
        batches = [torch.randint(0, cfg.vocab_size, (mb, a.seq), device=dev, generator=g) for _ in range(4 * accum)]

        def next_batch(i):
            return batches[i % len(batches)]

    fsdp = a.parallel == "fsdp"
    counter = [0]
    from gke_ray_train_amd.observability import StepMeter
    meter = None
    if a.metrics_jsonl:
        fpt_m = cfg.flops_per_token(a.seq) * (2.0 / 3.0 if a.peft != "none" else 1.0)
        meter = StepMeter(a.batch * a.seq * world, fpt_m, n_gpus=world, samples_per_step=a.batch * world,
                          jsonl=a.metrics_jsonl, rank=rank, device=dev)
    nullctx = contextlib.nullcontext

    def ph(name):
        return meter.phase(name) if meter is not None else nullctx()

    def step():
        for j in range(accum):
            ids = next_batch(counter[0])
            counter[0] += 1
            with eng.no_sync(j < accum - 1):
                with ph("forward"):
                    if a.sp > 1:  # this rank's S/sp tokens of its SP group's sequences
                        from gke_ray_train_amd.parallel.sequence import shard_sequence
                        ids_l, lab_l, w = shard_sequence(ids, a.sp_group)
                        loss = call(ids_l, shifted_labels=lab_l)["loss"] * (w / accum)
                    else:
                        loss = call(ids, labels=ids)["loss"] / accum
                with ph("backward"):
                    loss.backward()
        with ph("grad_sync"):
            eng.finish_gradient_sync()
        with ph("optimizer"):
            st = eng.clip_grad_norm_(a.max_grad_norm)  # global norm of the averaged gradient, on device
            opt.step(grad_scale=st)
            if not fsdp:
                eng.after_optimizer_step()  # ZeRO: async all-gather of the updated shards
            eng.zero_grad()
        return loss

    def timed_step(i):
        if meter is None:
            return step()
        with meter.step(i):
            loss = step()
        meter.log(i, loss=loss * accum)
        return loss

    for _ in range(a.warmup):
        loss = step()
    if not fsdp:
        eng.wait_params()
    progress.phase(f"{a.warmup} warm-up steps issued; timing {a.steps} steps")
    if not cpu:
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if not cpu:
        torch.cuda.synchronize()
    prof = None
    if a.profile_dir and rank == 0:
        from torch.profiler import ProfilerActivity, profile
        stacks = os.environ.get("GRT_PROFILE_STACKS", "0") == "1"  # attribute kernels to Python call sites
        prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=stacks, with_stack=stacks)
        prof.__enter__()
    progress.quiet = True  # no heartbeat lines inside the timed region
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = timed_step(i)
    if not fsdp:
        eng.wait_params()  # the last step's parameter all-gather belongs to the timed work
    if not cpu:
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if not cpu:
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    progress.stop()
    if world > 1:  # a failed xGMI IPC collective (parallel/ipc.py) fails the run instead of timing it
        from gke_ray_train_amd.parallel.ipc import check_all
        check_all()
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(a.profile_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(a.profile_dir, "trace.json"))
        with open(os.path.join(a.profile_dir, "kernels.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
            if stacks:
                f.write("\n\n" + prof.key_averages(group_by_stack_n=6).table(sort_by="cuda_time_total", row_limit=80))
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev if not cpu else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = 1000.0 * elapsed / a.steps
    tokens_per_step = a.batch * a.seq * (world // a.sp)
    tps = tokens_per_step / (elapsed / a.steps)
    fpt = cfg.flops_per_token(a.seq)
    if a.peft != "none":
        fpt = fpt * 2.0 / 3.0  # frozen base: no weight-gradient GEMMs (adapter FLOPs are negligible)
    mfu = tps / world * fpt / 2.5e15
    proxy = getattr(eng, "proxy", False)
    par = f"{'fsdp' if fsdp else 'dp'}{world // a.sp}" + (f"-proxy{a.proxy_world}" if proxy else "") + \
        (f"+sp{a.sp}" if a.sp > 1 else "") + ("+zero1" if getattr(eng, "zero", False) else "") + \
        ("+offload" if a.offload else "") + \
        ("" if a.peft == "none" else f"+{a.peft}")
    if rank == 0:
        out = {
            "metric": _baseline_metric(),
            "value": round(tps, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if not cpu else "fp32",
            "data": "synthetic Wikitext-2-shaped token stream (Zipf ids) via "
                    + {"loader": "the streaming loader", "pipeline": "the Ray-Data-like streaming pipeline (coordinated streaming_split, pinned-ring H2D)",
                       "static": "on-device batches"}[a.data] + "; random-init weights",
            "config": {"model": cfg.name, "global_batch": a.batch * (world // a.sp), "seq_len": a.seq, "parallelism": par,
                       "micro_batch": mb, "grad_accum": accum, "optimizer": "fused AdamW fp32 states",
                       "max_grad_norm": a.max_grad_norm, "activation_checkpointing": a.checkpointing,
                       "optimizer_overlap": type(opt).__name__ == "OverlappedOptimizer",
                       "forced_collectives": bool(a.force_collectives),
                       "library_gemms": "offline-tuned" if tuned else "default"},
            "samples_per_sec": round(tps / a.seq, 2),
            "pg_world_size": pg_world,
            "pg_backend": dist.get_backend() if dist.is_initialized() else "none",
            "launcher": a.launcher,
            "proxy_world": a.proxy_world if proxy else None,
            "offload_resident_units": getattr(opt, "resident_units", None) if a.offload else None,
            "offload_units": len(getattr(opt, "segments", [])) if a.offload else None,
            "offload_prefetch_slots": getattr(opt, "prefetch_slots", None) if a.offload else None,
            "offload_resident_fraction": round(a.resident_fraction, 3) if a.offload else None,
            # streamed moment bytes per step against the host link over the MEASURED step time
            "offload_link": _link_plan(plan, a, elapsed / a.steps) if a.offload else None,
            "mfu_bf16_dense": round(mfu, 4),
            "hbm_plan_gib": round(plan.hbm_total / GiB, 1),
            "hbm_peak_gib": round(torch.cuda.max_memory_allocated(dev) / GiB, 1) if not cpu else None,
            "loss": round(float(loss.item()) * accum, 4),
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
