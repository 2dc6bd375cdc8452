"""SFT trainer with HF-Trainer / TRL-SFTTrainer semantics on the framework's engines.

Reference: ``SFTConfig(...)`` + ``SFTTrainer(model, args, train_dataset, eval_dataset,
peft_config).train()`` inside ``train_loop_per_worker`` (ray-jobs/fine_tune_llama_ray.py:295-334)
with every key of fine_tune_config.json: gradient accumulation with ``no_sync`` on
non-boundary micro-steps, ``max_grad_norm`` clipping, the ``optim`` / ``lr_scheduler_type`` /
``warmup_ratio`` / ``weight_decay`` choices, ``group_by_length``, ``packing``, ``logging_steps``
(loss averaged across ranks), ``eval_steps``, ``save_steps`` -> ``checkpoint-<step>/`` (adapter or
full weights, optimizer.pt, scheduler.pt, trainer_state.json, training_args.bin, rng_state_<rank>.pth),
``save_total_limit``, ``report_to="tensorboard"`` (events under ``<output_dir>/runs/``), and the
``train_result.metrics`` the reference prints (train_runtime, train_samples_per_second, ...).

MI355X specifics: the model runs on the HIP ops; data parallelism is the flat-buffer RCCL DDP over
the TRAINABLE parameters only (LoRA: 0.67 GB of fp32-equivalent grads per step instead of the
whole model); clipping + AdamW are the two fused device passes; batches are right-padded to a
multiple of 8 by the native collator and copied from pinned memory. On the GPU the
gradient-accumulation micro-batches of one optimizer step run as ONE padded batch whose loss
weights keep each micro-batch's own mean (``fuse_accumulation``): the same update as HF's
accumulation loop with 4x larger GEMMs (reference SFT job on one MI355X: 17.8 -> 24.5+ samples/s).
"""
from __future__ import annotations

import glob
import json
import math
import os
import random
import shutil
import socket
import time
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, List, Optional, Union

import numpy as np
import torch
import torch.distributed as dist

from ..observability import roctx
from ..observability.metrics import MI355X_PEAK_BF16_DENSE
from ..ops import clip_grad_norm_, make_optimizer
from ..parallel.comm import small_all_reduce
from ..parallel.ddp import DistributedDataParallel
from .schedules import get_scheduler
from .sft_data import LengthGroupedSampler, PadCollator, pack_sequences


@dataclass
class SFTConfig:
    output_dir: str = "outputs"
    num_train_epochs: float = 1.0
    max_steps: int = -1
    per_device_train_batch_size: int = 8
    per_device_eval_batch_size: int = 8
    gradient_accumulation_steps: int = 1
    optim: str = "adamw_torch"
    learning_rate: float = 5e-5
    lr_scheduler_type: str = "linear"
    warmup_ratio: float = 0.0
    warmup_steps: int = 0
    max_grad_norm: float = 1.0
    weight_decay: float = 0.0
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_epsilon: float = 1e-8
    bf16: bool = False
    fp16: bool = False
    group_by_length: bool = False
    max_seq_length: int = 1024
    packing: bool = False
    dataset_text_field: str = "text"
    logging_steps: int = 500
    logging_dir: Optional[str] = None
    save_strategy: str = "steps"
    save_steps: int = 500
    save_total_limit: Optional[int] = None
    report_to: Union[str, List[str]] = "none"
    evaluation_strategy: Optional[str] = None
    eval_strategy: str = "no"
    eval_steps: Optional[int] = None
    seed: int = 42
    gradient_checkpointing: bool = False
    dataloader_drop_last: bool = False
    max_length: Optional[int] = None
    master_weights: bool = False
    disable_tqdm: bool = True
    # MI355X execution plan (not HF keys): run the gradient-accumulation micro-batches of one
    # optimizer step as ONE padded batch (up to fuse_max_tokens tokens per forward) with each
    # micro-batch's own loss mean kept through per-token loss weights — the same gradient, bigger
    # GEMMs. None = on for GPU models whose forward takes ``loss_weights``.
    fuse_accumulation: Optional[bool] = None
    fuse_max_tokens: int = 16384
    # fused batches are right-padded to a multiple of this length: whole 128-row attention tiles
    # and token counts that avoid hipBLASLt's slow tilings of odd M (measured on the reference SFT
    # job: 128 -> +7 % tokens/s over 8 despite the extra padding, profiles/r1_sft_job_kernel_breakdown.md)
    fuse_pad_multiple: int = 128
    # padding-free packing of each fused step (``ops.Varlen``): the step's sequences are concatenated
    # on one token axis (attention inside each sequence, RoPE positions restarting), so no GEMM,
    # norm or loss row is spent on padding; only the total is rounded up to fuse_pad_multiple with
    # one masked filler segment. Same loss and gradient as the padded batch. None = on for GPU
    # models whose forward takes ``varlen`` (with fused accumulation); GRT_SFT_PADDING_FREE=0/1
    # overrides. Reference SFT job, interleaved on one box: 33.7 / 33.6 vs 33.3 / 33.4 samples/s
    # padded, once the packed token counts were in the GEMM table and varlen attention dropped the
    # causal pairs (profiles/r3_lora_grad_gemms.md, r3_varlen_attention.md).
    padding_free: Optional[bool] = None
    # packed steps: micro-batches are grouped while their REAL tokens stay within pack_max_tokens,
    # and the packed length is rounded up to pack_multiple (the token counts the GEMM table is
    # tuned at: tools/tune_lora_gemms.py --rows 1 --seqs <multiples>)
    pack_max_tokens: int = 8192
    pack_multiple: int = 512
    # evaluation forwards: token cap per fused / packed chunk (the training step's sizes, which the
    # GEMM table is tuned at; 16 K-token eval chunks ran on untuned shapes)
    eval_max_tokens: int = 8192
    # evaluation batches packed padding-free (None: whenever the model supports it, see
    # SFTTrainer._eval_padding_free)
    eval_padding_free: Optional[bool] = None

    def __post_init__(self):
        if self.evaluation_strategy is not None:  # deprecated alias used by the reference (:317)
            self.eval_strategy = self.evaluation_strategy
        if self.max_length:
            self.max_seq_length = self.max_length
        if self.eval_steps is None:
            self.eval_steps = self.logging_steps
        if self.fp16:
            raise ValueError("fp16 is not supported on this stack; use bf16")

    def to_dict(self):
        return asdict(self)


@dataclass
class TrainOutput:
    global_step: int
    training_loss: float
    metrics: Dict[str, float]


def _world():
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _to_host(obj):
    """Deep copy with every tensor moved to host memory (checkpoint snapshot)."""
    if isinstance(obj, torch.Tensor):
        return obj.detach().to("cpu", copy=True)
    if isinstance(obj, dict):
        return {k: _to_host(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_host(v) for v in obj)
    return obj


class _HostSnapshot:
    """Device -> host checkpoint snapshot. Every CUDA tensor of the state is copied asynchronously
    into ONE pinned host buffer (reserved when the trainer is built, kept for later saves) and the
    stream is synchronised once — instead of one synchronous pageable copy per tensor (~1,350 for
    the reference job's adapters + AdamW moments, ~0.9 s of the step-50/100 pause).
    ``materialize`` (run on the writer thread) clones each slice into a tensor of its own, because
    torch.save / safetensors store a view's whole storage."""

    def __init__(self):
        self.buf = None

    @staticmethod
    def _leaves(obj, out):
        if isinstance(obj, torch.Tensor):
            if obj.is_cuda:
                out.append(obj)
        elif isinstance(obj, dict):
            for v in obj.values():
                _HostSnapshot._leaves(v, out)
        elif isinstance(obj, (list, tuple)):
            for v in obj:
                _HostSnapshot._leaves(v, out)
        return out

    @staticmethod
    def _nbytes(t):
        return -(-t.numel() * t.element_size() // 64) * 64

    def reserve(self, nbytes: int):
        if nbytes > 0 and (self.buf is None or self.buf.numel() < nbytes):
            self.buf = None
            self.buf = torch.empty(int(nbytes), dtype=torch.uint8, pin_memory=True)

    def take(self, obj):
        leaves = self._leaves(obj, [])
        self.reserve(sum(self._nbytes(t) for t in leaves))
        views, off = {}, 0
        for t in leaves:
            n = t.numel() * t.element_size()
            v = self.buf[off:off + n].view(t.dtype).view(t.shape)
            v.copy_(t.detach(), non_blocking=True)
            views[id(t)] = v
            off += self._nbytes(t)
        if leaves:
            torch.cuda.current_stream(leaves[0].device).synchronize()

        def rebuild(o):
            if isinstance(o, torch.Tensor):
                return views[id(o)] if o.is_cuda else o.detach().clone()
            if isinstance(o, dict):
                return {k: rebuild(v) for k, v in o.items()}
            if isinstance(o, (list, tuple)):
                return type(o)(rebuild(v) for v in o)
            return o
        return rebuild(obj)

    @staticmethod
    def materialize(obj):
        if isinstance(obj, torch.Tensor):
            return obj.clone()
        if isinstance(obj, dict):
            return {k: _HostSnapshot.materialize(v) for k, v in obj.items()}
        if isinstance(obj, (list, tuple)):
            return type(obj)(_HostSnapshot.materialize(v) for v in obj)
        return obj


def _rng_snapshot() -> Dict[str, Any]:
    """Every RNG a training step draws from, in a form ``torch.load(weights_only=True)`` reads
    back (numpy's key array as a tensor). The CPU generator also seeds the dropout kernels
    (``ops.fused.dropout_seed_offset``), so restoring it resumes the dropout-mask sequence."""
    name, keys, pos, has_gauss, cached = np.random.get_state()
    rng = {"python": random.getstate(), "cpu": torch.get_rng_state(),
           "numpy": {"name": name, "keys": torch.from_numpy(keys.astype(np.int64)), "pos": int(pos),
                     "has_gauss": int(has_gauss), "cached": float(cached)}}
    if torch.cuda.is_available():
        rng["cuda"] = torch.cuda.get_rng_state_all()
    return rng


def _rng_restore(rng: Dict[str, Any]):
    random.setstate(rng["python"])
    torch.set_rng_state(rng["cpu"])
    n = rng.get("numpy")
    if isinstance(n, dict):
        np.random.set_state((n["name"], n["keys"].numpy().astype(np.uint32), n["pos"], n["has_gauss"], n["cached"]))
    elif isinstance(n, (tuple, list)) and len(n) == 5:  # HF / legacy layout: np.random.get_state() itself
        np.random.set_state(tuple(n))
    cu = rng.get("cuda")
    if cu is not None and torch.cuda.is_available():
        if isinstance(cu, torch.Tensor):  # HF single-GPU layout
            torch.cuda.set_rng_state(cu)
        elif len(cu) == torch.cuda.device_count():
            torch.cuda.set_rng_state_all(cu)


def _rng_load(path: str) -> Optional[Dict[str, Any]]:
    """Read an rng_state_<rank>.pth without executing pickled code: weights_only first, then
    weights_only with numpy's array-reconstruction globals allow-listed (HF checkpoints and the
    pre-round-3 layout keep ``np.random.get_state()``'s ndarray). An unreadable file is skipped
    with a warning — resuming with fresh RNG streams beats refusing to resume."""
    try:
        return torch.load(path, weights_only=True)
    except Exception:
        pass
    try:
        core = getattr(np, "_core", None) or np.core
        allowed = [core.multiarray._reconstruct, np.ndarray, np.dtype]
        allowed += [getattr(np.dtypes, n) for n in ("UInt32DType", "Int64DType", "Float64DType") if hasattr(np, "dtypes")]
        with torch.serialization.safe_globals(allowed):
            return torch.load(path, weights_only=True)
    except Exception as e:  # noqa: BLE001
        import warnings
        warnings.warn(f"cannot restore RNG state from {path} ({e.__class__.__name__}: {e}); continuing with fresh streams")
        return None


def _rank_uniform_error(err: Optional[BaseException], world: int, what: str):
    """Raise on EVERY rank if any rank failed ``what``: the ranks exchange a failure flag first,
    so a failure on one rank cannot leave the others blocked in the next collective."""
    failed = err is not None
    if world > 1:
        flag = torch.tensor([1 if failed else 0], dtype=torch.int32,
                            device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(flag)
        failed = bool(flag.item())
    if err is not None:
        raise RuntimeError(f"{what} failed") from err
    if failed:
        raise RuntimeError(f"{what} failed on another rank")


def _rows(ds) -> List[Dict[str, Any]]:
    if ds is None:
        return []
    if hasattr(ds, "take_all"):
        return ds.take_all()
    return [r for r in ds]


class SFTTrainer:
    def __init__(self, model, args: SFTConfig, train_dataset=None, eval_dataset=None, peft_config=None,
                 processing_class=None, tokenizer=None, data_collator=None, callbacks=None, formatting_func=None):
        self.args = args
        self.rank, self.world = _world()
        self.tokenizer = processing_class or tokenizer
        if self.tokenizer is None:
            from ..data.tokenizer import ByteTokenizer
            self.tokenizer = ByteTokenizer(model.config.vocab_size)
        if getattr(self.tokenizer, "pad_token", None) is None:
            self.tokenizer.pad_token = self.tokenizer.eos_token
        self.pad_id = self.tokenizer.pad_token_id if self.tokenizer.pad_token_id is not None else self.tokenizer.eos_token_id
        if peft_config is not None:
            from ..peft import get_peft_model
            model = get_peft_model(model, peft_config)
        self.model = model
        self.peft_config = peft_config
        if args.gradient_checkpointing:
            inner = getattr(model, "base_model", model)
            if hasattr(inner, "gradient_checkpointing_enable"):
                inner.gradient_checkpointing_enable()
        self.device = next(model.parameters()).device
        if self.device.type == "cuda":
            from ..ops.gemm_tuning import enable_tuned_gemms
            enable_tuned_gemms()  # stored TunableOp winners for the listed projection shapes
        self.callbacks = list(callbacks or [])
        self.formatting_func = formatting_func
        self.train_seqs = self._prepare(train_dataset)
        self.eval_seqs = self._prepare(eval_dataset)
        self.collator = data_collator or PadCollator(self.pad_id, 8, args.max_seq_length)
        torch.manual_seed(args.seed)
        random.seed(args.seed)
        np.random.seed(args.seed)
        # The engine choices of bench.py's headline step (the same config #2 path): full fine-tuning
        # at world > 1 shards the AdamW state (ZeRO: bucketed reduce-scatter during backward, the
        # updated shards all-gathered under the next forward, W^T written at forward time); at world 1
        # (and for adapter models, whose replicated update is small) the AdamW update runs per module
        # on a side stream overlapped with the next forward and writes W^T for the TN dX GEMMs
        # (parallel/overlap.py). GRT_SFT_ZERO=0 / GRT_SFT_OVERLAP_OPT=0 select the plain paths.
        adapters = hasattr(getattr(model, "base_model", model), "lora_modules") or hasattr(model, "lora_modules")
        zero = self.world > 1 and not adapters and os.environ.get("GRT_SFT_ZERO", "1") != "0"
        self.engine = DistributedDataParallel(model, broadcast_params=True, shard_optimizer=zero)
        self.optimizer = make_optimizer(args.optim, self.engine.optimizer_param_groups(args.weight_decay),
                                        lr=args.learning_rate, weight_decay=args.weight_decay,
                                        betas=(args.adam_beta1, args.adam_beta2), eps=args.adam_epsilon,
                                        master_weights=args.master_weights)
        from ..ops.optim import FusedAdamW
        if (self.device.type == "cuda" and not self.engine.zero and type(self.optimizer) is FusedAdamW
                and os.environ.get("GRT_SFT_OVERLAP_OPT", "1") != "0"):
            from ..parallel.overlap import OverlappedOptimizer
            self.optimizer = OverlappedOptimizer(self.engine, self.optimizer)
        self._snapshot = _HostSnapshot()
        if self.device.type == "cuda":
            self._prepare_device()
        self.scheduler = None
        self.state = {"global_step": 0, "epoch": 0.0, "log_history": [], "best_metric": None,
                      "best_model_checkpoint": None, "total_flos": 0.0}
        self.tb = None
        rt = args.report_to if isinstance(args.report_to, list) else [args.report_to]
        if "tensorboard" in rt and self.rank == 0:
            from .tb import SummaryWriter
            ldir = args.logging_dir or os.path.join(args.output_dir, "runs",
                                                    time.strftime("%b%d_%H-%M-%S") + "_" + socket.gethostname())
            self.tb = SummaryWriter(ldir)

    def _prepare_device(self):
        """One-time device preparation while the trainer is constructed (as model loading /
        quantisation is, before ``train()``): the frozen base's derived layouts (K-concatenated
        LoRA weights, NF4 dequant caches, W^T of the dX GEMMs: ``PeftModel.prepare_frozen_weights``)
        and the GEMM library's first-call initialisation. Each is built once either way; measured
        on the reference SFT job they made the first optimizer step ~1.8 s slower than the rest
        (``GRT_SFT_STEP_TRACE=1``). ``GRT_SFT_PREPARE=0`` leaves them to the first step."""
        if os.environ.get("GRT_SFT_PREPARE", "1") == "0":
            return
        prep = getattr(self.model, "prepare_frozen_weights", None)
        if prep is not None:
            prep()
        a = torch.ones(256, 256, device=self.device, dtype=torch.bfloat16)
        (a @ a).sum().item()  # hipBLASLt handle, workspace and the tuned-solution table
        if self.args.save_strategy != "no" and self.rank == 0 and hasattr(self.model, "lora_modules"):
            # pinned checkpoint snapshot: trainable parameters + two fp32 AdamW moments each
            tr = [p for p in self.model.parameters() if p.requires_grad]
            self._snapshot.reserve(sum(p.numel() * (p.element_size() + 8) + 128 for p in tr) + (1 << 20))

    # ------------------------------------------------------------------ data
    def _prepare(self, ds) -> List[List[int]]:
        rows = _rows(ds)
        if not rows:
            return []
        a = self.args
        texts = []
        for r in rows:
            if self.formatting_func is not None:
                texts.append(self.formatting_func(r))
            elif isinstance(r, str):
                texts.append(r)
            else:
                texts.append(r[a.dataset_text_field])
        seqs = [self.tokenizer.encode(t)[: a.max_seq_length] for t in texts]
        if a.packing:
            seqs = pack_sequences(seqs, a.max_seq_length, self.tokenizer.eos_token_id)
        return seqs

    def _batches(self, seqs, bs, epoch, shuffle=True):
        n = len(seqs)
        if self.args.group_by_length and shuffle:
            sampler = LengthGroupedSampler([len(s) for s in seqs], bs, self.world, self.rank, self.args.seed)
            sampler.set_epoch(epoch)
            idx = list(iter(sampler))
        else:
            order = list(range(n))
            if shuffle:
                g = random.Random(self.args.seed + epoch)
                g.shuffle(order)
            per = n // self.world if self.args.dataloader_drop_last else -(-n // self.world)
            idx = [order[(self.rank + i * self.world) % n] for i in range(per)] if n else []
        out = []
        for i in range(0, len(idx), bs):
            chunk = idx[i:i + bs]
            if len(chunk) < bs and self.args.dataloader_drop_last:
                break
            out.append(self.collator([seqs[j] for j in chunk]))
        return out

    def _fuse_enabled(self) -> bool:
        a = self.args
        if a.gradient_accumulation_steps <= 1:
            return False
        if a.fuse_accumulation is not None:
            return bool(a.fuse_accumulation)
        if os.environ.get("GRT_SFT_FUSE_ACCUM", "1") == "0" or self.device.type != "cuda":
            return False
        import inspect
        inner = getattr(self.model, "base_model", self.model)
        try:
            return "loss_weights" in inspect.signature(inner.forward).parameters
        except (TypeError, ValueError):
            return False

    def _padding_free_enabled(self) -> bool:
        a = self.args
        if a.padding_free is not None:
            return bool(a.padding_free)
        env = os.environ.get("GRT_SFT_PADDING_FREE")
        if env is not None and env != "1":
            return False
        if env is None and self.device.type != "cuda":  # default: GPU only
            return False
        import inspect
        inner = getattr(self.model, "base_model", self.model)
        try:
            return "varlen" in inspect.signature(inner.forward).parameters
        except (TypeError, ValueError):
            return False

    def _pack(self, g, mult: int, weighted: bool):
        """Micro-batches ``g`` -> one padding-free packed row (see ``SFTConfig.padding_free``)."""
        accum = self.args.gradient_accumulation_steps
        ids, labs, wts, lens = [], [], [], []
        ntarget = 0
        for b in g:
            lengths = b["attention_mask"].sum(1).tolist()
            n = int(((b["labels"][:, 1:] != -100) & (b["attention_mask"][:, 1:] != 0)).sum())
            w = 1.0 / (n * accum) if n else 0.0
            for r, L in enumerate(lengths):
                L = int(L)
                if L == 0:
                    continue
                keep = b["attention_mask"][r] != 0
                if bool(keep[:L].all()):  # right padding (the reference collator's): the row's prefix
                    rid, rlab = b["input_ids"][r, :L], b["labels"][r, :L]
                else:  # any other mask (left padding, holes): select the real tokens by the mask
                    rid, rlab = b["input_ids"][r][keep], b["labels"][r][keep]
                ids.append(rid)
                labs.append(rlab)
                wts.append(torch.full((L,), w))
                lens.append(L)
                ntarget += int((rlab[1:] != -100).sum())
        T = sum(lens)
        pad = (-T) % max(1, mult)
        mask = torch.ones(T + pad, dtype=torch.long)
        if pad:  # one masked filler segment: keeps the token count on the tuned GEMM sizes
            ids.append(torch.full((pad,), self.pad_id, dtype=ids[0].dtype))
            labs.append(torch.full((pad,), -100, dtype=labs[0].dtype))
            wts.append(torch.zeros(pad))
            lens.append(pad)
            mask[T:] = 0
        out = {"input_ids": torch.cat(ids).view(1, -1), "labels": torch.cat(labs).view(1, -1),
               "attention_mask": mask.view(1, -1), "lengths": lens, "ntarget": ntarget}
        return out, (torch.cat(wts).view(1, -1) if weighted else None)

    def _pack_chunks(self, batches, mis, weighted: bool, max_tokens: Optional[int] = None):
        """Padding-free grouping: micro-batches join a packed row while the row's real tokens stay
        within ``pack_max_tokens``; each row is then rounded up to ``pack_multiple`` tokens."""
        a = self.args
        mult = int(os.environ.get("GRT_SFT_PAD_MULTIPLE", "0")) or a.pack_multiple or 1
        cap = max(max_tokens or a.pack_max_tokens, a.max_seq_length)
        groups, cur, cur_tok = [], [], 0
        for mi in mis:
            b = batches[mi]
            n = int(b["attention_mask"].sum())
            if cur and cur_tok + n > cap:
                groups.append(cur)
                cur, cur_tok = [], 0
            cur.append(b)
            cur_tok += n
        if cur:
            groups.append(cur)
        return [self._pack(g, mult, weighted) for g in groups]

    def _eval_padding_free(self) -> bool:
        """Evaluation packs its batches padding-free whenever the model takes ``varlen`` (forward
        only: no per-step GEMM-shape concern; eval_runtime 2.37 -> 2.19 s on the reference SFT job,
        profiles/r3_sft_job_trace.md). ``eval_padding_free=False`` / GRT_SFT_EVAL_PADDING_FREE=0: padded."""
        a = self.args
        if a.eval_padding_free is not None:
            return bool(a.eval_padding_free)
        if os.environ.get("GRT_SFT_EVAL_PADDING_FREE", "1") == "0":
            return False
        if self.device.type != "cuda":
            return self._padding_free_enabled()
        import inspect
        inner = getattr(self.model, "base_model", self.model)
        try:
            return "varlen" in inspect.signature(inner.forward).parameters
        except (TypeError, ValueError):
            return False

    def _step_chunks(self, batches, mis, fuse, weighted: bool = True, max_tokens: Optional[int] = None,
                     padding_free: Optional[bool] = None):
        """The micro-batches ``mis`` of one optimizer step -> [(batch, loss_weights | None)].
        Unfused: one entry per micro-batch (loss = mean / accum). Fused: micro-batches are right-
        padded to a common length and concatenated while the padded size stays within
        ``fuse_max_tokens``; every position of micro-batch m carries weight 1 / (n_m * accum)
        (n_m = its valid next-token labels), so the weighted-sum loss and its gradient equal the
        sum of the unfused micro-batch losses."""
        if not fuse:
            return [(batches[mi], None) for mi in mis]
        if self._padding_free_enabled() if padding_free is None else padding_free:
            return self._pack_chunks(batches, mis, weighted, max_tokens)
        accum = self.args.gradient_accumulation_steps
        mult = int(os.environ.get("GRT_SFT_PAD_MULTIPLE", "0")) or self.args.fuse_pad_multiple or 1
        cap = max(self.args.max_seq_length, 1)

        def padded(L):  # round up, but never past max_seq_length (unless already longer)
            return max(L, min(-(-L // mult) * mult, cap))

        groups, cur, cur_len, cur_rows = [], [], 0, 0
        for mi in mis:
            b = batches[mi]
            L, R = padded(b["input_ids"].shape[1]), b["input_ids"].shape[0]
            nl, nr = max(cur_len, L), cur_rows + R
            if cur and nl * nr > (max_tokens or self.args.fuse_max_tokens):
                groups.append(cur)
                cur, nl, nr = [], L, R
            cur.append(b)
            cur_len, cur_rows = nl, nr
        if cur:
            groups.append(cur)
        out = []
        for g in groups:
            L = padded(max(b["input_ids"].shape[1] for b in g))
            pads = {"input_ids": self.pad_id, "labels": -100, "attention_mask": 0}
            merged = {k: torch.cat([torch.nn.functional.pad(b[k], (0, L - b[k].shape[1]), value=v) for b in g])
                      for k, v in pads.items()}
            ws = []
            for b in g:
                n = int(((b["labels"][:, 1:] != -100) & (b["attention_mask"][:, 1:] != 0)).sum())
                ws.append(torch.full((b["input_ids"].shape[0], L), 1.0 / (n * accum) if n else 0.0))
            out.append((merged, torch.cat(ws)))
        return out

    def _to_dev(self, b):
        out = {k: (v.pin_memory().to(self.device, non_blocking=True) if self.device.type == "cuda" else v.to(self.device))
               for k, v in b.items() if isinstance(v, torch.Tensor)}
        if "lengths" in b:
            from ..ops import Varlen
            out["varlen"] = Varlen(b["lengths"], self.device)
        return out

    # ------------------------------------------------------------------ train
    def train(self, resume_from_checkpoint: Optional[str] = None) -> TrainOutput:
        a = self.args
        bs, accum = a.per_device_train_batch_size, a.gradient_accumulation_steps
        micro_per_epoch = len(self._batches(self.train_seqs, bs, 0, shuffle=False))
        steps_per_epoch = max(1, math.ceil(micro_per_epoch / accum))
        total = a.max_steps if a.max_steps > 0 else math.ceil(a.num_train_epochs * steps_per_epoch)
        warm = a.warmup_steps or math.ceil(a.warmup_ratio * total)
        # LambdaLR needs the torch optimizer; an OverlappedOptimizer shares its param_groups
        self.scheduler = get_scheduler(a.lr_scheduler_type, getattr(self.optimizer, "opt", self.optimizer), warm, total)
        start_step = 0
        if resume_from_checkpoint:
            start_step = self._load_checkpoint(resume_from_checkpoint)
        self.model.train()
        t0 = time.time()
        tr_loss_sum = torch.zeros((), device=self.device)
        log_loss = torch.zeros((), device=self.device)
        log_count = 0
        ntok = 0
        nsamples = 0
        self._pending_logs = []
        self._log_mark = (self._now_marker(), 0)  # (device event | host time, tokens) of the last log
        cfg = getattr(getattr(self.model, "base_model", self.model), "config", None)
        fpt = 0.0
        if cfg is not None and hasattr(cfg, "flops_per_token"):
            fpt = cfg.flops_per_token(a.max_seq_length)
            if self.peft_config is not None:
                fpt *= 2.0 / 3.0  # frozen base weights: no weight-gradient GEMMs
        step = start_step
        epochs = math.ceil(total / steps_per_epoch)
        done = False
        fuse = self._fuse_enabled()
        trace = [] if os.environ.get("GRT_SFT_STEP_TRACE") == "1" and self.rank == 0 else None
        for epoch in range(start_step // steps_per_epoch, epochs):
            batches = self._batches(self.train_seqs, bs, epoch)
            skip = (start_step - epoch * steps_per_epoch) if epoch == start_step // steps_per_epoch else 0
            nb = len(batches)
            for gi in range(max(0, skip), steps_per_epoch):
                mis = list(range(gi * accum, min(nb, (gi + 1) * accum)))
                if not mis:
                    break
                if step >= total:  # resumed at (or past) max_steps: nothing left to train
                    done = True
                    break
                mi = mis[-1]
                chunks = self._step_chunks(batches, mis, fuse)
                if trace is not None:  # diagnosis only: synchronises every step
                    self._sync()
                    t_step = time.time()
                for ci, (cb, lw) in enumerate(chunks):
                    ntok += int(cb["attention_mask"].sum())  # CPU tensor: no device sync
                    b = self._to_dev(cb if lw is None else dict(cb, loss_weights=lw))
                    with self.engine.no_sync(ci != len(chunks) - 1):
                        with roctx.range("forward"):
                            vk = {"varlen": b["varlen"]} if "varlen" in b else {}
                            if lw is None:
                                out = self.model(b["input_ids"], labels=b["labels"], attention_mask=b["attention_mask"],
                                                 **vk)
                                loss = out["loss"] / accum
                            else:
                                loss = self.model(b["input_ids"], labels=b["labels"], attention_mask=b["attention_mask"],
                                                  loss_weights=b["loss_weights"], **vk)["loss"]
                        with roctx.range("backward"):
                            loss.backward()
                    tr_loss_sum += loss.detach()
                    log_loss += loss.detach()
                    nsamples += (len(cb["lengths"]) - int(int(cb["attention_mask"][0, -1]) == 0)
                                 if "lengths" in cb else b["input_ids"].shape[0])
                with roctx.range("grad_sync"):
                    self.engine.finish_gradient_sync()
                with roctx.range("optimizer"):
                    # global norm of the averaged gradient (early per-bucket norms at world 1, the
                    # sharded all-reduce under ZeRO), applied by the fused update on device
                    st = self.engine.clip_grad_norm_(a.max_grad_norm)
                    self.optimizer.step(grad_scale=st)
                    self.engine.after_optimizer_step()  # ZeRO: all-gather the updated shards
                self.scheduler.step()
                self.engine.zero_grad()
                if trace is not None:
                    self._sync()
                    trace.append((step + 1, round((time.time() - t_step) * 1e3, 2),
                                  [tuple(c["input_ids"].shape) for c, _ in chunks],
                                  sum(int(c["attention_mask"].sum()) for c, _ in chunks)))
                step += 1
                log_count += 1
                self.state["global_step"] = step
                self.state["epoch"] = epoch + (mi + 1) / nb
                if a.logging_steps and step % a.logging_steps == 0:
                    self._stage_log(log_loss / log_count, st, ntok, fpt)
                    log_loss.zero_()
                    log_count = 0
                self._emit_logs()  # the staged entries whose values have landed (no device sync)
                t_aux = time.time()
                if a.eval_strategy == "steps" and self.eval_seqs and a.eval_steps and step % a.eval_steps == 0:
                    self._emit_logs(wait=True)
                    self.evaluate()
                t_save = time.time()
                if a.save_strategy == "steps" and a.save_steps and step % a.save_steps == 0:
                    self._emit_logs(wait=True)
                    self._save_checkpoint(step)
                if trace is not None and time.time() - t_aux > 1e-3:
                    trace.append((step, "eval", round((t_save - t_aux) * 1e3, 2), "save",
                                  round((time.time() - t_save) * 1e3, 2), getattr(self, "_save_times", None)))
                if step >= total:
                    done = True
                    break
            if a.eval_strategy == "epoch" and self.eval_seqs:
                self.evaluate()
            if a.save_strategy == "epoch":
                self._save_checkpoint(step)
            if done:
                break
        self._emit_logs(wait=True)
        self._settle()
        self._finish_save()  # the runtime includes the last checkpoint's write
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        rt = time.time() - t0
        if trace is not None:
            with open(os.path.join(a.output_dir, "step_trace.jsonl"), "w") as f:
                for row in trace:
                    f.write(json.dumps(row) + "\n")
            print(f"step trace: {len(trace)} rows -> {a.output_dir}/step_trace.jsonl", flush=True)
        train_loss = self._mean_across_ranks(tr_loss_sum / max(1, step - start_step))
        gsamples = nsamples * self.world
        metrics = {"train_runtime": round(rt, 4), "train_samples_per_second": round(gsamples / rt, 3),
                   "train_steps_per_second": round((step - start_step) / rt, 3),
                   "total_flos": float(self.state["total_flos"]), "train_loss": train_loss,
                   "train_tokens_per_second": round(ntok * self.world / rt, 1),
                   "epoch": round(self.state["epoch"], 4)}
        self.state["log_history"].append(dict(metrics, step=step))
        for cb in self.callbacks:
            if hasattr(cb, "on_train_end"):
                cb.on_train_end(self, metrics)
        if self.tb is not None:
            self.tb.flush()
        return TrainOutput(step, train_loss, metrics)

    # ------------------------------------------------------------------ deferred logging
    # A logging step used to read the loss and grad norm with .item(), draining the device queue:
    # the GPU then idled while the host printed and prepared the next step (~17 ms per log on the
    # reference SFT job). The values are instead copied into pinned memory behind an event and the
    # entry is emitted once the event has completed (checked every step; forced before evaluation,
    # checkpoints and the end of training). tokens_per_sec spans device events, i.e. device time
    # between logging steps.
    def _now_marker(self):
        if self.device.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.time()

    def _stage_log(self, mean_loss: torch.Tensor, st, ntok: int, fpt: float):
        vals = torch.stack([mean_loss.detach().float().reshape(()), st.norm.detach().float().reshape(())])
        if self.world > 1:
            loss = vals[:1].clone()
            small_all_reduce(loss)
            vals = torch.cat([loss / self.world, vals[1:]])
        if self.device.type == "cuda":
            host = torch.empty(2, dtype=torch.float32, pin_memory=True)
            host.copy_(vals, non_blocking=True)
        else:
            host = vals
        meta = {"learning_rate": self.scheduler.get_last_lr()[0], "epoch": round(self.state["epoch"], 4),
                "step": self.state["global_step"]}
        if self.world > 1 and self.device.type == "cuda":  # IPC error words, read when the log is emitted
            from ..parallel.ipc import stage_errors
            meta["ipc_errs"] = stage_errors()
        self._pending_logs.append((self._now_marker(), host, meta, ntok, fpt))

    def _emit_logs(self, wait: bool = False):
        while getattr(self, "_pending_logs", None):
            mark, host, meta, ntok, fpt = self._pending_logs[0]
            if not isinstance(mark, float):
                if wait:
                    mark.synchronize()
                elif not mark.query():
                    return
            self._pending_logs.pop(0)
            if meta.get("ipc_errs"):  # a failed xGMI IPC collective fails the run here (fail-stop)
                from ..parallel.ipc import raise_staged
                raise_staged(meta["ipc_errs"])
            prev, ntok_prev = self._log_mark
            if isinstance(mark, float):
                dt = max(mark - prev, 1e-9)
            else:
                dt = max(prev.elapsed_time(mark) / 1e3, 1e-9)
            loss, norm = (float(x) for x in host.tolist())
            logs = {"loss": loss, "grad_norm": norm, "learning_rate": meta["learning_rate"], "epoch": meta["epoch"],
                    "tokens_per_sec": round((ntok - ntok_prev) * self.world / dt, 1)}
            if fpt:
                logs["mfu"] = round((ntok - ntok_prev) / dt * fpt / MI355X_PEAK_BF16_DENSE, 4)
            logs["step"] = meta["step"]
            self._log_mark = (mark, ntok)
            self._log(logs)

    def _settle(self):
        """Parameters final: pending overlapped chunk updates and ZeRO all-gathers complete."""
        if hasattr(self.optimizer, "synchronize"):
            self.optimizer.synchronize()
        self.engine.wait_params()

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def _mean_across_ranks(self, t: torch.Tensor) -> float:
        t = t.detach().float().reshape(1).clone()
        if self.world > 1:
            small_all_reduce(t)
            t /= self.world
        return float(t.item())

    def _log(self, logs: Dict[str, float]):
        logs = dict(logs)
        logs.setdefault("step", self.state["global_step"])
        self.state["log_history"].append(logs)
        if self.rank == 0:
            print({k: (round(v, 6) if isinstance(v, float) else v) for k, v in logs.items()}, flush=True)
            os.makedirs(self.args.output_dir, exist_ok=True)
            with open(os.path.join(self.args.output_dir, "metrics.jsonl"), "a") as f:
                f.write(json.dumps(dict(logs, time=time.time())) + "\n")
            if self.tb is not None:
                for k, v in logs.items():
                    if k not in ("step", "epoch") and isinstance(v, (int, float)):
                        self.tb.add_scalar(f"train/{k}" if not k.startswith("eval_") else k.replace("eval_", "eval/"),
                                           v, logs["step"])
        for cb in self.callbacks:
            if hasattr(cb, "on_log"):
                cb.on_log(self, logs)

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def evaluate(self) -> Dict[str, float]:
        was = self.model.training
        self.model.eval()
        t0 = time.time()
        tot = torch.zeros(2, device=self.device, dtype=torch.float64)
        batches = self._batches(self.eval_seqs, self.args.per_device_eval_batch_size, 0, shuffle=False)
        if self._fuse_enabled():  # same token-weighted mean from fewer, larger forwards
            batches = [cb for cb, _ in self._step_chunks(batches, list(range(len(batches))), True, weighted=False,
                                                         max_tokens=self.args.eval_max_tokens,
                                                         padding_free=self._eval_padding_free())]
        with torch.no_grad():  # as HF's prediction_step: no saved activations, no fused CE gradient
            for cb in batches:
                b = self._to_dev(cb)
                vk = {"varlen": b["varlen"]} if "varlen" in b else {}
                loss = self.model(b["input_ids"], labels=b["labels"], attention_mask=b["attention_mask"], **vk)["loss"]
                n = cb["ntarget"] if "ntarget" in cb else (
                    (b["labels"][:, 1:] != -100) & (b["attention_mask"][:, 1:] != 0)).sum()
                tot[0] += loss.double() * n
                tot[1] += n
        if self.world > 1:
            dist.all_reduce(tot)
        tot = tot.cpu()  # the runtime covers the device work, not just its enqueueing
        rt = time.time() - t0
        m = {"eval_loss": float(tot[0] / tot[1].clamp_min(1)), "eval_runtime": round(rt, 4),
             "eval_samples_per_second": round(len(self.eval_seqs) / max(rt, 1e-9), 3),
             "epoch": round(self.state["epoch"], 4)}
        self._log(m)
        if was:
            self.model.train()
        return m

    # ------------------------------------------------------------------ save / load
    def _unwrapped(self):
        return self.model

    def save_model(self, output_dir: Optional[str] = None):
        out = output_dir or self.args.output_dir
        if self.rank == 0:
            m = self._unwrapped()
            if hasattr(m, "save_pretrained") and hasattr(m, "lora_modules"):
                m.save_pretrained(out)
            else:
                from ..models.hub import save_pretrained
                save_pretrained(m, out)
            if hasattr(self.tokenizer, "save_pretrained"):
                self.tokenizer.save_pretrained(out)

    def _save_checkpoint(self, step: int):
        """``checkpoint-<step>/`` (HF layout). For adapter models rank 0 snapshots the adapter and
        optimizer tensors to host memory (~2 GB for Llama-3.1-8B r=64, tens of ms) and writes the
        files on a background thread while training continues; full-model checkpoints are written
        synchronously. The previous write is always finished before a new one starts, before
        ``train`` returns and before a checkpoint is loaded."""
        tm = [time.time()]
        self._finish_save()
        self._settle()
        if self.world > 1 and self.device.type == "cuda":  # a failed IPC collective fails the save
            from ..parallel.ipc import check_all
            check_all()
        tm.append(time.time())
        a = self.args
        d = os.path.join(a.output_dir, f"checkpoint-{step}")
        job = None
        err = None
        sharded_opt = bool(getattr(self.engine, "zero", False))
        # optimizer.pt in HF's per-parameter layout at every world size and sharding: collective
        # (ZeRO gathers each bucket's 1/world chunks to rank 0), so every rank calls it; the file
        # then resumes at any world size (load_portable_optimizer_state_dict)
        portable = hasattr(self.engine, "portable_optimizer_state_dict")
        port_sd, port_err = None, None
        if portable:
            try:
                port_sd = self.engine.portable_optimizer_state_dict(self.optimizer)
            except Exception as e:  # noqa: BLE001 -- agreed below with the other ranks
                port_err = e
        if self.rank == 0:
            try:
                os.makedirs(d, exist_ok=True)
                m = self._unwrapped()
                is_adapter = hasattr(m, "adapter_state_dict") and hasattr(m, "lora_modules")
                snap = self._snapshot if self.device.type == "cuda" and is_adapter else None
                if port_err is not None:
                    raise port_err
                opt_sd = port_sd if portable else self.optimizer.state_dict()
                if snap is not None:  # ONE pinned snapshot of optimizer state (+ adapters)
                    host = snap.take({"o": opt_sd, "a": m.adapter_state_dict() if is_adapter else None})
                else:
                    host = {"o": _to_host(opt_sd), "a": _to_host(m.adapter_state_dict()) if is_adapter else None}
                tm.append(time.time())
                files = {"scheduler.pt": self.scheduler.state_dict(), "training_args.bin": a.to_dict(),
                         "optimizer.pt": host["o"]}
                st = dict(self.state, train_batch_size=a.per_device_train_batch_size, max_steps=a.max_steps,
                          logging_steps=a.logging_steps, save_steps=a.save_steps, eval_steps=a.eval_steps,
                          grt_optimizer_layout={"format": "per-parameter" if portable else "flat",
                                                "zero": sharded_opt, "world": self.world})
                st = json.loads(json.dumps(st))  # frozen copy: the live state keeps changing
                adapter = None
                if is_adapter:
                    adapter = host["a"]
                    m.save_adapter_config(d)
                    if hasattr(self.tokenizer, "save_pretrained"):
                        self.tokenizer.save_pretrained(d)
                else:
                    self.save_model(d)

                def job():
                    if adapter is not None:
                        from safetensors.torch import save_file
                        save_file(_HostSnapshot.materialize(adapter) if snap is not None else adapter,
                                  os.path.join(d, "adapter_model.safetensors"))
                    for name, obj in files.items():
                        torch.save(_HostSnapshot.materialize(obj) if snap is not None else obj, os.path.join(d, name))
                    with open(os.path.join(d, "trainer_state.json"), "w") as f:
                        json.dump(st, f, indent=2)
            except Exception as e:  # reported on every rank below, not raised ahead of the others
                err, job = e, None
        tm.append(time.time())
        try:
            os.makedirs(d, exist_ok=True)
            torch.save(_rng_snapshot(), os.path.join(d, f"rng_state_{self.rank}.pth"))
        except Exception as e:
            err = err or e
        err = err or port_err
        # every rank reaches this exchange, so a failed snapshot raises everywhere (no hang)
        _rank_uniform_error(err, self.world, f"checkpoint {d}")
        # the async decision must be identical on every rank: _finish_save exchanges the outcome
        use_async = os.environ.get("GRT_ASYNC_CHECKPOINT", "1") != "0"
        self._pending = (d, job)
        self._save_thread = None
        self._save_error = None
        if job is not None:
            if use_async:
                import threading
                def run(job=job):
                    try:
                        job()
                    except BaseException as e:  # surfaced by _finish_save on the training thread
                        self._save_error = e
                self._save_thread = threading.Thread(target=run, name="grt-ckpt", daemon=False)
                self._save_thread.start()
            else:
                try:
                    job()
                except Exception as e:
                    self._save_error = e
        if not use_async:
            self._finish_save()
        tm.append(time.time())
        self._save_times = [round((b - a_) * 1e3, 1) for a_, b in zip(tm[:-1], tm[1:])]  # step trace

    def _finish_save(self):
        """Complete the pending checkpoint: join the writer, rotate old checkpoints, run callbacks.
        A failed write on rank 0 raises on every rank (flag exchanged before anyone raises)."""
        pending = getattr(self, "_pending", None)
        if pending is None:
            return
        d, _ = pending
        t = getattr(self, "_save_thread", None)
        if t is not None:
            t.join()
            self._save_thread = None
        self._pending = None
        err, self._save_error = getattr(self, "_save_error", None), None
        _rank_uniform_error(err, self.world, f"writing checkpoint {d}")
        a = self.args
        if self.rank == 0 and a.save_total_limit:
            ck = sorted(glob.glob(os.path.join(a.output_dir, "checkpoint-*")), key=lambda p: int(p.rsplit("-", 1)[1]))
            for old in ck[:-a.save_total_limit]:
                shutil.rmtree(old, ignore_errors=True)
        for cb in self.callbacks:
            if hasattr(cb, "on_save"):
                cb.on_save(self, d)

    def _load_checkpoint(self, d: str) -> int:
        self._finish_save()
        m = self._unwrapped()
        if hasattr(m, "load_adapter") and os.path.exists(os.path.join(d, "adapter_model.safetensors")):
            m.load_adapter(d)
        else:
            from ..models.hub import from_pretrained
            loaded = from_pretrained(d, device=self.device, torch_dtype=next(m.parameters()).dtype)
            m.load_state_dict(loaded.state_dict())
        with open(os.path.join(d, "trainer_state.json")) as f:
            st = json.load(f)
        zero_now = bool(getattr(self.engine, "zero", False))
        layout = st.pop("grt_optimizer_layout", None)
        if layout is not None and layout.get("format") == "per-parameter":
            # HF per-parameter layout: resumes at any world size / sharding
            sd = torch.load(os.path.join(d, "optimizer.pt"), map_location="cpu", weights_only=True, mmap=True)
            self.engine.load_portable_optimizer_state_dict(self.optimizer, sd)
            del sd
            return self._finish_load(d, st)
        if layout is not None:  # legacy flat layout: must match (a shard is 1/world of the flat state)
            if bool(layout.get("zero")) != zero_now or (zero_now and int(layout.get("world", -1)) != self.world):
                raise ValueError(
                    f"{d}: optimizer state was written {'ZeRO-sharded' if layout.get('zero') else 'unsharded'} "
                    f"at world {layout.get('world')}; this run is {'ZeRO-sharded' if zero_now else 'unsharded'} "
                    f"at world {self.world}. Resume with the same world size and GRT_SFT_ZERO setting.")
        shard = os.path.join(d, f"optimizer_rank{self.rank}.pt")
        if zero_now and not os.path.exists(shard):
            raise FileNotFoundError(f"{d}: sharded (ZeRO) optimizer state for rank {self.rank} is missing "
                                    f"(checkpoint written at another world size?)")
        opt_f = shard if zero_now else os.path.join(d, "optimizer.pt")
        if not os.path.exists(opt_f):
            raise FileNotFoundError(f"{d}: {os.path.basename(opt_f)} is missing (checkpoint written with a ZeRO-sharded "
                                    f"optimizer? its state is in optimizer_rank<r>.pt)")
        self.optimizer.load_state_dict(torch.load(opt_f, map_location=self.device, weights_only=True))
        return self._finish_load(d, st)

    def _finish_load(self, d: str, st: dict) -> int:
        self.scheduler.load_state_dict(torch.load(os.path.join(d, "scheduler.pt"), weights_only=True))
        self.state.update(st)
        rp = os.path.join(d, f"rng_state_{self.rank}.pth")
        if os.path.exists(rp):  # continue the RNG streams (dropout masks, sampler) where they stopped
            rng = _rng_load(rp)
            if rng is not None:
                _rng_restore(rng)
        return int(st["global_step"])
