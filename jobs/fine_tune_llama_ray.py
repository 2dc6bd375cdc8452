#!/usr/bin/env python3
"""QLoRA / LoRA / full SFT of a Llama model through TorchTrainer (reference:
ray-jobs/fine_tune_llama_ray.py + fine_tune_config.json — all 35 keys are honoured).

Offline differences (documented): the base model is the named architecture with random-init
weights (or a local HF-layout directory in MODEL_ID), the tokenizer is the framework's byte-level
tokenizer with Llama-3 chat special tokens, and the gretel text-to-SQL rows are synthetic (same
columns, 1000 train / 200 eval after shuffle(seed=42)). Everything else follows the reference: NF4
4-bit base + LoRA r/alpha/dropout on the 7 projections (USE_QLORA), bf16 compute, paged-AdamW
alias, cosine schedule with warmup ratio, grad accumulation, group_by_length, eval/save steps,
TensorBoard logs, rank-0 ``merge_and_unload`` + ``save_pretrained``, optional greedy side-by-side
inference comparison written to ``inference_comparison_results.json``.

Extra (BASELINE config #4): ``USE_LORA_BF16`` = LoRA on an unquantized bf16 base.
"""
from __future__ import annotations

import json
import os

# kernel arguments in device memory (read by the HIP runtime at its first call; launch-time setting)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gke_ray_train_amd import train  # noqa: E402
from gke_ray_train_amd.train import ScalingConfig  # noqa: E402
from gke_ray_train_amd.train.torch import TorchTrainer  # noqa: E402


def _load_base(model_id, device, dtype, seed=0):
    from gke_ray_train_amd.models.hub import from_pretrained
    return from_pretrained(model_id, device=device, torch_dtype=dtype, random_init_seed=seed)


def run_inference_comparison(original_model_id, path_to_fine_tuned_model, eval_rows, max_seq_len, results_output_dir,
                             device, max_new_generation_tokens=150, tokenizer=None):
    """Greedy generation of the original vs fine-tuned model on 'window functions' samples."""
    from gke_ray_train_amd.data.tokenizer import ByteTokenizer
    from gke_ray_train_amd.trainer.sft_data import format_chat_sample
    from gke_ray_train_amd.models.hub import from_pretrained
    tok = tokenizer or ByteTokenizer.from_pretrained(path_to_fine_tuned_model)
    try:
        tuned = from_pretrained(path_to_fine_tuned_model, device=device, torch_dtype=torch.bfloat16).eval()
        orig = _load_base(original_model_id, device, torch.bfloat16).eval()
    except Exception as e:  # reference: log and return (:42-82)
        print(f"[rank 0] inference comparison skipped: cannot load models: {e}")
        return None
    samples = [r for r in eval_rows if r.get("sql_complexity", "").lower() == "window functions"]
    results = []
    eos = [tok.eos_token_id, tok.convert_tokens_to_ids("<|eot_id|>")]
    budget = max(50, max_seq_len - max_new_generation_tokens) if max_seq_len > max_new_generation_tokens else max(50, max_seq_len // 2)
    for i, s in enumerate(samples):
        prompt = format_chat_sample(s, tok, with_answer=False)["text"]
        ids = torch.tensor([tok.encode(prompt)[:budget]], device=device)
        outs = {}
        for name, m in (("original", orig), ("fine_tuned", tuned)):
            g = m.generate(ids, max_new_tokens=max_new_generation_tokens, eos_token_id=eos, pad_token_id=tok.eos_token_id)
            outs[name] = tok.decode(g[0, ids.shape[1]:].tolist(), skip_special_tokens=True).strip()
        results.append({"id": s.get("id", f"unknown_id_{i}"), "schema_context": s.get("sql_context", ""),
                        "question_prompt": s.get("sql_prompt", ""), "original_model_input_prompt": prompt,
                        "fine_tuned_model_input_prompt": prompt, "ground_truth_sql": s.get("sql", ""),
                        "original_model_sql_response": outs["original"],
                        "fine_tuned_model_sql_response": outs["fine_tuned"]})
    os.makedirs(results_output_dir, exist_ok=True)
    path = os.path.join(results_output_dir, "inference_comparison_results.json")
    with open(path, "w") as f:
        json.dump(results, f, indent=4)
    del tuned, orig
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    return path


def train_loop_per_worker(config: dict):
    from gke_ray_train_amd.data.tokenizer import ByteTokenizer
    from gke_ray_train_amd.peft import BitsAndBytesConfig, LoraConfig, quantize_model_
    from gke_ray_train_amd.trainer import SFTConfig, SFTTrainer, format_chat_sample, synthetic_text_to_sql

    ctx = train.get_context()
    rank, world = ctx.get_world_rank(), ctx.get_world_size()
    device = train.torch.get_device()
    print(f"rank {rank}/{world} starting on {device}", flush=True)
    compute_dtype = getattr(torch, config["BNB_4BIT_COMPUTE_DTYPE"]) if config["USE_QLORA"] else torch.bfloat16
    if device.type == "cpu":
        compute_dtype = torch.float32
    model = _load_base(config["MODEL_ID"], device, compute_dtype, seed=config.get("SEED", 0))
    tokenizer = ByteTokenizer(model.config.vocab_size)
    tokenizer.pad_token = tokenizer.eos_token
    tokenizer.padding_side = "right"
    if rank == 0:
        os.makedirs(config["OUTPUT_DIR_BASE"], exist_ok=True)
    lora = None
    if config["USE_QLORA"]:
        quantize_model_(model, BitsAndBytesConfig(load_in_4bit=True, bnb_4bit_quant_type=config["BNB_4BIT_QUANT_TYPE"],
                                                  bnb_4bit_compute_dtype=compute_dtype,
                                                  bnb_4bit_use_double_quant=config["USE_NESTED_QUANT"]))
    if config["USE_QLORA"] or config.get("USE_LORA_BF16"):
        lora = LoraConfig(lora_alpha=config["LORA_ALPHA"], lora_dropout=config["LORA_DROPOUT"], r=config["LORA_R"],
                          bias="none", task_type="CAUSAL_LM", target_modules=config["LLAMA_TARGET_MODULES"])
    n_train, n_eval = config.get("NUM_TRAIN_SAMPLES", 1000), config.get("NUM_EVAL_SAMPLES", 200)
    train_rows = synthetic_text_to_sql(max(n_train, 1), seed=42, split="train")
    eval_rows = synthetic_text_to_sql(max(n_eval, 1), seed=42, split="test")
    train_ds = [format_chat_sample(r, tokenizer) for r in train_rows]
    eval_ds = [format_chat_sample(r, tokenizer) for r in eval_rows]
    sft_dir = os.path.join(config["OUTPUT_DIR_BASE"], config["SFT_SUBDIR_NAME"])
    args = SFTConfig(
        num_train_epochs=config["NUM_TRAIN_EPOCHS"], per_device_train_batch_size=config["PER_DEVICE_TRAIN_BATCH_SIZE"],
        gradient_accumulation_steps=config["GRADIENT_ACCUMULATION_STEPS"], optim=config["OPTIM"],
        learning_rate=config["LEARNING_RATE"], lr_scheduler_type=config["LR_SCHEDULER_TYPE"],
        warmup_ratio=config["WARMUP_RATIO"], max_grad_norm=config["MAX_GRAD_NORM"], weight_decay=config["WEIGHT_DECAY"],
        bf16=compute_dtype == torch.bfloat16, group_by_length=config["GROUP_BY_LENGTH"],
        max_seq_length=config["MAX_SEQ_LENGTH"], packing=config["PACKING"], dataset_text_field="text",
        output_dir=sft_dir, logging_steps=config["LOGGING_STEPS"], save_strategy=config["SAVE_STRATEGY"],
        report_to=config["REPORT_TO"], evaluation_strategy=config["EVALUATION_STRATEGY_SFT"],
        eval_steps=config["EVAL_STEPS_SFT"], save_steps=config["SAVE_STEPS_SFT"],
        max_steps=config.get("MAX_STEPS", -1), gradient_checkpointing=config.get("GRADIENT_CHECKPOINTING", False))
    trainer = SFTTrainer(model=model, args=args, train_dataset=train_ds, eval_dataset=eval_ds, peft_config=lora,
                         processing_class=tokenizer)
    if rank == 0 and lora is not None:
        trainer.model.print_trainable_parameters()
    print(f"rank {rank}: SFTTrainer.train()", flush=True)
    result = trainer.train()
    print(f"rank {rank}: training finished. metrics: {result.metrics}", flush=True)

    saved = None
    if rank == 0:
        if lora is not None:
            out = os.path.join(config["OUTPUT_DIR_BASE"], config["MERGED_MODEL_SUBDIR_NAME"])
            try:
                merged = trainer.model.merge_and_unload()
                merged.save_pretrained(out)
                tokenizer.save_pretrained(out)
                saved = out
                del merged
            except Exception as e:  # reference keeps the adapters and skips inference (:358-365)
                print(f"[rank 0] merge failed ({e}); adapters remain in {sft_dir}")
        else:
            out = os.path.join(config["OUTPUT_DIR_BASE"], config["FULL_FT_MODEL_SUBDIR_NAME"])
            trainer.model.save_pretrained(out)
            tokenizer.save_pretrained(out)
            saved = out
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        if config["INFERENCE"] and saved and os.path.exists(saved):
            run_inference_comparison(config["MODEL_ID"], saved, eval_rows, config["MAX_SEQ_LENGTH"],
                                     config["OUTPUT_DIR_BASE"], device,
                                     config["MAX_NEW_GENERATION_TOKENS_INFERENCE"], tokenizer=tokenizer)
    train.report(dict(result.metrics, saved_model=saved or ""))


def load_config(path=None, overrides=None):
    """fine_tune_config.json (same 35 keys) validated / typed by utils.config.FineTuneConfig."""
    from gke_ray_train_amd.utils.config import FineTuneConfig, load_json_config, to_dict
    path = path or os.path.join(os.path.dirname(os.path.abspath(__file__)), "fine_tune_config.json")
    cfg = to_dict(load_json_config(FineTuneConfig, path, overrides))
    # the reference writes under its /mnt/pvc bucket mount: "pvc/..." resolves to the cluster storage
    pvc = os.environ.get("GRT_PVC") or os.environ.get("GRT_STORAGE_PATH")
    if pvc and str(cfg.get("OUTPUT_DIR_BASE", "")).startswith("pvc/"):
        cfg["OUTPUT_DIR_BASE"] = os.path.join(pvc, cfg["OUTPUT_DIR_BASE"][4:])
    return cfg


def main(config=None, num_workers=None, use_gpu=None):
    cfg = config or load_config()
    if use_gpu is None:
        use_gpu = torch.cuda.device_count() > 0  # counting does not initialise HIP in the driver
    if num_workers is None:
        n_nodes = int(os.getenv("NUM_NODES", "1"))
        n_gpu = int(os.getenv("NUM_GPUS_PER_NODE", str(torch.cuda.device_count() if use_gpu else 1)))
        num_workers = n_nodes * n_gpu
    trainer = TorchTrainer(train_loop_per_worker, train_loop_config=cfg,
                           scaling_config=ScalingConfig(num_workers=num_workers, use_gpu=use_gpu,
                                                        resources_per_worker={"GPU": 1} if use_gpu else None))
    t0 = time.time()
    result = trainer.fit()
    print(f"Fine-tuning job completed in {time.time() - t0:.1f}s")
    print(f"Results: {result.metrics}" if result.metrics else "No metrics returned from TorchTrainer result.")
    print(f"SFT outputs were saved to: {os.path.join(cfg['OUTPUT_DIR_BASE'], cfg['SFT_SUBDIR_NAME'])}")
    return result


if __name__ == "__main__":
    import argparse
    from gke_ray_train_amd.utils.config import num_workers_from_env, parse_overrides
    ap = argparse.ArgumentParser(description="Llama SFT (QLoRA / LoRA / full) through TorchTrainer")
    ap.add_argument("--config", default=None, help="JSON config (default: jobs/fine_tune_config.json)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE", help="override a config key")
    ap.add_argument("--num-workers", type=int, default=None,
                    help="default: NUM_NODES x NUM_GPUS_PER_NODE (GPUs per node = visible MI355X count)")
    ap.add_argument("--cpu", action="store_true", help="gloo CPU workers (plumbing runs)")
    a = ap.parse_args()
    cfg = load_config(a.config, parse_overrides(a.set))
    nw = a.num_workers or (num_workers_from_env() if not a.cpu else 1)
    main(cfg, num_workers=nw, use_gpu=False if a.cpu else None)
