#!/usr/bin/env python3
"""TunableOp-tune every library GEMM of a LoRA / QLoRA training step (the skinny adapter GEMMs:
x A^T, h B^T accumulated into y, dY B, dY^T h, g^T x) on top of the shipped table, and write the
merged table to --out. Run on an MI355X; A/B the result with GRT_TUNED_GEMM_FILE=<out> before
adopting it."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.ops.gemm_tuning import RESULTS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="gpurun_out/tunableop_lora.csv")
ap.add_argument("--model", default="llama2-7b")
ap.add_argument("--peft", default="lora", choices=["lora", "qlora"])
ap.add_argument("--rows", type=int, default=8, help="sequences per step (SFT: batch 2 x accumulation 4 fused)")
ap.add_argument("--seqs", default="1024", help="padded sequence lengths to tune at (M = rows x seq)")
ap.add_argument("--duration", type=int, default=20, help="max tuning ms per shape")
ap.add_argument("--base", default="", help="start from this results file instead of the shipped table")
a = ap.parse_args()

from gke_ray_train_amd.models import build_llama, get_config  # noqa: E402
from gke_ray_train_amd.parallel import DistributedDataParallel  # noqa: E402
from gke_ray_train_amd.peft import BitsAndBytesConfig, LoraConfig, get_peft_model, quantize_model_  # noqa: E402

# no rotating operand copies: TunableOp sizes them from the leading dimensions, which overruns
# the allocation for column-block views (the "HIP error: invalid argument" abort of round 2)
os.environ.setdefault("PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE", "0")
tun = torch.cuda.tunable
tun.enable(True)
tun.read_file(a.base or str(RESULTS))
tun.tuning_enable(True)
tun.set_max_tuning_duration(a.duration)
tun.set_max_tuning_iterations(30)
os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
tun.set_filename(a.out)

cfg = get_config(a.model)
dev = torch.device("cuda", 0)
model = build_llama(cfg, device=dev, dtype=torch.bfloat16, seed=1)
if a.peft == "qlora":
    quantize_model_(model, BitsAndBytesConfig(bnb_4bit_compute_dtype=torch.bfloat16))
pm = get_peft_model(model, LoraConfig(r=64, lora_alpha=16, lora_dropout=0.1))
ddp = DistributedDataParallel(pm)
for L in [int(x) for x in a.seqs.split(",")]:
    ids = torch.randint(0, cfg.vocab_size, (a.rows, L), device=dev)
    loss = pm(ids, labels=ids)["loss"]
    loss.backward()
    ddp.finish_gradient_sync()
    ddp.zero_grad()
    torch.cuda.synchronize()
    print(f"M = {a.rows * L} tuned", flush=True)
tun.tuning_enable(False)
with open(a.out, "w") as fh:
    for k, v in tun.get_validators():
        fh.write(f"Validator,{k},{v}\n")
    for op_sig, param_sig, kernel, ms in tun.get_results():
        fh.write(f"{op_sig},{param_sig},{kernel},{ms}\n")
print("results:", a.out, sum(1 for _ in open(a.out)), "lines", flush=True)
