#!/usr/bin/env python3
"""Forward + backward cost of one LoRA step by packed token count (padding-free ``Varlen``) vs the
padded [rows, S] batch of the same tokens: where the SFT job's packed steps at odd multiples of
512 tokens lose (profiles/r3_sft_job_trace.md). Llama-3.1-8B-shaped, random init, LoRA r=64 on the
7 targets, dropout 0.1; prints one JSON line per config.

  python tools/varlen_probe.py --cfgs 5120,5632,6144,6656 [--padded 8x768] [--only 5632]
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--cfgs", default="5120,5632,6144,6656,7168,7680")
    ap.add_argument("--padded", default="8x640,8x768,8x896")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--layers", type=int, default=0)
    a = ap.parse_args()
    from gke_ray_train_amd.models import build_llama
    from gke_ray_train_amd.ops.fused import Varlen
    from gke_ray_train_amd.peft import LoraConfig, get_peft_model
    from gke_ray_train_amd.ops.gemm_tuning import enable_tuned_gemms
    dev = torch.device("cuda", 0)
    if os.environ.get("GRT_TUNED_GEMMS", "1") != "0":
        enable_tuned_gemms()
    model = build_llama(a.model, device=dev, dtype=torch.bfloat16, seed=0,
                        **({"num_hidden_layers": a.layers} if a.layers else {}))
    cfg = model.config
    model = get_peft_model(model, LoraConfig(r=64, lora_alpha=16, lora_dropout=0.1))
    V = cfg.vocab_size
    rng = random.Random(0)

    def run(name, make):
        ids, kw2, T = make()
        for _ in range(a.warmup):
            model(ids, labels=ids, **kw2)["loss"].backward()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            model(ids, labels=ids, **kw2)["loss"].backward()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.steps
        print(json.dumps({"cfg": name, "tokens": T, "ms": round(ms, 2), "ms_per_1k": round(ms * 1000 / T, 2)}),
              flush=True)

    for c in [x for x in a.cfgs.split(",") if x]:
        T = int(c)

        def make(T=T):
            lens, left = [], T
            while left > 1024:
                n = rng.randint(512, 1024)
                lens.append(n)
                left -= n
            lens.append(left)
            ids = torch.randint(0, V, (1, T), device=dev)
            return ids, {"varlen": Varlen(lens, dev)}, T
        run(f"varlen{T}", make)
    for c in [x for x in a.padded.split(",") if x]:
        R, S = (int(v) for v in c.split("x"))

        def make(R=R, S=S):
            return torch.randint(0, V, (R, S), device=dev), {}, R * S
        run(f"padded{c}", make)


if __name__ == "__main__":
    main()
