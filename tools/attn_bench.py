"""Attention kernel timing on MI355X: flash kernels (bf16 / exact fp32) vs the fp32 math path.
Shapes: BasicLLM (B16 S256 H16 D128, fp32 — reference pytorch_llm_ray.py:324-344) and Llama-2-7B
(B8 S1024 H32 D128, bf16). Prints one JSON line per case (fwd ms, fwd+bwd ms, TFLOP/s)."""
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd import ops  # noqa: E402
from gke_ray_train_amd.ops import _ref  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def case(name, B, S, H, D, dtype, p, impl):
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=dtype, requires_grad=True) for _ in range(3))
    do = torch.randn(B, S, H, D, device="cuda", dtype=dtype)
    f = (lambda: ops.flash_attention(q, k, v, causal=True, dropout_p=p, seed=1)) if impl == "kernel" else \
        (lambda: _ref.attention(q, k, v, causal=True, dropout_p=p, seed=1))
    tf = timeit(lambda: f())

    def fb():
        o = f()
        torch.autograd.backward(o, do)
    tfb = timeit(fb)
    flop_f = 4 * B * H * S * S * D / 2  # causal
    print(json.dumps({"case": name, "impl": impl, "dtype": str(dtype), "dropout": p, "fwd_ms": round(tf, 4),
                      "fwd_bwd_ms": round(tfb, 4), "fwd_tflops": round(flop_f / tf / 1e9, 1),
                      "fwd_bwd_tflops": round(3.5 * flop_f / tfb / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    for impl in ("kernel", "math"):
        case("basicllm", 16, 256, 16, 128, torch.float32, 0.1, impl)
    case("basicllm_nodrop", 16, 256, 16, 128, torch.float32, 0.0, "kernel")
    case("llama2-7b", 8, 1024, 32, 128, torch.bfloat16, 0.0, "kernel")
