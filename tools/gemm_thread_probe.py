"""Does TunableOp apply to dX GEMMs (dy @ w) in the main thread, a plain Python thread, a thread
that re-enables TunableOp, and the autograd engine's backward thread? Markers between variants."""
import os
import sys
import threading

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gke_ray_train_amd.ops import gemm_tuning  # noqa: E402

print("tuned:", gemm_tuning.enable_tuned_gemms(), flush=True)
mark = torch.zeros(1, device="cuda")
M, K, N = 8192, 4096, 12288
dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)


def sep(tag):
    torch.cuda.synchronize()
    mark.fill_(1.0)
    torch.cuda.synchronize()
    print("variant", tag, torch.cuda.tunable.is_enabled(), flush=True)


sep("main")
for _ in range(2):
    dy @ w
sep("thread")
t = threading.Thread(target=lambda: [dy @ w for _ in range(2)])
t.start(); t.join()
sep("thread+ensure")


def f():
    gemm_tuning._tls.done = False
    gemm_tuning.ensure_thread()
    print("in thread enabled:", torch.cuda.tunable.is_enabled(), flush=True)
    for _ in range(2):
        dy @ w
t = threading.Thread(target=f)
t.start(); t.join()
sep("autograd")


class Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        print("bwd thread enabled:", torch.cuda.tunable.is_enabled(), threading.current_thread().name, flush=True)
        gemm_tuning.ensure_thread()
        print("bwd thread enabled after:", torch.cuda.tunable.is_enabled(), flush=True)
        for _ in range(2):
            dy @ w
        return g


x = torch.randn(4, device="cuda", requires_grad=True)
Fn.apply(x).sum().backward()
sep("end")
