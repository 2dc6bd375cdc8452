"""Where is a hand-written GEMM variant wrong? Runs ``gemm_nt`` variant V on a few shapes against an
fp32 reference and prints, per shape: relative error, whether two launches agree bit for bit (a
race shows up as run-to-run differences), and the bad-element fraction folded onto the 256 x 256
output tile (by 16-row / 16-column block) and by output tile.

    python tools/gemm_diag.py --variant 9
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gke_ray_train_amd import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=9)
    ap.add_argument("--shapes", default="256x256x128,256x256x256,256x256x4096,512x512x1024,2048x2048x4096,8192x12288x4096")
    a = ap.parse_args()
    C = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for sh in a.shapes.split(","):
        M, N, K = (int(x) for x in sh.split("x"))
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        B = torch.randn(N, K, device=dev).to(torch.bfloat16)
        ref = A.float() @ B.float().t()
        outs = []
        for _ in range(2):
            out = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
            assert C.gemm_nt(A, B, out, False, a.variant), "unsupported"
            torch.cuda.synchronize()
            outs.append(out)
        same = bool(torch.equal(outs[0], outs[1]))
        out = outs[0].float()
        err = (out - ref).abs()
        bad = (err > (ref.abs() * 2 ** -6 + 0.05)) | torch.isnan(out)
        rel = float(((out - ref).nan_to_num(1e9).norm() / ref.norm()).item())
        print(f"{sh}: rel={rel:.3e} bad={float(bad.float().mean()):.4f} runs_identical={same}", flush=True)
        if bad.any():
            b = bad.view(M // 256, 16, 16, N // 256, 16, 16).float()
            rb = b.mean(dim=(0, 2, 3, 4, 5))  # by 16-row block within the tile
            cb = b.mean(dim=(0, 1, 2, 3, 5))  # by 16-col block within the tile
            r16 = b.mean(dim=(0, 1, 3, 4, 5))  # by row within a 16-row block
            c16 = b.mean(dim=(0, 1, 2, 3, 4))
            tile = b.mean(dim=(1, 2, 4, 5))
            print("  row-blocks:", " ".join(f"{x:.2f}" for x in rb.tolist()))
            print("  col-blocks:", " ".join(f"{x:.2f}" for x in cb.tolist()))
            print("  row%16    :", " ".join(f"{x:.2f}" for x in r16.tolist()))
            print("  col%16    :", " ".join(f"{x:.2f}" for x in c16.tolist()))
            print(f"  tiles bad: {int((tile > 0).sum())}/{tile.numel()}, max tile frac {float(tile.max()):.3f}")
            # error magnitude relative to |ref| on the bad elements: one K-tile missing ~ 1/sqrt(T)
            print(f"  mean |err|/rms(ref) on bad: {float(err[bad].mean() / ref.pow(2).mean().sqrt()):.3f}")


if __name__ == "__main__" and not os.environ.get("GRT_DIAG_TILES"):
    main()


def per_tile(variant=9, M=256, N=256, K=512):
    """Which 32-deep K slab is wrong: A is zero outside one slab at a time."""
    C = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev).to(torch.bfloat16)
    for s in range(K // 32):
        As = torch.zeros_like(A)
        As[:, 32 * s:32 * s + 32] = A[:, 32 * s:32 * s + 32]
        ref = As.float() @ B.float().t()
        out = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
        C.gemm_nt(As, B, out, False, variant)
        torch.cuda.synchronize()
        rel = float(((out.float() - ref).norm() / ref.norm()).item())
        # does the kernel's output match another slab's product instead?
        alt = []
        for s2 in range(K // 32):
            Bs = torch.zeros_like(B)
            Bs[:, 32 * s:32 * s + 32] = B[:, 32 * s2:32 * s2 + 32]
            r2 = As.float() @ Bs.float().t()
            alt.append(float(((out.float() - r2).norm() / r2.norm()).item()))
        best = min(range(len(alt)), key=lambda i: alt[i])
        print(f"slab {s} (tile {s // 2} kk{s % 2}): rel={rel:.3e}  best-matching B slab {best} rel={alt[best]:.3e}", flush=True)


if __name__ == "__main__" and os.environ.get("GRT_DIAG_TILES"):
    for v in os.environ["GRT_DIAG_TILES"].split(","):
        print(f"--- variant {v}")
        per_tile(variant=int(v), K=256)
