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


def lds_dump(K=256):
    """variant 13: the kernel dumps LDS buffer 0 after the prologue; decode it against A / B."""
    C = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(2)
    M = N = 256
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev).to(torch.bfloat16)
    out = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
    C.gemm_nt(A, B, out, False, 13)
    torch.cuda.synchronize()
    raw = out.view(-1).view(torch.int16).cpu()  # bytes as bf16 bit patterns
    CH, TEN = 1040, 32 * 1040
    for name, X, base in (("A", A.cpu(), 0), ("B", B.cpu(), TEN)):
        xb = X.view(torch.int16)
        ok = tot = 0
        firstbad = None
        for c in range(32):
            for b in range(8):
                row = 128 * (c >> 4) + 16 * b + (c & 15)
                off = (base + c * CH + b * 128) // 2
                got = raw[off:off + 64]
                exp = xb[row, 0:64]
                tot += 1
                if torch.equal(got, exp):
                    ok += 1
                elif firstbad is None:
                    firstbad = (c, b, row, got[:4].tolist(), exp[:4].tolist(), bool((got == 0).all()))
        print(f"{name}: {ok}/{tot} image rows match; first bad (chunk, b, row, got, exp, all-zero) = {firstbad}", flush=True)
        # where did the expected rows land? search row 0's first 8 values anywhere in the dump
        key = xb[0, 0:8]
        hits = [i for i in range(0, raw.numel() - 8) if torch.equal(raw[i:i + 8], key)]
        print(f"  {name} row 0 k0..7 found at element offsets {hits[:5]} (expected {(base) // 2})", flush=True)


if __name__ == "__main__" and os.environ.get("GRT_DIAG_LDS"):
    lds_dump()


def first_slab(variant=14, K=256):
    """variant 14 computes only the prologue's tile-0 kk0 half: compare with A[:, :32] B[:, :32]^T."""
    C = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    A = torch.randn(256, K, device=dev).to(torch.bfloat16)
    B = torch.randn(256, K, device=dev).to(torch.bfloat16)
    out = torch.zeros(256, 256, device=dev, dtype=torch.bfloat16)
    C.gemm_nt(A, B, out, False, variant)
    torch.cuda.synchronize()
    for nm, ref in (("slab0", A[:, :32].float() @ B[:, :32].float().t()), ("zero", torch.zeros(256, 256, device=dev))):
        rel = float(((out.float() - ref).norm() / max(float(ref.norm()), 1e-9)).item())
        print(f"variant {variant} vs {nm}: rel={rel:.3e} |out|={float(out.float().norm()):.3e}", flush=True)


if __name__ == "__main__" and os.environ.get("GRT_DIAG_FIRST"):
    first_slab(14)
    for v in (15, 9):
        print(f"--- variant {v}")
        per_tile(variant=v, K=256)


def frag_dump(K=128):
    C = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(4)
    A = torch.randn(256, K, device=dev).to(torch.bfloat16)
    B = torch.randn(256, K, device=dev).to(torch.bfloat16)
    out = torch.zeros(256, 256, device=dev, dtype=torch.bfloat16)
    C.gemm_nt(A, B, out, False, 16)
    torch.cuda.synchronize()
    raw = out.view(-1).cpu()
    af = raw[:512].view(64, 8).float()
    bf = raw[512:1024].view(64, 8).float()
    z = out.view(-1).view(torch.float32)[512:512 + 256].cpu().view(64, 4)
    Ac, Bc = A.cpu().float(), B.cpu().float()
    ea = torch.stack([Ac[l & 15, 8 * (l >> 4):8 * (l >> 4) + 8] for l in range(64)])
    eb = torch.stack([Bc[l & 15, 8 * (l >> 4):8 * (l >> 4) + 8] for l in range(64)])
    print("a0[0] matches:", bool(torch.equal(af, ea)), "b0[0] matches:", bool(torch.equal(bf, eb)), flush=True)
    if not torch.equal(af, ea):
        print(" lane0 got", af[0].tolist(), "exp", ea[0].tolist())
    ref = Bc[:16, :32] @ Ac[:16, :32].t()  # D[n][m] for block (0,0)
    ez = torch.stack([torch.tensor([ref[4 * (l >> 4) + e, l & 15] for e in range(4)]) for l in range(64)])
    print("mfma(b0,a0) matches D[n][m]:", float((z - ez).abs().max()), "max|D|", float(ez.abs().max()), flush=True)


if __name__ == "__main__" and os.environ.get("GRT_DIAG_FRAG"):
    frag_dump()


def acc_dump():
    C = _native.kernels()
    dev = torch.device("cuda", 0)
    for variant in (17, 18):
        for K in (128, 256, 512):
            torch.manual_seed(5)
            A = torch.randn(256, K, device=dev).to(torch.bfloat16)
            B = torch.randn(256, K, device=dev).to(torch.bfloat16)
            out = torch.zeros(256, 256, device=dev, dtype=torch.bfloat16)
            C.gemm_nt(A, B, out, False, variant)
            torch.cuda.synchronize()
            z = out.view(-1).view(torch.float32)[:512].cpu().view(2, 64, 4)
            Ac, Bc = A.cpu().float(), B.cpu().float()
            for bi, (r0, c0) in enumerate(((0, 0), (112, 112))):
                parts = {}
                for lo, hi in ((0, K), (0, 128), (128, K)):
                    if hi <= lo:
                        continue
                    ref = Bc[c0:c0 + 16, lo:hi] @ Ac[r0:r0 + 16, lo:hi].t()
                    ez = torch.stack([torch.tensor([ref[4 * (l >> 4) + e, l & 15] for e in range(4)]) for l in range(64)])
                    parts[f"k{lo}-{hi}"] = round(float((z[bi] - ez).abs().max() / ez.abs().max()), 4)
                print(f"variant {variant} K={K} block{bi}: rel err vs {parts}", flush=True)


if __name__ == "__main__" and os.environ.get("GRT_DIAG_ACC"):
    acc_dump()
