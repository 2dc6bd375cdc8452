#!/usr/bin/env python3
"""Wikitext-2-raw preparation as a runtime task (reference: ray-jobs/prepare_wikitext2_ray_job.py).

Writes ``wiki.{train,valid,test}.tokens`` under ``<pvc>/datasets/wikitext-2-raw``; idempotent (skips
when all three files exist and are non-empty). With no network on this machine the corpus is the
deterministic synthetic Wikitext-2 of ``gke_ray_train_amd.data.wikitext`` at the real split sizes.
Unlike the reference (which prints the error and exits 0, :111-113) a failure or timeout here exits
non-zero.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gke_ray_train_amd import runtime as rt  # noqa: E402

PVC = os.environ.get("GRT_PVC") or os.environ.get("GRT_STORAGE_PATH") or os.path.abspath("pvc")


@rt.remote(num_cpus=1)
def prepare_wikitext2(target_dir: str, scale: float = 1.0, seed: int = 0):
    from gke_ray_train_amd.data import wikitext
    t0 = time.time()
    paths = wikitext.prepare(target_dir, seed=seed, scale=scale)
    sizes = {k: os.path.getsize(p) / 2 ** 20 for k, p in paths.items()}
    return {"paths": paths, "size_mb": sizes, "seconds": time.time() - t0}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--target", default=os.path.join(PVC, "datasets", "wikitext-2-raw"))
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the real split sizes")
    ap.add_argument("--timeout", type=float, default=1800)
    a = ap.parse_args(argv)
    if not rt.is_initialized():
        rt.init(address="auto", ignore_reinit_error=True)
    ref = prepare_wikitext2.remote(a.target, a.scale)
    try:
        out = rt.get(ref, timeout=a.timeout)
    except Exception as e:
        print(f"data preparation failed: {type(e).__name__}: {e}", flush=True)
        return 1
    for split, mb in out["size_mb"].items():
        print(f"{split:>10}: {out['paths'][split]} ({mb:.2f} MB)")
    print(f"done in {out['seconds']:.1f}s")
    return 0


if __name__ == "__main__":
    sys.exit(main())
