#!/usr/bin/env python3
"""Diagnostic only (never a benchmark number): the headline step with the overlapped AdamW's kernels
removed, to price the optimizer's interference with the forward (its HBM traffic / CU slots beside
the forward kernels) against the same step with the update. Runs bench.py's main() with
OverlappedOptimizer.step replaced by a no-op that keeps the hooks and bookkeeping.
usage: python tools/no_update_probe.py --steps 20 --warmup 5"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gke_ray_train_amd.parallel import overlap  # noqa: E402


def _no_update(self, grad_scale=None):
    overlap.bump_param_generation()
    self.opt._opt_called = True


overlap.OverlappedOptimizer.step = _no_update

import bench  # noqa: E402

if __name__ == "__main__":
    sys.argv[0] = "bench.py"
    bench.main()
