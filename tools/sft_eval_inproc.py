#!/usr/bin/env python3
"""The reference SFT job's evaluation pass alone, in THIS process (for ``rocprofv3 --kernel-trace``):
the job's worker loop with ``SFTTrainer.train`` replaced by ``--evals`` calls of ``evaluate()``
(the 200-sample eval set of the unchanged fine_tune_config.json), each timed.

    python3 tools/sft_eval_inproc.py [--evals 3] [--set KEY=VALUE ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "jobs"))

import fine_tune_llama_ray as job  # noqa: E402
from gke_ray_train_amd.trainer import sft  # noqa: E402
from gke_ray_train_amd.utils.config import parse_overrides  # noqa: E402


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=None)
    ap.add_argument("--evals", type=int, default=3)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    a = ap.parse_args(argv)
    for k, v in (("RANK", "0"), ("LOCAL_RANK", "0"), ("WORLD_SIZE", "1")):
        os.environ.setdefault(k, v)

    def evals_only(self, resume_from_checkpoint=None):
        times = []
        for _ in range(a.evals):
            t = time.time()
            m = self.evaluate()
            times.append(round(time.time() - t, 4))
        print(f"eval wall s: {times} last: {m}", flush=True)
        return sft.TrainOutput(0, 0.0, {"eval_wall_s": times})

    sft.SFTTrainer.train = evals_only
    cfg = job.load_config(a.config, parse_overrides(a.set))
    job.train_loop_per_worker(cfg)


if __name__ == "__main__":
    main()
