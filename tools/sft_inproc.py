#!/usr/bin/env python3
"""Run the SFT job's ``train_loop_per_worker`` in THIS process (one worker, no TorchTrainer pool).

For profilers that only see the launched process (``rocprofv3 --kernel-trace --stats -- python3
tools/sft_inproc.py --set NUM_TRAIN_SAMPLES=320``): the job's worker pool runs the loop in spawned
children that the pool terminates at shutdown, before the profiler's finalisation can flush.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "jobs"))

import fine_tune_llama_ray as job  # noqa: E402
from gke_ray_train_amd.utils.config import parse_overrides  # noqa: E402


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=None)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    a = ap.parse_args(argv)
    for k, v in (("RANK", "0"), ("LOCAL_RANK", "0"), ("WORLD_SIZE", "1")):
        os.environ.setdefault(k, v)
    cfg = job.load_config(a.config, parse_overrides(a.set))
    job.train_loop_per_worker(cfg)


if __name__ == "__main__":
    main()
