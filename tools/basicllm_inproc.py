#!/usr/bin/env python3
"""Run the BasicLLM job's ``train_loop_per_worker`` (jobs/pytorch_llm_ray.py, reference job #1) in
THIS process as one local worker, for profilers that only see the launched process:

    rocprofv3 --kernel-trace --stats -- python3 tools/basicllm_inproc.py --max-windows 3200

Same arguments as the job (``--preset``, ``--batch``, ``--seq``, ``--dtype``, ``--max-windows``).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "jobs"))

import pytorch_llm_ray as job  # noqa: E402


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="reference", choices=sorted(job.PRESETS))
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--pvc", default=job.PVC)
    ap.add_argument("--name", default="basicllm_inproc")
    ap.add_argument("--data-scale", type=float, default=1.0)
    ap.add_argument("--max-windows", type=int, default=None)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    a = ap.parse_args(argv)
    for k, v in (("RANK", "0"), ("LOCAL_RANK", "0"), ("WORLD_SIZE", "1")):
        os.environ.setdefault(k, v)
    job.train_loop_per_worker(job.build_config(a))


if __name__ == "__main__":
    main()
