"""Memory planner vs the allocator's measured peak on an MI355X (parallel/planner.py): for the PEFT
paths the plan counts the K-concatenated W' (the frozen bf16 weight is a view of it), the cached
W^T of the TN dX GEMMs, the adapter-gradient B^T buffer and the h' tails, and must land within 5 %
of ``torch.cuda.max_memory_allocated`` of a real Llama-2-7B LoRA / QLoRA step (bench.py reports
both numbers in its JSON line)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("peft", ["lora", "qlora"])
def test_peft_plan_within_5pct_of_measured_peak(peft):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--peft", peft, "--steps", "1", "--warmup", "1"],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    plan, peak = d["hbm_plan_gib"], d["hbm_peak_gib"]
    assert abs(plan - peak) <= 0.05 * peak, (peft, plan, peak)
