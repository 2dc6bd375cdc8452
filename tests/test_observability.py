"""Observability: StepMeter records (throughput, MFU, phase breakdown) to JSONL/CSV, HF-style summary,
Prometheus exposition, ROCTX no-op safety, rocprofv3 command recipe."""
import json
import time

import torch

from gke_ray_train_amd.observability import PrometheusExporter, StepMeter, roctx, rocprof_command


def test_step_meter_jsonl_csv(tmp_path):
    prom = PrometheusExporter(start_server=False)
    m = StepMeter(tokens_per_step=1000, flops_per_token=1e9, n_gpus=2, samples_per_step=4,
                  jsonl=str(tmp_path / "m.jsonl"), csv_path=str(tmp_path / "m.csv"), device="cpu", prometheus=prom,
                  peak_flops=1e12)
    with m.phase("warmup_only"):
        pass
    for i in range(3):
        with m.step(i):
            with m.phase("forward"):
                time.sleep(0.01)
            with m.phase("backward"):
                time.sleep(0.02)
        rec = m.log(i, loss=torch.tensor(2.5), lr=1e-4)
    assert "warmup_only_ms" not in rec
    assert rec["forward_ms"] >= 9 and rec["backward_ms"] >= 19
    assert rec["step_ms"] >= rec["forward_ms"] + rec["backward_ms"] - 1
    assert abs(rec["tokens_per_sec"] - 1000 / (rec["step_ms"] / 1000)) < 1.0
    assert abs(rec["mfu"] - rec["tokens_per_sec"] / 2 * 1e9 / 1e12) < 1e-3
    lines = [json.loads(x) for x in open(tmp_path / "m.jsonl")]
    assert [x["step"] for x in lines] == [0, 1, 2] and lines[0]["loss"] == 2.5
    assert open(tmp_path / "m.csv").read().splitlines()[0].startswith("step,")
    s = m.summary()
    assert s["train_tokens_per_second"] > 0 and s["total_flos"] == 3000 * 1e9 and "train_samples_per_second" in s
    assert "grt_train_tokens_per_sec" in prom.text()


def test_log_every_and_roctx_safe():
    m = StepMeter(tokens_per_step=10, device="cpu", log_every=2)
    with m.step(1):
        with roctx.range("x"):
            roctx.mark("m")
    assert m.log(1) is None
    with m.step(2):
        pass
    assert m.log(2)["step"] == 2


def test_rocprof_recipe():
    c = rocprof_command(["python3", "bench.py", "--steps", "3"], out_dir="gpurun_out/p")
    assert c.startswith("rocprofv3 --kernel-trace --stats") and c.endswith("-- python3 bench.py --steps 3")
    c = rocprof_command(["python3", "x.py"], pmc=["SQ_INSTS_VALU_MFMA_MOPS_BF16"], markers=True)
    assert "--pmc" in c and "--marker-trace" not in c and "--stats" not in c
