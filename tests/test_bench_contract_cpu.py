"""bench.py contract at N>1 (the driver's launch line, one rank per device) rehearsed on 2 gloo CPU
ranks with a tiny Llama: exactly one JSON line from rank 0 with the BASELINE metric, whole-job
value, n_gpus, steps/warmup echo and the dp2 (+ZeRO) parallelism string."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_cpu(tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--model", "llama-tiny-gqa", "--device", "cpu",
           "--seq", "64", "--batch", "2"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert out["metric"] == base.get("metric", out["metric"])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["higher_is_better"] is True
    assert out["config"]["parallelism"].startswith("dp2")
    assert out["config"]["global_batch"] == 4
    # whole-job aggregate: tokens/s = global tokens per step / step time
    assert abs(out["value"] - 4 * 64 / (out["ms_per_step"] / 1e3)) / out["value"] < 0.02


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(lines) == 1, stdout[-3000:]
    return json.loads(lines[0])


def test_bench_gpus_flag_spawns_trainer_workers(tmp_path):
    """Plain ``python bench.py --gpus 2`` (no torchrun): the parent starts 2 ranks through the
    framework's TorchTrainer and relays rank 0's single JSON line."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--model", "llama-tiny-gqa", "--device", "cpu", "--seq", "64", "--batch", "2"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    out = _json_line(r.stdout)
    assert out["n_gpus"] == 2 and out["pg_world_size"] == 2 and out["pg_backend"] == "gloo"
    assert out["config"]["parallelism"] == "dp2+zero1"
    assert out["launcher"].startswith("TorchTrainer")
    assert out["config"]["global_batch"] == 4


def test_bench_one_gpu_stays_in_process(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1",
           "--model", "llama-tiny-gqa", "--device", "cpu", "--seq", "64", "--batch", "2"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    out = _json_line(r.stdout)
    assert out["n_gpus"] == 1 and out["launcher"] == "in-process" and out["config"]["parallelism"] == "dp1"


def test_bench_world_size_mismatch_is_an_error(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--model", "llama-tiny-gqa", "--device", "cpu"]
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=300)
    assert r.returncode == 2, r.stdout[-2000:]
    assert "refusing" in r.stdout
