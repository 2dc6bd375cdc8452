"""Memory preflight (parallel/planner.py) and the full 80-layer Llama-3-70B FSDP partition at world 8,
sized on a meta-device model (BASELINE config #5 readiness without an 8-GPU box)."""
import json
import os
import subprocess
import sys

import pytest

from gke_ray_train_amd.models import get_config
from gke_ray_train_amd.parallel.planner import GiB, plan_memory, preflight

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM = 288e9


def test_llama3_70b_partition_world8_on_meta():
    cfg = get_config("llama3-70b")
    plan = plan_memory(cfg, 8, "fsdp", offload=True, micro_batch=1, seq=1024, hbm_capacity=HBM, host_capacity=2e12)
    u = plan.units
    assert u["decoder_units"] == 80 and u["root_units"] == 1
    h, f, kv = 8192, 28672, 1024
    block = (h + 2 * kv) * h + h * h + 2 * f * h + h * f  # fused qkv, o, fused gate/up, down
    assert u["block_params"] == block == 855_638_016
    assert u["block_shard_params"] == block // 8  # 64-aligned already
    assert u["root_params"] == 2 * 128256 * h  # embed_tokens + lm_head
    assert u["replicated_params"] == 80 * 2 * h + h  # norm weights
    # one-ahead prefetch: the running block + the prefetched one + the root unit
    assert u["peak_gathered_bytes"] == (2 * block + 2 * 128256 * h) * 2
    # every parameter is in exactly one shard / the replicated set
    assert 80 * block + u["root_params"] + u["replicated_params"] == cfg.num_params()
    # offload moves the 8 B/param fp32 moments of the shard to pinned host memory
    assert abs(plan.host_per_rank["adam_moments_fp32"] - 8.0 * (80 * block + u["root_params"]) / 8) < 1e6
    assert plan.fits and plan.hbm_total < 100 * GiB


def test_70b_refusals_are_explicit():
    cfg = get_config("llama3-70b")
    one = plan_memory(cfg, 1, "fsdp", hbm_capacity=HBM, host_capacity=2e12)
    assert not one.fits and any(p.startswith("HBM") for p in one.problems())
    with pytest.raises(MemoryError, match="does not fit"):
        preflight(one)
    # 8 ranks x 66 GiB of pinned moments needs more host RAM than 256 GiB
    small_host = plan_memory(cfg, 8, "fsdp", offload=True, micro_batch=1, hbm_capacity=HBM, host_capacity=256 * GiB)
    assert any(p.startswith("host RAM") for p in small_host.problems())


def test_7b_headline_config_fits_and_zero_shrinks_optimizer():
    cfg = get_config("llama2-7b")
    one = plan_memory(cfg, 1, "ddp", micro_batch=8, seq=1024, hbm_capacity=HBM)
    eight = plan_memory(cfg, 8, "ddp", micro_batch=8, seq=1024, hbm_capacity=HBM)
    assert one.fits and eight.fits
    assert eight.hbm_per_rank["adam_moments_fp32"] * 8 == pytest.approx(one.hbm_per_rank["adam_moments_fp32"])
    qlora = plan_memory(get_config("llama3.1-8b"), 1, "ddp", peft="qlora", micro_batch=2, seq=1024, hbm_capacity=HBM)
    # NF4 codes are ~0.53 B / parameter; the bf16 W' (K-concat) and W^T layouts of the fast path
    # are counted separately (they are what the measured peak holds, profiles/r3s3_end_state.md)
    assert qlora.hbm_per_rank["frozen_nf4_codes"] < 5 * GiB
    assert qlora.hbm_per_rank["frozen_kcat_weight"] > 12 * GiB and qlora.hbm_per_rank["frozen_base_transposed"] > 12 * GiB
    lora = plan_memory(get_config("llama2-7b"), 1, "ddp", peft="lora", micro_batch=8, seq=1024, hbm_capacity=HBM)
    # bf16 LoRA: the base projection is held once as W' (its weight is a view) plus W^T
    assert "frozen_base" not in lora.hbm_per_rank and lora.fits
    nokcat = plan_memory(get_config("llama2-7b"), 1, "ddp", peft="lora", lora_r=16, micro_batch=8, seq=1024,
                         hbm_capacity=HBM)
    assert nokcat.hbm_per_rank["frozen_base"] > 11 * GiB and "frozen_kcat_weight" not in nokcat.hbm_per_rank


def test_qlora_70b_plan_follows_the_nf4_dequant_cache_rule(monkeypatch):
    """peft/quant.py set_dequant_cache "auto": the resident bf16 W / W^T (and the resident K-concat
    W') exist only when 4 B per base parameter fits in 15 % of HBM — on for 8B, off for 70B, where
    the plan holds the NF4 codes plus one projection's per-use dequantisation (a transient W') instead."""
    monkeypatch.delenv("GRT_NF4_CACHE", raising=False)
    big = plan_memory(get_config("llama3-70b"), 1, "ddp", peft="qlora", micro_batch=2, seq=1024, hbm_capacity=HBM)
    hb = big.hbm_per_rank
    for k in ("frozen_kcat_weight", "frozen_base_transposed", "frozen_base"):
        assert k not in hb
    assert hb["lora_bt"] < 2 * GiB  # the streamed W' path keeps only the adapters' B^T resident
    assert hb["frozen_nf4_codes"] < 40 * GiB and hb["nf4_dequant_scratch"] < 2 * GiB
    assert big.fits and big.hbm_total < 120 * GiB
    small = plan_memory(get_config("llama3.1-8b"), 1, "ddp", peft="qlora", micro_batch=2, seq=1024, hbm_capacity=HBM)
    assert "frozen_kcat_weight" in small.hbm_per_rank and "nf4_dequant_scratch" not in small.hbm_per_rank
    monkeypatch.setenv("GRT_NF4_CACHE", "0")  # forced off for 8B too
    off = plan_memory(get_config("llama3.1-8b"), 1, "ddp", peft="qlora", micro_batch=2, seq=1024, hbm_capacity=HBM)
    assert "frozen_kcat_weight" not in off.hbm_per_rank and off.hbm_total < small.hbm_total - 20 * GiB


def test_bench_plan_only_cli():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--plan-only", "--model", "llama2-7b",
                        "--device", "cpu"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])["memory_plan"]
    assert d["model"] == "llama2-7b" and d["fits"] is True


def test_proxy_host_ram_counts_one_rank_and_reports_the_node():
    """A one-process proxy of rank 0 (bench.py --proxy-world 8) holds rank 0's pinned moments only:
    the fit check counts one rank, while the plan still reports what the 8-rank node needs."""
    cfg = get_config("llama3-70b")
    plan = plan_memory(cfg, 8, "fsdp", offload=True, micro_batch=8, seq=1024, checkpointing=True,
                       hbm_capacity=HBM, host_capacity=200 * GiB)
    per_rank = plan.host_per_rank["adam_moments_fp32"]
    assert 60 * GiB < per_rank < 70 * GiB  # 8 B x 70.6e9 / 8
    assert not plan.fits and "across 8 ranks" in plan.problems()[0]  # the real node: 526 GiB > 200
    plan.host_ranks_here = 1
    assert plan.fits
    d = plan.to_dict()
    assert d["host_total_node_gib"] > 500 and d["host_fits_full_node"] is False
    assert abs(d["host_per_rank_gib"] - per_rank / GiB) < 0.01


def test_offload_prefetch_ring_sizing():
    from gke_ray_train_amd.parallel.offload import PREFETCH_CAP_BYTES, prefetch_slots_for
    chunk = 1 << 26  # 64 Mi elements: m + v = 512 MiB per slot
    assert prefetch_slots_for(PREFETCH_CAP_BYTES, chunk) == 128  # the 64 GiB automatic cap
    assert prefetch_slots_for(32 * (1 << 30), chunk) == 64
    assert prefetch_slots_for(511 * (1 << 20), chunk) == 0
    assert prefetch_slots_for(0, chunk) == 0


def test_bucket_plan_cost_model_and_calibration_file(tmp_path, monkeypatch):
    """Bucket size = argmin (G / b) alpha + b / beta = sqrt(G alpha beta), clamped; alpha / beta from
    a calibration file written by tools/rccl_calibrate.py (run here over gloo, 2 ranks)."""
    from gke_ray_train_amd.parallel.comm import comm_model, plan_bucket_bytes
    monkeypatch.delenv("GRT_BUCKET_MB", raising=False)
    monkeypatch.delenv("GRT_COMM_CALIBRATION", raising=False)
    G = 13_476_831_232  # Llama-2-7B bf16 gradient bytes
    m = comm_model("all_reduce", 8)
    assert m["source"] == "prior"
    b = plan_bucket_bytes(G, 8)
    assert abs(b - (G * m["alpha_us"] * 1e-6 * m["beta_GBps"] * 1e9) ** 0.5) <= 8 * 2 ** 20
    assert plan_bucket_bytes(G, 8, "reduce_scatter") > b  # reduce-scatter moves half the bytes
    assert plan_bucket_bytes(10 ** 6, 8) == 16 * 2 ** 20 and plan_bucket_bytes(10 ** 13, 8) == 2 ** 30
    assert plan_bucket_bytes(G, 1) == G
    out = tmp_path / "cal.json"
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 1000),
                        os.path.join(ROOT, "tools", "rccl_calibrate.py"), "--device", "cpu", "--out", str(out),
                        "--min-kib", "64", "--max-mib", "4", "--reps", "3"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    cal = json.loads(out.read_text())
    assert cal["world"] == 2 and cal["all_reduce"]["beta_GBps"] > 0 and cal["all_reduce"]["alpha_us"] >= 0
    monkeypatch.setenv("GRT_COMM_CALIBRATION", str(out))
    m2 = comm_model("all_reduce", 2)  # measured world: used as measured
    assert m2["source"] == str(out) and m2["beta_GBps"] == cal["all_reduce"]["beta_GBps"] and m2["world"] == 2
    # another world size: the measured bus bandwidth carries over, rescaled to algorithm bandwidth
    m8 = comm_model("all_reduce", 8)
    ring = (8 / (2 * 7)) / (2 / (2 * 1))
    assert m8["world"] == 2 and abs(m8["beta_GBps"] - cal["all_reduce"]["beta_GBps"] * ring) < 1e-9
    # a file holding several world sizes: the nearest one wins (per-world entries)
    cal8 = dict(cal["by_world"]["2"], world=8, all_reduce=dict(cal["all_reduce"], beta_GBps=123.0))
    multi = tmp_path / "multi.json"
    multi.write_text(json.dumps({"by_world": {"2": cal["by_world"]["2"], "8": cal8}}))
    monkeypatch.setenv("GRT_COMM_CALIBRATION", str(multi))
    assert comm_model("all_reduce", 8)["beta_GBps"] == 123.0 and comm_model("all_reduce", 7)["world"] == 8
    assert comm_model("all_reduce", 2)["beta_GBps"] == cal["all_reduce"]["beta_GBps"]
    monkeypatch.setenv("GRT_COMM_CALIBRATION", str(out))
    b2 = plan_bucket_bytes(G, 8)
    assert 16 * 2 ** 20 <= b2 <= 2 ** 30


def test_offload_resident_share_reserve_and_host_link(monkeypatch):
    """auto keeps every moment byte HBM can hold beside the configurable reserve; the link plan
    says whether the streamed rest fits under a step (config #5, Llama-3-70B at 8 ranks)."""
    from gke_ray_train_amd.parallel.offload import host_link_plan, resident_fraction_from_plan
    cfg = get_config("llama3-70b")
    plan = plan_memory(cfg, 8, "fsdp", offload=True, micro_batch=8, seq=1024, checkpointing=True,
                       hbm_capacity=HBM, host_capacity=2000 * GiB)
    moved = plan.host_per_rank["adam_moments_fp32"]
    monkeypatch.delenv("GRT_OFFLOAD_HBM_RESERVE_GIB", raising=False)
    assert resident_fraction_from_plan(plan) == 1.0  # 288 GB holds all of rank 0's moments
    free = plan.hbm_capacity - plan.hbm_total
    # a reserve that leaves room for only half of the moments -> auto streams the other half
    monkeypatch.setenv("GRT_OFFLOAD_HBM_RESERVE_GIB", str((free - 0.5 * moved) / GiB))
    f = resident_fraction_from_plan(plan)
    assert abs(f - 0.5) < 1e-6
    lp = host_link_plan(plan, f, step_s=3.5, link_GBps=57.0)
    assert abs(lp["streamed_gib_per_direction"] - 0.5 * moved / GiB) < 0.01
    assert lp["link_bound"] is False and lp["link_s"] < 3.5
    slow = host_link_plan(plan, 0.0, step_s=1.0, link_GBps=57.0)  # everything streamed, short step
    assert slow["link_bound"] is True and 0.0 < slow["resident_fraction_for_link"] < 1.0
    # at that resident share the streamed bytes take exactly one step
    edge = host_link_plan(plan, slow["resident_fraction_for_link"], step_s=1.0, link_GBps=57.0)
    assert abs(edge["link_s"] - 1.0) < 0.01
