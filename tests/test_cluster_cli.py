"""Node-local cluster bring-up + Ray-Jobs-style submission (replaces the reference's GKE/KubeRay
setup scripts and ``ray job submit``): spec templating/validation, head daemon lifecycle, job
success / failure / stop, runtime_env working_dir + env_vars, logs, and a driver inside a job
attaching with ``ray.init(address='auto')`` through the ``ray`` shim."""
import json
import os
import socket
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_spec_envsubst_and_validate(tmp_path):
    from gke_ray_train_amd.cluster.spec import ClusterSpec, envsubst
    assert envsubst("a ${X:-7} $Y ${Z}", {"Y": "y"}) == "a 7 y "
    spec = ClusterSpec.load(os.path.join(ROOT, "deploy", "mi355x", "cluster.yaml"),
                            env={"NUM_GPUS_PER_NODE": "4", "DASHBOARD_PORT": "9999"})
    assert spec.workers.num_gpus_per_node == 4 and spec.head.dashboard_port == 9999
    assert spec.workers.env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert spec.head.num_cpus == 0
    with pytest.raises(ValueError):
        spec.validate(available_gpus=2)
    with pytest.raises(ValueError):
        ClusterSpec.from_dict({"nodes": 3})


def _grt(args, env, timeout=120):
    return subprocess.run([sys.executable, "-m", "gke_ray_train_amd.cli"] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_head_job_lifecycle(tmp_path):
    env = dict(os.environ, GRT_TMPDIR=str(tmp_path / "grt"), GRT_NUM_GPUS="0", PYTHONPATH=ROOT)
    port = _free_port()
    r = _grt(["start", "--head", "--port", str(port), "--num-gpus", "0", "--storage", str(tmp_path / "store")], env)
    assert r.returncode == 0, r.stderr + r.stdout
    addr = f"http://127.0.0.1:{port}"
    try:
        wd = tmp_path / "wd"
        wd.mkdir()
        (wd / "hello.py").write_text(textwrap.dedent("""
            import os, sys
            import ray

            @ray.remote(num_cpus=1)
            def sq(x):
                return x * x

            if __name__ == "__main__":
                ray.init(address="auto")
                print("GREETING", os.environ["GREETING"], sum(ray.get([sq.remote(i) for i in range(4)])))
                print("STORAGE", os.environ["GRT_STORAGE_PATH"])
                ray.shutdown()
        """))
        renv = json.dumps({"working_dir": str(wd), "env_vars": {"GREETING": "hi"}, "pip": ["surely-not-a-pkg==1.0"]})
        r = _grt(["job", "submit", "--address", addr, "--submission-id", "ok1", "--runtime-env-json", renv, "--",
                  "python", "hello.py"], env, timeout=180)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "GREETING hi 14" in r.stdout
        assert "surely-not-a-pkg" in r.stdout  # offline pip requirement reported, not fatal
        assert f"STORAGE {tmp_path / 'store'}" in r.stdout

        from gke_ray_train_amd.cluster.jobs import JobStatus, JobSubmissionClient
        c = JobSubmissionClient(addr)
        assert c.get_job_status("ok1") == JobStatus.SUCCEEDED
        bad = c.submit_job(entrypoint="python -c 'import sys; print(\"boom\"); sys.exit(3)'")
        assert c.wait(bad, timeout=60) == JobStatus.FAILED
        assert c.get_job_info(bad)["driver_exit_code"] == 3 and "boom" in c.get_job_logs(bad)
        long = c.submit_job(entrypoint="sleep 120", submission_id="sleeper")
        t0 = time.time()
        while c.get_job_status(long) != JobStatus.RUNNING and time.time() - t0 < 30:
            time.sleep(0.1)
        assert c.stop_job(long)
        assert c.wait(long, timeout=30) == JobStatus.STOPPED
        ids = {j["submission_id"] for j in c.list_jobs()}
        assert {"ok1", bad, "sleeper"} <= ids
        assert c.delete_job("ok1") and "ok1" not in {j["submission_id"] for j in c.list_jobs()}
        r = _grt(["status"], env)
        assert r.returncode == 0 and '"GPU": 0' in r.stdout
    finally:
        r = _grt(["stop"], env)
    assert "stopped" in r.stdout
    assert not os.path.exists(tmp_path / "grt" / "grt_current_cluster")
