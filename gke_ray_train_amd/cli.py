"""``grt`` command line: node-local cluster bring-up and Ray-Jobs-style submission.

Replaces the reference's GKE / KubeRay / ``ray`` CLI flow (reference a3-mega/gke-ray-cluster-setup.sh:1-91):

    grt cluster up -f deploy/mi355x/cluster.yaml     # ~ gcloud cluster create + kubectl apply RayCluster
    grt start --head [--num-gpus 8] [--port 8265]     # ~ ray start --head
    grt job submit --address http://localhost:8265 --runtime-env-json '{"working_dir": ".", ...}' \
        -- python jobs/fine_tune_llama_ray.py       # ~ ray job submit
    grt job status|logs|stop|list|delete
    grt status / grt stop / grt cluster down

``python -m gke_ray_train_amd.cli`` is the same program (``bin/grt`` and ``bin/ray`` wrap it).
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys
import time

from .cluster.head import current_cluster_file, grt_tmpdir, read_current_cluster
from .cluster.jobs import JobStatus, JobSubmissionClient
from .cluster.spec import ClusterSpec


def _count_gpus() -> int:
    env = os.environ.get("GRT_NUM_GPUS")
    if env is not None:
        return int(env)
    try:
        import torch
        return torch.cuda.device_count()  # does not initialise HIP on this image
    except Exception:
        return 0


def start_head(spec: ClusterSpec, wait: float = 60.0, block: bool = False) -> dict:
    cur = read_current_cluster()
    if cur is not None:
        raise SystemExit(f"a grt head is already running at {cur['address']} (pid {cur['pid']}); `grt stop` first")
    spec.validate(_count_gpus() if spec.workers.num_gpus_per_node else None)
    session = os.path.join(grt_tmpdir(), f"session_{time.strftime('%Y-%m-%d_%H-%M-%S')}_{os.getpid()}")
    os.makedirs(session, exist_ok=True)
    cmd = [sys.executable, "-m", "gke_ray_train_amd.cluster.head", "--spec-json", json.dumps(spec.to_dict()),
           "--session-dir", session]
    env = dict(os.environ)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = os.pathsep.join([root] + [p for p in env.get("PYTHONPATH", "").split(os.pathsep) if p])
    if block:
        return {"rc": subprocess.call(cmd, env=env)}
    with open(os.path.join(session, "head.log"), "w") as log:
        proc = subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    t0 = time.time()
    while time.time() - t0 < wait:
        cur = read_current_cluster()
        if cur is not None and cur.get("pid") == proc.pid:
            return cur
        if proc.poll() is not None:
            raise SystemExit(f"head exited with {proc.returncode}; see {session}/head.log")
        time.sleep(0.1)
    raise SystemExit(f"head did not come up within {wait}s; see {session}/head.log")


def stop_head(address=None, timeout: float = 30.0) -> bool:
    cur = read_current_cluster()
    try:
        c = JobSubmissionClient(address)
    except Exception:
        return False
    c.shutdown_cluster()
    t0 = time.time()
    while time.time() - t0 < timeout:
        if read_current_cluster() is None or (cur and not _alive(cur["pid"])):
            return True
        time.sleep(0.1)
    return False


def _alive(pid) -> bool:
    try:
        os.kill(int(pid), 0)
        return True
    except OSError:
        return False


def _spec_from_args(a) -> ClusterSpec:
    spec = ClusterSpec.load(a.file) if getattr(a, "file", None) else ClusterSpec()
    if getattr(a, "num_gpus", None) is not None:
        spec.workers.num_gpus_per_node = a.num_gpus
    elif not getattr(a, "file", None):
        spec.workers.num_gpus_per_node = _count_gpus()
    if getattr(a, "port", None) is not None:
        spec.head.dashboard_port = a.port
    if getattr(a, "dashboard_host", None):
        spec.head.dashboard_host = a.dashboard_host
    if getattr(a, "storage", None):
        spec.storage.path = a.storage
    return spec


def cmd_job_submit(a) -> int:
    entry = a.entrypoint
    if entry and entry[0] == "--":
        entry = entry[1:]
    if not entry:
        print("grt job submit: missing entrypoint (put it after `--`)", file=sys.stderr)
        return 2
    renv = json.loads(a.runtime_env_json) if a.runtime_env_json else {}
    if a.runtime_env:
        import yaml
        with open(a.runtime_env) as f:
            renv.update(yaml.safe_load(f) or {})
    if a.working_dir:
        renv["working_dir"] = a.working_dir
    if renv.get("working_dir"):
        renv["working_dir"] = os.path.abspath(renv["working_dir"])
    c = JobSubmissionClient(a.address)
    sid = c.submit_job(entrypoint=" ".join(shlex.quote(x) for x in entry) if len(entry) > 1 else entry[0],
                       runtime_env=renv, submission_id=a.submission_id,
                       metadata=json.loads(a.metadata_json) if a.metadata_json else None,
                       entrypoint_num_gpus=a.entrypoint_num_gpus or 0)
    print(f"Job '{sid}' submitted successfully", flush=True)
    if a.no_wait:
        return 0
    for chunk in c.tail_job_logs(sid):
        sys.stdout.write(chunk)
        sys.stdout.flush()
    st = c.get_job_status(sid)
    print(f"Job '{sid}' {st.value.lower()}", flush=True)
    return 0 if st == JobStatus.SUCCEEDED else 1


def build_parser():
    ap = argparse.ArgumentParser(prog="grt", description="MI355X node-local cluster + job CLI")
    sub = ap.add_subparsers(dest="cmd", required=True)

    s = sub.add_parser("start", help="start the head daemon (ray start --head)")
    s.add_argument("--head", action="store_true")
    s.add_argument("--num-gpus", type=int)
    s.add_argument("--port", "--dashboard-port", dest="port", type=int)
    s.add_argument("--dashboard-host")
    s.add_argument("--storage")
    s.add_argument("--block", action="store_true")
    s.add_argument("-f", "--file", help="cluster spec YAML")

    s = sub.add_parser("stop", help="stop the head daemon and its jobs")
    s.add_argument("--address")
    s = sub.add_parser("status", help="show the running head")
    s.add_argument("--address")

    cl = sub.add_parser("cluster", help="cluster spec lifecycle").add_subparsers(dest="sub", required=True)
    s = cl.add_parser("up")
    s.add_argument("-f", "--file", required=True)
    s.add_argument("--num-gpus", type=int)
    s.add_argument("--port", type=int)
    s.add_argument("--block", action="store_true")
    s = cl.add_parser("down")
    s.add_argument("--address")
    s = cl.add_parser("validate")
    s.add_argument("-f", "--file", required=True)

    job = sub.add_parser("job", help="job submission").add_subparsers(dest="sub", required=True)
    s = job.add_parser("submit")
    s.add_argument("--address")
    s.add_argument("--runtime-env-json")
    s.add_argument("--runtime-env", help="runtime env YAML file")
    s.add_argument("--working-dir")
    s.add_argument("--submission-id", "--job-id", dest="submission_id")
    s.add_argument("--metadata-json")
    s.add_argument("--entrypoint-num-gpus", type=float)
    s.add_argument("--no-wait", action="store_true")
    s.add_argument("entrypoint", nargs=argparse.REMAINDER)
    for name in ("status", "logs", "stop", "delete"):
        s = job.add_parser(name)
        s.add_argument("job_id")
        s.add_argument("--address")
        if name == "logs":
            s.add_argument("-f", "--follow", action="store_true")
    s = job.add_parser("list")
    s.add_argument("--address")
    return ap


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    if a.cmd == "start" or (a.cmd == "cluster" and a.sub == "up"):
        info = start_head(_spec_from_args(a), block=getattr(a, "block", False))
        if "address" in info:
            print(f"grt head started at {info['address']} with {info['num_gpus']} GPU(s); "
                  f"session {info['session_dir']}")
        return int(info.get("rc", 0))
    if a.cmd == "stop" or (a.cmd == "cluster" and a.sub == "down"):
        ok = stop_head(a.address)
        print("stopped" if ok else "no running head")
        return 0
    if a.cmd == "status":
        cur = read_current_cluster()
        if cur is None and not a.address:
            print(f"no running head ({current_cluster_file()})")
            return 1
        print(json.dumps(JobSubmissionClient(a.address).cluster_status(), indent=1))
        return 0
    if a.cmd == "cluster" and a.sub == "validate":
        spec = ClusterSpec.load(a.file).validate()
        print(json.dumps(spec.to_dict(), indent=1))
        return 0
    if a.cmd == "job":
        if a.sub == "submit":
            return cmd_job_submit(a)
        c = JobSubmissionClient(a.address)
        if a.sub == "status":
            info = c.get_job_info(a.job_id)
            print(f"Status for job '{a.job_id}': {info['status']}\nStatus message: {info['message']}")
            return 0
        if a.sub == "logs":
            if a.follow:
                for chunk in c.tail_job_logs(a.job_id):
                    sys.stdout.write(chunk)
            else:
                sys.stdout.write(c.get_job_logs(a.job_id))
            return 0
        if a.sub == "stop":
            print("stop requested" if c.stop_job(a.job_id) else "job is not running")
            return 0
        if a.sub == "delete":
            print("deleted" if c.delete_job(a.job_id) else "job is still running or unknown")
            return 0
        if a.sub == "list":
            for j in c.list_jobs():
                print(f"{j['submission_id']}\t{j['status']}\t{j['entrypoint']}")
            return 0
    return 2


if __name__ == "__main__":
    sys.exit(main())
