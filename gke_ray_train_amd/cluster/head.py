"""Head node daemon: the job server the reference reaches through ``ray job submit``.

Reference flow (a3-mega/gke-ray-cluster-setup.sh:64-91): look up the head pod, ``kubectl
port-forward`` 8265, then ``ray job submit --address http://localhost:8265 --runtime-env-json
'{"working_dir": ..., "pip": [...], "env_vars": {...}}' -- python ray-jobs/<job>.py``. The Ray job
server uploads the working dir, builds the runtime env, runs the entrypoint as the job driver and
keeps its status and logs.

This daemon does the same on one MI355X node, speaking the same REST shape as Ray's job API
(``/api/jobs/``, ``/api/jobs/<id>``, ``/api/jobs/<id>/logs``, ``/api/jobs/<id>/stop``) so
``JobSubmissionClient`` code and the ``grt job`` CLI work unchanged:
* the entrypoint runs as a shell command in its own process group (stop = signal that group);
* ``working_dir`` is snapshotted into the job's directory (``.git``/``__pycache__`` skipped) and is
  the job's cwd and first ``sys.path`` entry;
* ``env_vars`` are exported; ``pip`` requirements are CHECKED for importability only — the node is
  offline — and missing ones are reported in the job log;
* the framework and its ``ray`` shim are put on ``PYTHONPATH`` so reference-style drivers
  (``import ray``; ``ray.init(address='auto')``) attach to this node's resources (``GRT_ADDRESS``,
  ``GRT_NUM_GPUS``);
* job records persist under ``<session>/jobs/<id>/`` (info.json, driver.log, working_dir/).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shlex
import shutil
import signal
import subprocess
import sys
import threading
import time
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from importlib.util import find_spec
from typing import Dict, Optional

from .spec import ClusterSpec

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SHIM_DIR = os.path.join(PKG_ROOT, "gke_ray_train_amd", "ray_compat")
TERMINAL = ("SUCCEEDED", "FAILED", "STOPPED")


def grt_tmpdir() -> str:
    return os.environ.get("GRT_TMPDIR", "/tmp/grt")


def current_cluster_file() -> str:
    return os.path.join(grt_tmpdir(), "grt_current_cluster")


def read_current_cluster() -> Optional[dict]:
    try:
        with open(current_cluster_file()) as f:
            info = json.load(f)
    except (OSError, ValueError):
        return None
    try:
        os.kill(int(info["pid"]), 0)
    except (OSError, KeyError, ValueError):
        return None  # stale record of a head that is gone
    return info


def _pip_name(req: str) -> str:
    name = re.split(r"[<>=!~\[; ]", req.strip(), maxsplit=1)[0]
    return {"scikit-learn": "sklearn", "pyyaml": "yaml", "protobuf": "google.protobuf"}.get(name.lower(),
                                                                                         name.replace("-", "_"))


class JobManager:
    def __init__(self, session_dir: str, spec: ClusterSpec, address: str):
        self.session_dir = session_dir
        self.spec = spec
        self.address = address
        self.jobs_dir = os.path.join(session_dir, "jobs")
        os.makedirs(self.jobs_dir, exist_ok=True)
        self._lock = threading.Lock()
        self._jobs: Dict[str, dict] = {}
        self._procs: Dict[str, subprocess.Popen] = {}

    # ------------------------------------------------------------------ records
    def _save(self, info):
        d = os.path.join(self.jobs_dir, info["submission_id"])
        os.makedirs(d, exist_ok=True)
        tmp = os.path.join(d, "info.json.tmp")
        with open(tmp, "w") as f:
            json.dump(info, f, indent=1)
        os.replace(tmp, os.path.join(d, "info.json"))

    def _update(self, sid, **kw):
        with self._lock:
            self._jobs[sid].update(kw)
            self._save(self._jobs[sid])

    def info(self, sid) -> Optional[dict]:
        with self._lock:
            j = self._jobs.get(sid)
            return dict(j) if j else None

    def list(self):
        with self._lock:
            return [dict(j) for j in self._jobs.values()]

    def log_path(self, sid):
        return os.path.join(self.jobs_dir, sid, "driver.log")

    def logs(self, sid) -> str:
        try:
            with open(self.log_path(sid), errors="replace") as f:
                return f.read()
        except OSError:
            return ""

    # ------------------------------------------------------------------ lifecycle
    def submit(self, entrypoint: str, runtime_env: Optional[dict] = None, submission_id: Optional[str] = None,
               metadata: Optional[dict] = None, entrypoint_num_gpus: float = 0, entrypoint_num_cpus: float = 0) -> str:
        sid = submission_id or f"raysubmit_{uuid.uuid4().hex[:16]}"
        with self._lock:
            if sid in self._jobs:
                raise ValueError(f"job {sid} already exists")
            info = {"submission_id": sid, "job_id": sid, "type": "SUBMISSION", "entrypoint": entrypoint,
                    "status": "PENDING", "message": "Job is queued", "runtime_env": runtime_env or {},
                    "metadata": metadata or {}, "start_time": int(time.time() * 1000), "end_time": None,
                    "driver_exit_code": None, "entrypoint_num_gpus": entrypoint_num_gpus,
                    "entrypoint_num_cpus": entrypoint_num_cpus}
            self._jobs[sid] = info
            self._save(info)
        threading.Thread(target=self._run, args=(sid,), daemon=True, name=f"job-{sid}").start()
        return sid

    def _prepare(self, sid, renv, log):
        jd = os.path.join(self.jobs_dir, sid)
        cwd = jd
        wd = renv.get("working_dir")
        if wd:
            if not os.path.isdir(wd):
                raise FileNotFoundError(f"runtime_env working_dir {wd!r} does not exist")
            cwd = os.path.join(jd, "working_dir")
            excludes = set(renv.get("excludes") or []) | {".git", "__pycache__", "gpurun_out"}
            shutil.copytree(wd, cwd, ignore=lambda d, names: [n for n in names if n in excludes], dirs_exist_ok=True)
        for req in renv.get("pip") or []:
            mod = _pip_name(req)
            if find_spec(mod.split(".")[0]) is None:
                log.write(f"[grt] runtime_env pip: {req!r} is not installed on this offline node; continuing "
                          f"without it\n")
        env = dict(os.environ)
        env.update(self.spec.workers.env)
        env.update({str(k): str(v) for k, v in (renv.get("env_vars") or {}).items()})
        py = [cwd, PKG_ROOT, SHIM_DIR] + [p for p in env.get("PYTHONPATH", "").split(os.pathsep) if p]
        env["PYTHONPATH"] = os.pathsep.join(py)
        env["GRT_ADDRESS"] = self.address
        env["GRT_NUM_GPUS"] = str(self.spec.workers.num_gpus_per_node)
        env["GRT_STORAGE_PATH"] = self.spec.storage.path
        env["GRT_JOB_ID"] = sid
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        return cwd, env

    def _run(self, sid):
        info = self.info(sid)
        with open(self.log_path(sid), "a", buffering=1) as log:
            try:
                cwd, env = self._prepare(sid, info["runtime_env"], log)
                proc = subprocess.Popen(info["entrypoint"], shell=True, cwd=cwd, env=env, stdout=log,
                                        stderr=subprocess.STDOUT, start_new_session=True)
            except Exception as e:  # runtime-env setup failure
                log.write(f"[grt] job setup failed: {e}\n")
                self._update(sid, status="FAILED", message=f"runtime env setup failed: {e}",
                             end_time=int(time.time() * 1000))
                return
            with self._lock:
                self._procs[sid] = proc
            self._update(sid, status="RUNNING", message="Job is currently running.", driver_pid=proc.pid)
            rc = proc.wait()
        with self._lock:
            self._procs.pop(sid, None)
            stopped = self._jobs[sid].get("stop_requested")
        if stopped:
            st, msg = "STOPPED", "Job was intentionally stopped."
        elif rc == 0:
            st, msg = "SUCCEEDED", "Job finished successfully."
        else:
            st, msg = "FAILED", f"Job entrypoint command failed with exit code {rc}"
        self._update(sid, status=st, message=msg, driver_exit_code=rc, end_time=int(time.time() * 1000))

    def stop(self, sid, grace: float = 5.0) -> bool:
        with self._lock:
            proc = self._procs.get(sid)
            if sid in self._jobs and self._jobs[sid]["status"] not in TERMINAL:
                self._jobs[sid]["stop_requested"] = True
        if proc is None:
            return False
        try:
            os.killpg(proc.pid, signal.SIGTERM)  # the job's own process group (start_new_session)
        except ProcessLookupError:
            return True

        def _escalate():
            try:
                proc.wait(grace)
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(proc.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        threading.Thread(target=_escalate, daemon=True).start()
        return True

    def delete(self, sid) -> bool:
        with self._lock:
            j = self._jobs.get(sid)
            if j is None or j["status"] not in TERMINAL:
                return False
            del self._jobs[sid]
        shutil.rmtree(os.path.join(self.jobs_dir, sid), ignore_errors=True)
        return True

    def stop_all(self):
        for sid in list(self._procs):
            self.stop(sid, grace=2.0)


def _make_handler(mgr: JobManager, server_ref: dict):
    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):  # quiet
            pass

        def _send(self, code, obj):
            b = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(b)))
            self.end_headers()
            self.wfile.write(b)

        def _body(self):
            n = int(self.headers.get("Content-Length") or 0)
            return json.loads(self.rfile.read(n) or b"{}") if n else {}

        def _parts(self):
            return [p for p in self.path.split("?")[0].split("/") if p]

        def do_GET(self):
            p = self._parts()
            if p == ["api", "version"]:
                return self._send(200, {"version": "grt-1", "ray_version": "2.46.0+grt", "ray_commit": "grt"})
            if p == ["api", "cluster_status"]:
                s = mgr.spec
                return self._send(200, {"name": s.name, "resources": {"GPU": s.workers.num_gpus_per_node,
                                                                      "CPU": s.workers.num_cpus or os.cpu_count()},
                                        "storage": s.storage.path, "session_dir": mgr.session_dir})
            if p == ["api", "jobs"]:
                return self._send(200, mgr.list())
            if len(p) == 3 and p[:2] == ["api", "jobs"]:
                info = mgr.info(p[2])
                return self._send(200, info) if info else self._send(404, {"error": f"job {p[2]} not found"})
            if len(p) == 4 and p[:2] == ["api", "jobs"] and p[3] == "logs":
                if mgr.info(p[2]) is None:
                    return self._send(404, {"error": f"job {p[2]} not found"})
                return self._send(200, {"logs": mgr.logs(p[2])})
            self._send(404, {"error": "not found"})

        def do_POST(self):
            p = self._parts()
            try:
                body = self._body()
            except ValueError:
                return self._send(400, {"error": "bad json"})
            if p == ["api", "jobs"]:
                try:
                    sid = mgr.submit(body["entrypoint"], body.get("runtime_env"), body.get("submission_id"),
                                     body.get("metadata"), body.get("entrypoint_num_gpus") or 0,
                                     body.get("entrypoint_num_cpus") or 0)
                except (KeyError, ValueError) as e:
                    return self._send(400, {"error": str(e)})
                return self._send(200, {"submission_id": sid, "job_id": sid})
            if len(p) == 4 and p[:2] == ["api", "jobs"] and p[3] == "stop":
                if mgr.info(p[2]) is None:
                    return self._send(404, {"error": f"job {p[2]} not found"})
                return self._send(200, {"stopped": mgr.stop(p[2])})
            if p == ["api", "shutdown"]:
                self._send(200, {"ok": True})
                threading.Thread(target=server_ref["shutdown"], daemon=True).start()
                return
            self._send(404, {"error": "not found"})

        def do_DELETE(self):
            p = self._parts()
            if len(p) == 3 and p[:2] == ["api", "jobs"]:
                return self._send(200, {"deleted": mgr.delete(p[2])})
            self._send(404, {"error": "not found"})
    return H


def serve(spec: ClusterSpec, session_dir: Optional[str] = None, write_cluster_file: bool = True):
    """Run the head (blocking) until ``/api/shutdown`` or SIGTERM."""
    session_dir = session_dir or os.path.join(grt_tmpdir(), f"session_{time.strftime('%Y-%m-%d_%H-%M-%S')}_{os.getpid()}")
    os.makedirs(session_dir, exist_ok=True)
    os.makedirs(spec.storage.path, exist_ok=True)
    srv = ThreadingHTTPServer((spec.head.dashboard_host, int(spec.head.dashboard_port)), None)
    host, port = srv.server_address[:2]
    address = f"http://{host}:{port}"
    mgr = JobManager(session_dir, spec, address)
    ref = {}

    def shutdown():
        mgr.stop_all()
        srv.shutdown()
    ref["shutdown"] = shutdown
    srv.RequestHandlerClass = _make_handler(mgr, ref)
    signal.signal(signal.SIGTERM, lambda *_: threading.Thread(target=shutdown, daemon=True).start())
    rec = {"address": address, "pid": os.getpid(), "session_dir": session_dir, "name": spec.name,
           "num_gpus": spec.workers.num_gpus_per_node, "num_cpus": spec.workers.num_cpus,
           "storage": spec.storage.path}
    with open(os.path.join(session_dir, "cluster.json"), "w") as f:
        json.dump({**rec, "spec": spec.to_dict()}, f, indent=1)
    if write_cluster_file:
        os.makedirs(grt_tmpdir(), exist_ok=True)
        tmp = current_cluster_file() + f".{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(rec, f)
        os.replace(tmp, current_cluster_file())
    print(f"[grt] head up at {address} (session {session_dir})", flush=True)
    try:
        srv.serve_forever(poll_interval=0.2)
    finally:
        srv.server_close()
        if write_cluster_file:
            cur = read_current_cluster()
            if cur is None or cur.get("pid") == os.getpid():
                try:
                    os.remove(current_cluster_file())
                except OSError:
                    pass


def main(argv=None):
    ap = argparse.ArgumentParser(description="grt head node (job server)")
    ap.add_argument("--spec-json", default="")
    ap.add_argument("--session-dir", default="")
    a = ap.parse_args(argv)
    spec = ClusterSpec.from_dict(json.loads(a.spec_json)) if a.spec_json else ClusterSpec()
    serve(spec, a.session_dir or None)


if __name__ == "__main__":
    main()


__all__ = ["JobManager", "serve", "read_current_cluster", "current_cluster_file", "grt_tmpdir", "shlex"]
