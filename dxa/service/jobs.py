"""Local job management: start / stop / restart / sync engine processes (the reference's SparkJobOperation +
LocalSparkClient: Services/DataX.Config/DataX.Config/InternalService/SparkJobOperation.cs:29-268 and
DataX.Config.Local/LocalSparkClient.cs:20-206).

A job runs as ``python -m dxa.app conf=<job.conf>`` — or, for ``gpus > 1``, under ``torch.distributed.run`` with one
rank per MI355X.  A job with a ``client`` field (``{"type": "livy" | "databricks", "connectionString": …}``) runs
remotely instead: it is submitted through ``job_clients`` (e.g. to another node's Livy-compatible ``/batches``
endpoint) and its state is synced from there.  Liveness = PID alive AND its recorded start time matches (PID reuse safe).  States follow the
reference: Idle → Starting → Running → Success / Error; ``start`` first ensures the job is not running (polling up
to 30 × 1 s), ``restart_all_with_retries`` retries failed starts.
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import threading
import time
from typing import Any, Dict, List, Optional

from .store import DocumentStore

IDLE, STARTING, RUNNING, SUCCESS, ERROR = "Idle", "Starting", "Running", "Success", "Error"
_COLL = "sparkJobs"


def _proc_start_time(pid: int) -> Optional[float]:
    try:
        with open(f"/proc/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        return float(fields[19])      # starttime in clock ticks since boot
    except (OSError, IndexError, ValueError):
        return None


class JobManager:
    def __init__(self, store: DocumentStore, log_dir: str, python: str = sys.executable):
        self.store = store
        self.log_dir = log_dir
        self.python = python
        self._procs: Dict[str, subprocess.Popen] = {}
        self._lock = threading.Lock()
        os.makedirs(log_dir, exist_ok=True)

    # -- entity management ------------------------------------------------------------------------------------------
    def upsert(self, job: Dict[str, Any]) -> Dict[str, Any]:
        old = self.store.get(_COLL, job["name"]) or {}
        merged = {**old, **job}
        merged.setdefault("state", IDLE)
        self.store.upsert(_COLL, job["name"], merged)
        return merged

    def get(self, name: str) -> Optional[Dict[str, Any]]:
        j = self.store.get(_COLL, name)
        return self._sync(j) if j else None

    def get_all(self) -> List[Dict[str, Any]]:
        return [self._sync(j) for j in self.store.get_all(_COLL)]

    def get_by_names(self, names: List[str]) -> List[Dict[str, Any]]:
        return [j for j in (self.get(n) for n in names) if j]

    def delete(self, name: str):
        self.stop(name)
        self.store.delete(_COLL, name)

    # -- lifecycle --------------------------------------------------------------------------------------------------
    def _command(self, job: Dict[str, Any]) -> List[str]:
        args = [f"conf={job['confPath']}"]
        if job.get("app"):
            args.append(f"app={job['app']}")
        for k, v in (job.get("args") or {}).items():
            args.append(f"{k}={v}")
        gpus = int(job.get("gpus", 1))
        if gpus > 1:
            return [self.python, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
                    "--master-addr", "127.0.0.1", "--master-port", str(job.get("port", 29600)), "-m", "dxa.app"] + args
        return [self.python, "-m", "dxa.app"] + args

    def _remote(self, job):
        spec = job.get("client")
        if not spec:
            return None
        from .job_clients import make_client
        return make_client(spec, getattr(self, "http", None))

    def _remote_job_data(self, job) -> Dict[str, Any]:
        if job.get("jobData"):
            return job["jobData"]
        args = [f"conf={job['confPath']}"] + [f"{k}={v}" for k, v in (job.get("args") or {}).items()]
        return {"name": job["name"], "file": "dxa.app", "args": args, "conf": {"gpus": int(job.get("gpus", 1))}}

    def start(self, name: str, ensure_stopped_retries: int = 30) -> Dict[str, Any]:
        job = self.store.get(_COLL, name)
        if job is None:
            raise KeyError(f"job {name} not found")
        client = self._remote(job)
        if client is not None:
            job = self._sync(job)
            if job["state"] in (STARTING, RUNNING):
                raise RuntimeError(f"job {name} is still {job['state']}")
            res = client.submit(self._remote_job_data(job))
            job.update(state=res.state if res.state != IDLE else STARTING, clientCache=res.client_cache,
                       remoteId=res.job_id, links=res.links, note=res.note, startedAt=time.time())
            self.store.upsert(_COLL, name, job)
            return job
        for _ in range(ensure_stopped_retries):
            job = self._sync(job)
            if job["state"] in (IDLE, SUCCESS, ERROR):
                break
            time.sleep(1.0)
        else:
            raise RuntimeError(f"job {name} is still {job['state']}")
        log_path = os.path.join(self.log_dir, f"{name}.log")
        env = dict(os.environ)
        env.update({k: str(v) for k, v in (job.get("env") or {}).items()})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
        with open(log_path, "ab") as logf:
            p = subprocess.Popen(self._command(job), stdout=logf, stderr=subprocess.STDOUT, env=env,
                                 start_new_session=True)
        with self._lock:
            self._procs[name] = p
        job.update(state=STARTING, pid=p.pid, pidStart=_proc_start_time(p.pid), startedAt=time.time(),
                   log=log_path)
        self.store.upsert(_COLL, name, job)
        return job

    def stop(self, name: str, timeout: float = 30.0) -> Optional[Dict[str, Any]]:
        job = self.store.get(_COLL, name)
        if job is None:
            return None
        client = self._remote(job)
        if client is not None:
            if job.get("clientCache"):
                res = client.stop(job["clientCache"])
                job.update(note=res.note)
            job.update(state=IDLE)
            self.store.upsert(_COLL, name, job)
            return job
        pid = job.get("pid")
        if pid and self._alive(job):
            try:
                os.killpg(pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
            t0 = time.time()
            while self._alive(job) and time.time() - t0 < timeout:
                self._reap(name)
                time.sleep(0.2)
            if self._alive(job):
                try:
                    os.killpg(pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
        self._reap(name)
        job.update(state=IDLE, pid=None)
        self.store.upsert(_COLL, name, job)
        return job

    def restart(self, name: str) -> Dict[str, Any]:
        self.stop(name)
        return self.start(name)

    def restart_all_with_retries(self, names: Optional[List[str]] = None, retries: int = 3) -> Dict[str, str]:
        out = {}
        for j in (self.get_by_names(names) if names else self.get_all()):
            for attempt in range(retries):
                try:
                    self.restart(j["name"])
                    out[j["name"]] = STARTING
                    break
                except Exception as e:  # noqa: BLE001
                    out[j["name"]] = f"{ERROR}: {e}"
                    time.sleep(1.0)
        return out

    def sync_all(self) -> List[Dict[str, Any]]:
        return self.get_all()

    # -- state ------------------------------------------------------------------------------------------------------
    def _reap(self, name):
        with self._lock:
            p = self._procs.get(name)
        if p is not None and p.poll() is not None:
            with self._lock:
                self._procs.pop(name, None)
            return p.returncode
        return None

    def _alive(self, job) -> bool:
        pid = job.get("pid")
        if not pid:
            return False
        st = _proc_start_time(pid)
        if st is None or (job.get("pidStart") is not None and st != job.get("pidStart")):
            return False
        try:
            with open(f"/proc/{pid}/stat") as f:
                state = f.read().rsplit(")", 1)[1].split()[0]
            return state != "Z"
        except OSError:
            return False

    def _sync(self, job: Dict[str, Any]) -> Dict[str, Any]:
        name = job["name"]
        client = self._remote(job)
        if client is not None:
            if job.get("clientCache") and job.get("state") in (STARTING, RUNNING):
                res = client.get(job["clientCache"])
                if res.state != job.get("state"):
                    job.update(state=res.state, note=res.note)
                    if res.client_cache is not None:
                        job["clientCache"] = res.client_cache
                    self.store.upsert(_COLL, name, job)
            return job
        rc = self._reap(name)
        state = job.get("state", IDLE)
        if state in (STARTING, RUNNING):
            if self._alive(job):
                state = RUNNING
            else:
                if rc is None:
                    with self._lock:
                        p = self._procs.get(name)
                    rc = p.returncode if p is not None else None
                state = SUCCESS if rc == 0 else ERROR
                job["pid"] = None
            if state != job.get("state"):
                job["state"] = state
                self.store.upsert(_COLL, name, job)
        return job


class Supervisor(threading.Thread):
    """Restarts failed streaming jobs from their last checkpoint (the role YARN attempt retries played for the
    reference: defaultSparkJob.json ``spark.yarn.maxAppAttempts`` + ``attemptFailuresValidityInterval``).

    A job in state Error with ``autoRestart`` (default on, off for batch jobs) is restarted after an exponential
    backoff; more than ``max_restarts`` failures inside ``window_s`` marks it ``Failed`` and stops restarting."""

    def __init__(self, jobs: JobManager, period_s: float = 5.0, max_restarts: int = 5, window_s: float = 3600.0,
                 backoff_s: float = 2.0, max_backoff_s: float = 120.0):
        super().__init__(daemon=True, name="dxa-supervisor")
        self.jobs = jobs
        self.period_s = period_s
        self.max_restarts = max_restarts
        self.window_s = window_s
        self.backoff_s = backoff_s
        self.max_backoff_s = max_backoff_s
        self._stop = threading.Event()
        self.restarts: Dict[str, List[float]] = {}

    def check_once(self, now: Optional[float] = None) -> List[str]:
        now = time.time() if now is None else now
        restarted = []
        for job in self.jobs.get_all():
            name = job["name"]
            if job.get("state") != ERROR or not job.get("autoRestart", job.get("app") != "batch"):
                continue
            hist = [t for t in self.restarts.get(name, []) if now - t < self.window_s]
            if len(hist) >= self.max_restarts:
                job["state"] = "Failed"
                self.jobs.store.upsert(_COLL, name, job)
                continue
            delay = min(self.max_backoff_s, self.backoff_s * (2 ** len(hist)))
            if hist and now - hist[-1] < delay:
                continue
            try:
                self.jobs.start(name)
                hist.append(now)
                restarted.append(name)
            except Exception:  # noqa: BLE001 — try again next period
                pass
            self.restarts[name] = hist
        return restarted

    def run(self):
        while not self._stop.wait(self.period_s):
            self.check_once()

    def stop(self):
        self._stop.set()
