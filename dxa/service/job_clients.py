"""Remote job clients: submit / sync / stop engine jobs on another node through a Livy-style batch API or the
Databricks Jobs API (the reference's ISparkJobClient implementations: Services/DataX.Config/DataX.Config.LivyClient/
LivyClient.cs:30-200 and DataX.Config.DatabricksClient/DatabricksClient.cs:24-170), plus the node-side half: a
Livy-compatible ``/batches`` endpoint that runs ``dxa.app`` engine jobs on the GPUs of the node it serves
(``batch_routes``), so one control plane can drive a fleet of MI355X nodes.

Connection strings keep the reference's formats — ``endpoint=<url>;username=<u>;password=<p>`` (Livy,
ConnectionStringParser.cs) and ``endpoint=<url>;dbtoken=<token>`` (Databricks) — and may be ``keyvault://`` /
``secretscope://`` references.  State mapping follows the reference exactly: Livy ``starting/running/dead/success``
→ Starting/Running/Idle/Success; Databricks ``PENDING/RUNNING/INTERNAL_ERROR/SKIPPED|TERMINATING|TERMINATED`` →
Starting/Running/Error/Idle; a 404 for the batch/run resets the job to Idle so it can be started again.
"""
from __future__ import annotations

import base64
import json
import os
import re
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

import requests
from fastapi import Header, Request

from .jobs import ERROR, IDLE, RUNNING, STARTING, SUCCESS


class JobClientError(RuntimeError):
    pass


@dataclass
class JobSyncResult:
    job_id: Optional[str]
    state: str
    note: Optional[str] = None
    links: Optional[Dict[str, str]] = None
    client_cache: Optional[Dict[str, Any]] = None

    def to_dict(self) -> Dict[str, Any]:
        return {"jobId": self.job_id, "state": self.state, "note": self.note, "links": self.links,
                "clientCache": self.client_cache}


@dataclass
class HttpResult:
    ok: bool
    status: int
    content: str


def _resolve(conn: str) -> str:
    if conn.startswith(("keyvault://", "secretscope://")):
        from ..config.secrets import resolve
        return resolve(conn)
    return conn


class _Http:
    """Tiny HTTP layer (swappable in tests, like the reference's ILivyHttpClient / IDatabricksHttpClient)."""

    def __init__(self, headers: Dict[str, str], timeout: float = 30.0):
        self.headers = headers
        self.timeout = timeout

    def __call__(self, method: str, url: str, body: Optional[str] = None) -> HttpResult:
        try:
            r = requests.request(method, url, data=body, headers=self.headers, timeout=self.timeout)
        except requests.RequestException as e:
            raise JobClientError(f"{method} {url} failed: {e}") from e
        return HttpResult(200 <= r.status_code < 300, r.status_code, r.text)


# ---------------------------------------------------------------------------------------------------------------
# Livy
# ---------------------------------------------------------------------------------------------------------------

_LIVY_CONN = re.compile(r"^endpoint=([^;]*);username=([^;]*);password=(.*)$")
_LIVY_STATES = {"starting": STARTING, "running": RUNNING, "dead": IDLE, "success": SUCCESS}


def parse_livy_connection(conn: str) -> Dict[str, str]:
    m = _LIVY_CONN.match(_resolve(conn or ""))
    if not m:
        raise JobClientError("cannot parse connection string to access livy service")
    return {"endpoint": m.group(1), "username": m.group(2), "password": m.group(3)}


def parse_livy_state(state: str) -> str:
    if state not in _LIVY_STATES:
        raise JobClientError(f"Unexpected livy batch state:'{state}'")
    return _LIVY_STATES[state]


def parse_livy_batch(batch: Dict[str, Any]) -> JobSyncResult:
    ui = (batch.get("appInfo") or {}).get("sparkUiUrl")
    links = None if ui is None else {"App UI": ui, "Logs": ui.replace("/proxy/", "/cluster/app/")}
    log = batch.get("log")
    return JobSyncResult(str(batch["id"]), parse_livy_state(batch["state"]), "\n".join(log) if log else None, links,
                         batch)


class LivyClient:
    SUFFIX = "/batches"

    def __init__(self, connection_string: str, http: Optional[Callable[..., HttpResult]] = None):
        info = parse_livy_connection(connection_string)
        self.endpoint = info["endpoint"].rstrip("/")
        token = base64.b64encode(f"{info['username']}:{info['password']}".encode()).decode()
        self.http = http or _Http({"Authorization": f"Basic {token}", "Content-Type": "application/json",
                                   "X-Requested-By": "dxa"})

    def _result(self, r: HttpResult) -> JobSyncResult:
        if r.ok:
            try:
                return parse_livy_batch(json.loads(r.content))
            except (ValueError, KeyError) as e:
                raise JobClientError(f"Couldn't parse response from Livy service:'{r.content}', message:'{e}'")
        if r.status == 404:
            return JobSyncResult(None, IDLE, r.content)
        raise JobClientError(f"unexpected response from livy service:'{r.status}', message:'{r.content}'")

    def submit(self, job_data: Dict[str, Any]) -> JobSyncResult:
        return self._result(self.http("POST", self.endpoint + self.SUFFIX, json.dumps(job_data)))

    def get(self, client_cache: Dict[str, Any]) -> JobSyncResult:
        return self._result(self.http("GET", f"{self.endpoint}{self.SUFFIX}/{client_cache['id']}"))

    def stop(self, client_cache: Dict[str, Any]) -> JobSyncResult:
        r = self.http("DELETE", f"{self.endpoint}{self.SUFFIX}/{client_cache['id']}")
        if not r.ok and r.status != 404:
            raise JobClientError(f"failed to stop livy batch: '{r.content}'")
        return JobSyncResult(str(client_cache["id"]), IDLE, r.content)

    def get_all(self) -> List[JobSyncResult]:
        r = self.http("GET", self.endpoint + self.SUFFIX)
        if not r.ok:
            raise JobClientError(f"failed to get all batches: '{r.content}'")
        return [parse_livy_batch(b) for b in json.loads(r.content).get("sessions", [])]


# ---------------------------------------------------------------------------------------------------------------
# Databricks
# ---------------------------------------------------------------------------------------------------------------

_DB_CONN = re.compile(r"^endpoint=([^;]*);dbtoken=(.*)$")
_DB_STATES = {"PENDING": STARTING, "RUNNING": RUNNING, "INTERNAL_ERROR": ERROR, "SKIPPED": IDLE,
              "TERMINATING": IDLE, "TERMINATED": IDLE}


def parse_databricks_connection(conn: str) -> Dict[str, str]:
    m = _DB_CONN.match(_resolve(conn or ""))
    if not m:
        raise JobClientError("cannot parse connection string to access databricks service")
    return {"endpoint": m.group(1), "dbtoken": m.group(2)}


def parse_databricks_state(state: Optional[str]) -> str:
    if state not in _DB_STATES:
        raise JobClientError(f"Unexpected databricks job state:'{state}'")
    return _DB_STATES[state]


class DatabricksClient:
    def __init__(self, connection_string: str, http: Optional[Callable[..., HttpResult]] = None):
        info = parse_databricks_connection(connection_string)
        ep = info["endpoint"]
        self.endpoint = ep if ep.endswith("/") else ep + "/"
        self.http = http or _Http({"Authorization": f"Bearer {info['dbtoken']}", "Content-Type": "application/json"})

    def _call(self, method: str, api: str, body: str = "") -> HttpResult:
        return self.http(method, self.endpoint + api, body or None)

    def _result(self, r: HttpResult) -> JobSyncResult:
        if r.ok:
            try:
                job = json.loads(r.content)
                st = job.get("state") or {}
                return JobSyncResult(str(job.get("job_id")), parse_databricks_state(st.get("life_cycle_state")),
                                     st.get("state_message"), None, job)
            except (ValueError, KeyError, AttributeError) as e:
                raise JobClientError(f"Couldn't parse response from Databricks service:'{r.content}', message:'{e}'")
        if r.status == 404:
            return JobSyncResult(None, IDLE, r.content)
        raise JobClientError(f"unexpected response from Databricks service:'{r.status}', message:'{r.content}'")

    def submit(self, job_data: Dict[str, Any]) -> JobSyncResult:
        obj = json.loads(json.dumps(job_data))
        nc = obj.get("new_cluster") or {}
        if not nc.get("enableAutoscale"):
            nc.pop("autoscale", None)
        else:
            nc.pop("num_workers", None)
        created = self._call("POST", "jobs/create", json.dumps(obj))
        if not created.ok:
            raise JobClientError(f"jobs/create failed: {created.content}")
        job_id = json.loads(created.content)["job_id"]
        run = self._call("POST", "jobs/run-now", json.dumps({"job_id": job_id}))
        if not run.ok:
            raise JobClientError(f"jobs/run-now failed: {run.content}")
        run_id = json.loads(run.content)["run_id"]
        return self._result(self._call("GET", f"jobs/runs/get?run_id={run_id}"))

    def get(self, client_cache: Dict[str, Any]) -> JobSyncResult:
        return self._result(self._call("GET", f"jobs/runs/get?run_id={client_cache['run_id']}"))

    def stop(self, client_cache: Dict[str, Any]) -> JobSyncResult:
        self._call("POST", "jobs/runs/cancel", json.dumps({"run_id": client_cache["run_id"]}))
        self._call("POST", "jobs/delete", json.dumps({"job_id": client_cache.get("job_id")}))
        res = None
        for _ in range(6):              # while terminating, re-read the run state at most 5 more times
            res = self.get(client_cache)
            if res.state != RUNNING:
                break
        return res


def make_client(spec: Dict[str, Any], http=None):
    """``spec``: ``{"type": "livy" | "databricks", "connectionString": ...}`` (a job's ``client`` field)."""
    kind = (spec.get("type") or "").lower()
    if kind == "livy":
        return LivyClient(spec["connectionString"], http)
    if kind == "databricks":
        return DatabricksClient(spec["connectionString"], http)
    raise JobClientError(f"unknown job client type '{spec.get('type')}'")


# ---------------------------------------------------------------------------------------------------------------
# node side: Livy-compatible batch endpoint backed by the local JobManager
# ---------------------------------------------------------------------------------------------------------------

_TO_LIVY = {IDLE: "dead", STARTING: "starting", RUNNING: "running", SUCCESS: "success", ERROR: "dead"}


@dataclass
class BatchRegistry:
    jobs: Any                       # JobManager
    next_id: int = 0
    names: Dict[int, str] = field(default_factory=dict)

    def _view(self, bid: int) -> Dict[str, Any]:
        job = self.jobs.get(self.names[bid])
        if job is None:
            raise KeyError(bid)
        log = []
        if job.get("log"):
            try:
                with open(job["log"], errors="replace") as f:
                    log = f.read().splitlines()[-20:]
            except OSError:
                pass
        return {"id": bid, "name": job["name"], "state": _TO_LIVY.get(job.get("state"), "dead"),
                "appId": job.get("pid"), "appInfo": {"driverLogUrl": None, "sparkUiUrl": None}, "log": log}

    def submit(self, body: Dict[str, Any]) -> Dict[str, Any]:
        """``{"file": "dxa.app", "args": ["conf=…", …], "name": …, "conf": {"gpus": N, "env.X": v}}``."""
        args = {}
        conf_path = None
        for a in body.get("args") or []:
            k, _, v = str(a).partition("=")
            if k == "conf":
                conf_path = v
            else:
                args[k] = v
        if not conf_path:
            raise ValueError("batch needs a conf=<job.conf> argument")
        conf = body.get("conf") or {}
        self.next_id += 1
        bid = self.next_id
        name = body.get("name") or f"batch-{bid}"
        self.jobs.upsert({"name": name, "confPath": conf_path, "args": args, "gpus": int(conf.get("gpus", 1)),
                          "env": {k[4:]: v for k, v in conf.items() if k.startswith("env.")}})
        self.names[bid] = name
        self.jobs.start(name)
        return self._view(bid)

    def get(self, bid: int) -> Dict[str, Any]:
        return self._view(bid)

    def list(self) -> Dict[str, Any]:
        sessions = [self._view(b) for b in sorted(self.names)]
        return {"from": 0, "total": len(sessions), "sessions": sessions}

    def delete(self, bid: int) -> Dict[str, Any]:
        name = self.names.pop(bid)
        self.jobs.stop(name)
        return {"msg": "deleted"}


def batch_routes(app, jobs, authn=None, env: Optional[Dict[str, str]] = None):
    """Mount ``/batches`` (Livy batch protocol) on a FastAPI app, backed by ``jobs``.

    Submission and deletion start and stop engine processes with caller-chosen ``conf`` and ``env.*`` variables,
    so they need the Writer role and listing needs Reader — through ``authn`` (``dxa.service.auth``: bearer JWT,
    gateway roles header, or loopback-only onebox), or HTTP Basic credentials matching ``DXA_BATCHES_BASIC``
    (``user:password``; what ``LivyClient`` sends, from the job's ``livy://`` connection string)."""
    import hmac
    from fastapi import Body, HTTPException
    reg = BatchRegistry(jobs)
    app.state.batches = reg
    basic = (env if env is not None else os.environ).get("DXA_BATCHES_BASIC")

    def check(request: Request, need_writer: bool, authorization: Optional[str], roles: Optional[str]):
        if basic and authorization and authorization.lower().startswith("basic "):
            try:
                given = base64.b64decode(authorization[6:].strip()).decode("utf-8")
            except (ValueError, UnicodeDecodeError):
                given = ""
            if hmac.compare_digest(given.encode(), basic.encode()):
                return
            raise HTTPException(status_code=401, detail="invalid credentials")
        if authn is None:
            return
        from .auth import AuthError
        try:
            authn.check(need_writer, authorization, roles, request.client.host if request.client else None)
        except AuthError as e:
            raise HTTPException(status_code=e.status, detail=str(e))

    @app.post("/batches")
    def batches_submit(request: Request, body: Dict[str, Any] = Body(...),
                       authorization: Optional[str] = Header(None), x_dxa_roles: Optional[str] = Header(None)):
        check(request, True, authorization, x_dxa_roles)
        try:
            return reg.submit(body)
        except (ValueError, KeyError) as e:
            raise HTTPException(status_code=400, detail=str(e))

    @app.get("/batches")
    def batches_list(request: Request, authorization: Optional[str] = Header(None),
                     x_dxa_roles: Optional[str] = Header(None)):
        check(request, False, authorization, x_dxa_roles)
        return reg.list()

    @app.get("/batches/{bid}")
    def batches_get(bid: int, request: Request, authorization: Optional[str] = Header(None),
                    x_dxa_roles: Optional[str] = Header(None)):
        check(request, False, authorization, x_dxa_roles)
        if bid not in reg.names:
            raise HTTPException(status_code=404, detail=f"batch {bid} not found")
        return reg.get(bid)

    @app.delete("/batches/{bid}")
    def batches_delete(bid: int, request: Request, authorization: Optional[str] = Header(None),
                       x_dxa_roles: Optional[str] = Header(None)):
        check(request, True, authorization, x_dxa_roles)
        if bid not in reg.names:
            raise HTTPException(status_code=404, detail=f"batch {bid} not found")
        return reg.delete(bid)

    return reg
