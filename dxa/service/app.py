"""REST control plane (FastAPI) — the reference's Flow.ManagementService, Flow.InteractiveQueryService,
Flow.SchemaInferenceService, Flow.LiveDataService, onebox DataX.FlowManagement host, the gateway's role check and the
website's metrics API, in one process:

  flow/save · flow/schedulebatch · flow/generateconfigs · flow/get · flow/getall · flow/getall/min ·
  flow/startjobs · flow/restartjobs · flow/stopjobs · flow/delete · userqueries/schema · userqueries/codegen ·
  job/getall · job/get · job/getbynames · job/start · job/stop · job/restart · job/restartallwithretries ·
  job/syncall · job/syncbynames                                  (FlowManagementController.cs:26-510)
  kernel · kernel/refresh · kernel/deleteList · kernel/delete · kernels/delete · kernels/deleteall ·
  kernel/sampleinputfromquery · kernel/executequery                    (InteractiveQueryController.cs:33-171)
  inputdata/inferschema · inputdata/refreshsample · inputdata/refreshsampleandkernel
  api/metrics/get?m=&s=&e= · api/data/upload · api/metrics/ingest · api/ingest/{flow}

Every response is ``{"error": bool, "message": str|null, "result": …}`` (Services/DataX.Contract/Result/ApiResult.cs).
Routes are served both at ``/api/<route>`` and behind the gateway shape ``/api/{application}/{service}/<route>``;
every route is authenticated by ``dxa.service.auth`` (Azure AD / JWT bearer tokens with the DataXReader /
DataXWriter app roles, a trusted gateway's roles header, or loopback-only onebox mode; DataXAuthConstants.cs,
RolesCheck.cs) and write routes require the Writer role.

    python -m dxa.service.app --port 5000 --root ./.dxa
"""
from __future__ import annotations

import argparse
import json
import re
import os
import threading
import time
import uuid
from typing import Any, Dict, List, Optional

from fastapi import Body, FastAPI, Header, HTTPException, Query, Request
from fastapi.responses import JSONResponse

from ..flow import configgen
from ..flow import designer
from ..sql.codegen import generate_code
from ..telemetry.metrics import MetricStore
from .jobs import JobManager
from .livequery import KernelError, KernelManager
from .schema_inference import infer_schema
from .sqlanalyzer import analyze
from .store import DocumentStore

# routes needing the Writer role: FlowManagementController's mutations, and — as in the reference, whose
# SchemaInferenceController / InteractiveQueryController / LiveDataController are [DataXWriter] — schema inference
# and every LiveQuery kernel route
WRITE_ROUTES = {"flow/save", "flow/schedulebatch", "flow/generateconfigs", "flow/startjobs", "flow/restartjobs",
                "flow/stopjobs", "flow/delete", "job/start", "job/stop", "job/restart", "job/restartallwithretries",
                "job/syncall", "job/syncbynames", "inputdata/inferschema", "inputdata/refreshsample",
                "inputdata/refreshsampleandkernel", "kernel", "kernel/refresh", "kernel/deleteList", "kernel/delete",
                "kernels/delete", "kernels/deleteall", "kernel/sampleinputfromquery", "kernel/executequery",
                "ingest", "metrics/ingest"}


_FLOW_NAME = re.compile(r"^[A-Za-z0-9]+$")


def valid_flow_name(display_name: str) -> str:
    """The reference's ``GenerateValidFlowName`` (FlowConfigBuilder.cs:66-75, EngineEnvironment.cs:165-171): keep
    ``[A-Za-z0-9]``, lower-case; an empty display name gets a GUID."""
    if not display_name or not display_name.strip():
        display_name = uuid.uuid4().hex
    name = re.sub(r"[^A-Za-z0-9]", "", display_name).lower()
    if not name:
        raise ValueError(f"display name '{display_name}' has no alphanumeric characters")
    return name


def check_flow_name(name) -> str:
    """Flow names become folder and file names (runtime configs, checkpoints, secrets): only ``[A-Za-z0-9]+`` is
    accepted, so no name can be absolute or climb out of the runtime root."""
    if not isinstance(name, str) or not _FLOW_NAME.match(name):
        raise ValueError(f"invalid flow name {name!r}: only letters and digits are allowed")
    return name


def ok(result=None, message=None):
    return {"error": False, "message": message, "result": result}


def err(message, result=None):
    return {"error": True, "message": str(message), "result": result}


class ServiceState:
    def __init__(self, root: str, device: str = "cpu", metrics_endpoint: Optional[str] = None):
        self.root = os.path.abspath(root)
        os.makedirs(self.root, exist_ok=True)
        os.environ.setdefault("DXA_SECRETS_DIR", os.path.join(self.root, "secrets"))
        # DXA_DESIGN_STORE=cosmos:<conn>;Database=<db> shares flows/jobs across control planes; default local SQLite
        from .store import open_store
        self.store = open_store(os.environ.get("DXA_DESIGN_STORE") or os.path.join(self.root, "local.db"))
        self.jobs = JobManager(self.store, os.path.join(self.root, "logs"))
        from .jobs import Supervisor
        self.supervisor = Supervisor(self.jobs)
        if os.environ.get("DXA_SUPERVISE", "1") == "1":
            self.supervisor.start()
        self.kernels = KernelManager(device)
        self.metrics = MetricStore.default()
        self.metrics_endpoint = metrics_endpoint
        self.local_cache: List[Dict[str, Any]] = []       # onebox metric ring (localCache.js: 10 000 points)
        self.samples: Dict[str, List[str]] = {}
        self.queues: Dict[str, Any] = {}


def create_app(root: str = ".dxa", device: str = "cpu", metrics_endpoint: Optional[str] = None) -> FastAPI:
    app = FastAPI(title="dxa control plane")
    st = ServiceState(root, device, metrics_endpoint)
    app.state.dxa = st

    from .auth import AuthError, Authenticator
    authn = Authenticator()
    app.state.auth = authn

    def authorize(route: str, roles: Optional[str], authorization: Optional[str] = None,
                  client_host: Optional[str] = None):
        """Reader / Writer role check (dxa.service.auth: JWT bearer tokens, trusted gateway header, or local
        onebox only)."""
        try:
            return authn.check(route in WRITE_ROUTES, authorization, roles, client_host)
        except AuthError as e:
            raise HTTPException(status_code=e.status, detail=str(e))

    # ---------------------------------------------------------------------------------------------------------------
    def _flow(name: str) -> Dict[str, Any]:
        f = st.store.get("flows", check_flow_name(name))
        if f is None:
            raise KeyError(f"flow '{name}' not found")
        return f

    def _generate(name: str):
        flow = _flow(name)
        res = configgen.generate(flow, os.path.join(st.root, "runtime"), metrics_endpoint=st.metrics_endpoint)
        st.store.upsert("flows", name, res.flow)
        for j in res.jobs:
            st.jobs.upsert(j)
        return res

    handlers = {}

    def route(path):
        def deco(fn):
            handlers[path] = fn
            return fn
        return deco

    @route("flow/save")
    def flow_save(body):
        flow = body if "gui" in body else {"name": body.get("name"), "gui": body}
        if "gui" not in body and body.get("displayName"):
            flow["displayName"] = body["displayName"]
        name = flow.get("name") or flow["gui"].get("name")
        if not name:
            # FlowConfigBuilder.cs:66-75: a new flow's name is its display name reduced to [a-z0-9]
            name = valid_flow_name(flow["gui"].get("displayName") or flow.get("displayName") or "")
        flow["name"] = check_flow_name(name)
        if isinstance(flow.get("gui"), dict) and flow["gui"].get("name"):
            flow["gui"]["name"] = flow["name"]
        old = st.store.get("flows", name) or {}
        merged = {**old, **flow}
        st.store.upsert("flows", name, merged)
        return {"name": name, "displayName": merged.get("displayName", name)}

    @route("flow/get")
    def flow_get(body):
        return _flow(body if isinstance(body, str) else body.get("flowName") or body.get("name"))

    @route("flow/getall")
    def flow_getall(body):
        return st.store.get_all("flows")

    @route("flow/getall/min")
    def flow_getall_min(body):
        return [{"name": f["name"], "displayName": f.get("displayName", f["name"]),
                 "owner": f.get("gui", {}).get("owner", "")} for f in st.store.get_all("flows")]

    @route("flow/generateconfigs")
    def flow_generate(body):
        name = body if isinstance(body, str) else body.get("name")
        res = _generate(name)
        return {"conf": res.conf_path, "jobs": [j["name"] for j in res.jobs]}

    @route("flow/startjobs")
    def flow_start(body):
        name = body if isinstance(body, str) else body.get("name")
        flow = _flow(name)
        if not flow.get("jobNames"):
            _generate(name)
            flow = _flow(name)
        return [st.jobs.start(j) for j in flow.get("jobNames", [])]

    @route("flow/stopjobs")
    def flow_stop(body):
        name = body if isinstance(body, str) else body.get("name")
        return [st.jobs.stop(j) for j in _flow(name).get("jobNames", [])]

    @route("flow/restartjobs")
    def flow_restart(body):
        name = body if isinstance(body, str) else body.get("name")
        _generate(name)
        return [st.jobs.restart(j) for j in _flow(name).get("jobNames", [])]

    @route("flow/delete")
    def flow_delete(body):
        name = check_flow_name(body if isinstance(body, str) else body.get("name") or body.get("flowName"))
        flow = st.store.get("flows", name) or {}
        for j in flow.get("jobNames", []):
            st.jobs.delete(j)
        st.store.delete("flows", name)
        # DeleteHelper: runtime configs, checkpoints/state and the flow's generated secrets go with it
        import shutil
        from ..config import secrets
        runtime = os.path.realpath(os.path.join(st.root, "runtime"))
        target = os.path.realpath(os.path.join(runtime, name))
        if os.path.dirname(target) != runtime:
            raise ValueError(f"flow runtime folder {target} is outside {runtime}")
        shutil.rmtree(target, ignore_errors=True)
        secrets.delete_prefix("dxa", f"{name}-")
        return True

    @route("flow/schedulebatch")
    def flow_schedule(body):
        from .scheduler import schedule_batches
        return schedule_batches(st, body)

    @route("userqueries/schema")
    def uq_schema(body):
        return analyze(body.get("query", ""), body.get("inputSchema"), rules=json.dumps(body.get("rules") or []))

    @route("userqueries/codegen")
    def uq_codegen(body):
        rules = [r.get("properties", r) for r in (body.get("rules") or [])]
        rc = generate_code(body.get("query", ""), rules, body.get("productId", ""))
        return {"code": rc.code, "outputs": rc.outputs, "accumulationTables": rc.accumulation_tables,
                "timeWindows": rc.time_windows, "metrics": rc.metrics}

    # ---- flow designer model (the reference computes these in the browser: datax-pipeline flowHelpers.js)
    @route("designer/conditions/sql")
    def designer_conditions_sql(body):
        agg = body.get("ruleType") == designer.AGGREGATE_RULE
        conds = body.get("conditions") or designer.default_group()
        return {"condition": designer.conditions_to_sql(conds, agg),
                "error": designer.validate_conditions(conds, body.get("ruleType", designer.SIMPLE_RULE)),
                "aggs": designer.config_aggregates(agg, conds, body.get("aggs") or []),
                "pivots": designer.config_pivots(agg, conds, body.get("pivots") or [])}

    @route("designer/flow/toconfig")
    def designer_to_config(body):
        return designer.flow_to_config(body.get("flow", body), body.get("query", ""))

    @route("designer/flow/fromconfig")
    def designer_from_config(body):
        return designer.config_to_flow(body.get("config", body))

    @route("job/getall")
    def job_getall(body):
        return st.jobs.get_all()

    @route("job/get")
    def job_get(body):
        return st.jobs.get(body if isinstance(body, str) else body.get("name"))

    @route("job/getbynames")
    def job_getbynames(body):
        return st.jobs.get_by_names(body)

    @route("job/start")
    def job_start(body):
        return st.jobs.start(body if isinstance(body, str) else body.get("name"))

    @route("job/stop")
    def job_stop(body):
        return st.jobs.stop(body if isinstance(body, str) else body.get("name"))

    @route("job/restart")
    def job_restart(body):
        return st.jobs.restart(body if isinstance(body, str) else body.get("name"))

    @route("job/restartallwithretries")
    def job_restart_all(body):
        return st.jobs.restart_all_with_retries(body if isinstance(body, list) else None)

    @route("job/syncall")
    def job_syncall(body):
        return st.jobs.sync_all()

    @route("job/syncbynames")
    def job_syncbynames(body):
        return st.jobs.get_by_names(body)

    # -- LiveQuery -----------------------------------------------------------------------------------------------
    def _gui_from(body):
        if "flowName" in body and not body.get("inputSchema"):
            return _flow(body["flowName"])["gui"]
        gui = body.get("gui") or {
            "input": {"properties": {"inputSchemaFile": body.get("inputSchema"),
                                     "normalizationSnippet": body.get("normalizationSnippet") or "Raw.*"},
                      "referenceData": body.get("referenceDatas") or body.get("referenceData") or []},
            "process": {"functions": body.get("functions") or []}}
        return gui

    @route("kernel")
    def kernel_create(body):
        name = body.get("name") or body.get("flowName")
        kid = st.kernels.create(_gui_from(body), st.samples.get(name))
        return kid

    @route("kernel/refresh")
    def kernel_refresh(body):
        k = st.kernels.get(body.get("kernelId"))
        k.refresh(st.samples.get(body.get("name") or body.get("flowName")))
        return body.get("kernelId")

    @route("kernel/deleteList")
    def kernel_delete_list(body):
        return [st.kernels.delete(k) for k in body]

    @route("kernel/delete")
    def kernel_delete(body):
        return st.kernels.delete(body if isinstance(body, str) else body.get("kernelId"))

    @route("kernels/delete")
    def kernels_delete(body):
        return [st.kernels.delete(k) for k in (body or [])]

    @route("kernels/deleteall")
    def kernels_deleteall(body):
        st.kernels.delete_all()
        return True

    @route("kernel/sampleinputfromquery")
    def kernel_sample(body):
        return st.kernels.get(body["kernelId"]).sample_input()

    @route("kernel/executequery")
    def kernel_exec(body):
        return st.kernels.get(body["kernelId"]).execute(body.get("query", ""))

    # -- schema inference / samples ----------------------------------------------------------------------------------
    def _sample(body) -> Optional[List[str]]:
        """Sample the flow's configured input (``inputType`` / ``inputMode`` of the InteractiveQueryObject) for
        ``seconds``, save the sample file (SchemaGenerator.SaveSample) and keep the raw events for LiveQuery."""
        from .sampler import SampleError, sample_input, save_sample
        if not (body.get("inputType") or (body.get("inputMode") or "").lower() == "batching"):
            return None
        try:
            sampled = sample_input(body)
        except SampleError as e:
            raise HTTPException(status_code=400, detail=str(e))
        if not sampled:
            raise HTTPException(status_code=400, detail="Can't capture any data from the data source.")
        name = body.get("name") or body.get("displayName") or "flow"
        save_sample(os.path.join(st.root, "samples"), name, body.get("userName") or "", sampled)
        return [e["Raw"] for e in sampled]

    @route("inputdata/inferschema")
    def infer(body):
        """SchemaInferenceManager.GetInputSchema: sample the configured input (or take posted ``events``), union-merge
        the JSON shapes into a Spark StructType."""
        events = body.get("events")
        if not events:
            events = _sample(body)
        if not events:
            events = st.samples.get(body.get("name"), [])
        if not events and body.get("name") in st.queues:
            events = st.queues[body.get("name")][:1000]
        res = infer_schema(events)
        if body.get("name"):
            st.samples[body["name"]] = [e if isinstance(e, str) else json.dumps(e) for e in events]
        return res

    @route("inputdata/refreshsample")
    def refresh_sample(body):
        events = body.get("events") or _sample(body) or []
        st.samples[body["name"]] = [e if isinstance(e, str) else json.dumps(e) for e in events]
        return len(st.samples[body["name"]])

    @route("inputdata/refreshsampleandkernel")
    def refresh_sample_kernel(body):
        refresh_sample(body)
        if body.get("kernelId"):
            st.kernels.get(body["kernelId"]).refresh(st.samples[body["name"]])
        return body.get("kernelId")

    def dispatch(route_name: str, body, roles, authorization=None, client_host=None):
        authorize(route_name, roles, authorization, client_host)
        fn = handlers.get(route_name)
        if fn is None:
            raise HTTPException(status_code=404, detail=f"unknown route {route_name}")
        try:
            return ok(fn(body if body is not None else {}))
        except (KeyError, ValueError, KernelError, configgen.ConfigGenerationError, RuntimeError) as e:
            return err(e)
        except Exception as e:  # noqa: BLE001
            return err(f"{type(e).__name__}: {e}")

    # -- metrics -------------------------------------------------------------------------------------------------
    def _client(request: Request) -> Optional[str]:
        return request.client.host if request.client else None

    @app.get("/api/metrics/get")
    def metrics_get(request: Request, m: str, s: float = 0, e: float = 1e18,
                    x_dxa_roles: Optional[str] = Header(None), authorization: Optional[str] = Header(None)):
        authorize("metrics/get", x_dxa_roles, authorization, _client(request))
        rows = st.metrics.zrangebyscore(m, s, e)
        return [json.loads(v) for _, v in rows]

    @app.post("/api/data/upload")
    def data_upload(request: Request, items: List[Dict[str, Any]] = Body(...),
                    x_dxa_roles: Optional[str] = Header(None), authorization: Optional[str] = Header(None)):
        authorize("metrics/ingest", x_dxa_roles, authorization, _client(request))
        from .metrics_ingestor import ingest_items
        ingest_items(st.metrics, items, st.local_cache)
        return "done"

    @app.post("/api/metrics/ingest")
    def metrics_ingest(request: Request, request_body: str = Body(..., media_type="text/plain"),
                       x_dxa_roles: Optional[str] = Header(None), authorization: Optional[str] = Header(None)):
        authorize("metrics/ingest", x_dxa_roles, authorization, _client(request))
        from .metrics_ingestor import ingest_lines
        return ok(ingest_lines(st.metrics, request_body.splitlines()))

    @app.post("/api/ingest/{flow}")
    def ingest(flow: str, request: Request, events: List[Any] = Body(...),
               x_dxa_roles: Optional[str] = Header(None), authorization: Optional[str] = Header(None)):
        authorize("ingest", x_dxa_roles, authorization, request.client.host if request.client else None)
        q = st.queues.setdefault(flow, [])
        q.extend(e if isinstance(e, str) else json.dumps(e) for e in events)
        del q[:-100_000]
        return ok(len(events))

    # the website: page routes, /dist packages, web-composition / user / functionenabled / freshness (website.py);
    # registered before the generic /api/{path} route below so its /api/* routes win
    from .website import mount_website
    mount_website(app, st, authn)

    # node-side Livy-compatible batch API (remote job submission: job_clients.LivyClient)
    from .job_clients import batch_routes
    batch_routes(app, st.jobs, authn)

    @app.get("/api/health")
    def health():
        return ok({"time": time.time()})

    # generic routes: /api/<route> and gateway-shaped /api/{application}/{service}/<route>
    async def _body(request: Request):
        raw = await request.body()
        if not raw:
            return None
        try:
            return json.loads(raw)
        except ValueError:
            return raw.decode()

    @app.api_route("/api/{path:path}", methods=["GET", "POST"])
    async def generic(path: str, request: Request, x_dxa_roles: Optional[str] = Header(None),
                      authorization: Optional[str] = Header(None)):
        parts = path.strip("/").split("/")
        body = await _body(request)
        if request.method == "GET" and body is None:
            body = dict(request.query_params) or None
        host = request.client.host if request.client else None
        for k in range(len(parts)):
            cand = "/".join(parts[k:])
            if cand in handlers:
                return JSONResponse(dispatch(cand, body, x_dxa_roles, authorization, host))
        raise HTTPException(status_code=404, detail=f"unknown route {path}")

    return app


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=5000)
    ap.add_argument("--root", default=".dxa")
    ap.add_argument("--device", default="cpu")
    args = ap.parse_args()
    import uvicorn
    endpoint = f"http://{args.host}:{args.port}/api/data/upload"
    uvicorn.run(create_app(args.root, args.device, endpoint), host=args.host, port=args.port)


if __name__ == "__main__":
    main()
