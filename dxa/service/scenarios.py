"""Scenario runner + end-to-end service scenarios (the reference's Tests/ScenarioTester and Tests/DataXScenarios,
also driven on a schedule by Services/JobRunner).

A scenario is an ordered list of named steps sharing a context dict; a failing step marks the scenario failed but
the remaining steps still run (so cleanup steps execute) — ScenarioResult.cs:44-78.  ``run_parallel`` runs N
iterations concurrently, each with a copy of the context (ScenarioResult.RunAsync).  Scenarios can be described as
JSON ``[{"action": "saveJob"}, …]`` (ScenarioDescription.FromJson).

Built-in steps mirror SaveAndDeploy.cs:39-121 and InteractiveQueryAndSchemaGenScenarios.cs:61-150 against the REST
API (``http://host:port`` or an in-process FastAPI TestClient):

    python -m dxa.service.scenarios --url http://127.0.0.1:5000 --flow flow.json \\
        --steps saveJob,generateConfigs,startJob,restartJob,getFlow,stopJob --iterations 4
"""
from __future__ import annotations

import argparse
import copy
import json
import time
import uuid
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

STEPS: Dict[str, Callable[[Dict[str, Any]], "StepResult"]] = {}


def step(name: str):
    def deco(fn):
        STEPS[name] = fn
        fn.step_name = name
        return fn
    return deco


@dataclass
class StepResult:
    success: bool
    description: str
    result: str = ""
    exception: Optional[str] = None
    elapsed_s: float = 0.0


@dataclass
class ScenarioResult:
    description: str
    steps: List[Callable]
    step_results: List[StepResult] = field(default_factory=list)
    failed: bool = False
    elapsed_s: float = 0.0

    def run(self, ctx: Dict[str, Any]) -> "ScenarioResult":
        t0 = time.perf_counter()
        for fn in self.steps:
            s0 = time.perf_counter()
            try:
                r = fn(ctx)
                self.failed |= not r.success
            except Exception as e:  # noqa: BLE001 — keep going so later (cleanup) steps still run
                r = StepResult(False, getattr(fn, "step_name", fn.__name__), exception=f"{type(e).__name__}: {e}")
                self.failed = True
            r.elapsed_s = time.perf_counter() - s0
            self.step_results.append(r)
        self.elapsed_s = time.perf_counter() - t0
        return self


def scenario_from_json(description: str, text: str) -> List[Callable]:
    actions = json.loads(text.replace("'", '"'))
    out = []
    for a in actions:
        fn = STEPS.get(a["action"])
        if fn is None:
            raise KeyError(f"{a['action']} not found in step definitions")
        out.append(fn)
    return out


def run_parallel(description: str, steps: List[Callable], ctx: Dict[str, Any], iterations: int
                 ) -> List[ScenarioResult]:
    def iteration_ctx(i):
        c = dict(ctx)                         # the client is shared; everything an iteration writes is its own
        c["suffix"] = f"{ctx.get('suffix', '')}x{i}"
        return c
    with ThreadPoolExecutor(max_workers=max(1, iterations)) as ex:
        futs = [ex.submit(ScenarioResult(description, steps).run, iteration_ctx(i)) for i in range(iterations)]
        return [f.result() for f in futs]


# -- HTTP helpers -----------------------------------------------------------------------------------------------------
def _post(ctx, route: str, body):
    client = ctx["client"]
    if hasattr(client, "post"):                                 # FastAPI TestClient / httpx client
        r = client.post(f"/api/{route}", json=body, headers=ctx.get("headers") or {})
        return r.json()
    import urllib.request
    req = urllib.request.Request(f"{client}/api/{route}", data=json.dumps(body).encode(),
                                 headers={"Content-Type": "application/json", **(ctx.get("headers") or {})},
                                 method="POST")
    with urllib.request.urlopen(req, timeout=120) as resp:
        return json.loads(resp.read())


def _get(ctx, route: str, params: Dict[str, str]):
    client = ctx["client"]
    if hasattr(client, "get"):
        return client.get(f"/api/{route}", params=params, headers=ctx.get("headers") or {}).json()
    import urllib.parse
    import urllib.request
    with urllib.request.urlopen(f"{client}/api/{route}?{urllib.parse.urlencode(params)}", timeout=120) as r:
        return json.loads(r.read())


def _ok(res) -> bool:
    return isinstance(res, dict) and not res.get("error")


# -- SaveAndDeploy steps -----------------------------------------------------------------------------------------------
@step("saveJob")
def save_job(ctx):
    flow = copy.deepcopy(ctx["flow"])
    name = f"{flow.get('name', 'scenario')}{ctx.get('suffix', '')}"
    flow["name"] = name
    flow.setdefault("gui", {})["name"] = name
    res = _post(ctx, "flow/save", flow)
    if _ok(res):
        ctx["flowName"] = res["result"]["name"]
    return StepResult(_ok(res), "saveJob", f"created a flow '{ctx.get('flowName')}'")


@step("generateConfigs")
def generate_configs(ctx):
    res = _post(ctx, "flow/generateconfigs", ctx["flowName"])
    conf = res.get("result", {}).get("conf") if _ok(res) else None
    ctx["runtimeConf"] = conf
    return StepResult(bool(conf), "generateConfigs", f"created configs for the flow: '{conf}'")


@step("startJob")
def start_job(ctx):
    res = _post(ctx, "flow/startjobs", ctx["flowName"])
    return StepResult(_ok(res), "startJob", json.dumps(res.get("result"))[:200])


@step("restartJob")
def restart_job(ctx):
    res = _post(ctx, "flow/restartjobs", ctx["flowName"])
    return StepResult(_ok(res), "restartJob", json.dumps(res.get("result"))[:200])


@step("stopJob")
def stop_job(ctx):
    res = _post(ctx, "flow/stopjobs", ctx["flowName"])
    return StepResult(_ok(res), "stopJob", json.dumps(res.get("result"))[:200])


@step("getFlow")
def get_flow(ctx):
    res = _get(ctx, "flow/get", {"flowName": ctx["flowName"]})
    ok = _ok(res) and res["result"].get("name") == ctx["flowName"]
    return StepResult(ok, "getFlow", "acquired flow")


@step("deleteFlow")
def delete_flow(ctx):
    res = _post(ctx, "flow/delete", ctx["flowName"])
    return StepResult(_ok(res), "deleteFlow", "deleted")


# -- InteractiveQuery + schema steps -------------------------------------------------------------------------------
@step("inferSchema")
def infer_schema(ctx):
    res = _post(ctx, "inputdata/inferschema", {"name": ctx["flowName"], "events": ctx.get("events") or []})
    ok = _ok(res) and bool(res["result"].get("Schema"))
    if ok:
        ctx["inferredSchema"] = res["result"]["Schema"]
    return StepResult(ok, "inferSchema", (res.get("result") or {}).get("Schema", "")[:200])


@step("initializeKernel")
def initialize_kernel(ctx):
    res = _post(ctx, "kernel", {"flowName": ctx["flowName"]})
    ctx["kernelId"] = res.get("result") if _ok(res) else None
    return StepResult(bool(ctx["kernelId"]), "initializeKernel", str(ctx["kernelId"]))


@step("refreshKernel")
def refresh_kernel(ctx):
    res = _post(ctx, "kernel/refresh", {"kernelId": ctx["kernelId"], "flowName": ctx["flowName"]})
    return StepResult(_ok(res), "refreshKernel", str(res.get("result")))


@step("refreshSample")
def refresh_sample(ctx):
    res = _post(ctx, "inputdata/refreshsample", {"name": ctx["flowName"], "events": ctx.get("events") or []})
    return StepResult(_ok(res), "refreshSample", str(res.get("result")))


@step("refreshSampleAndKernel")
def refresh_sample_and_kernel(ctx):
    res = _post(ctx, "inputdata/refreshsampleandkernel",
                {"name": ctx["flowName"], "events": ctx.get("events") or [], "kernelId": ctx.get("kernelId")})
    return StepResult(_ok(res), "refreshSampleAndKernel", str(res.get("result")))


@step("executeQuery")
def execute_query(ctx):
    res = _post(ctx, "kernel/executequery", {"kernelId": ctx["kernelId"],
                                               "query": ctx.get("query") or "SELECT * FROM DataXProcessedInput"})
    return StepResult(_ok(res), "executeQuery", json.dumps(res.get("result"))[:200])


@step("deleteKernel")
def delete_kernel(ctx):
    res = _post(ctx, "kernel/delete", {"kernelId": ctx.get("kernelId")})
    return StepResult(_ok(res) and res.get("result") is True, "deleteKernel", str(res.get("result")))


SAVE_AND_DEPLOY = ["saveJob", "generateConfigs", "startJob", "restartJob", "getFlow", "stopJob"]
QUERY_AND_SCHEMA = ["saveJob", "inferSchema", "initializeKernel", "refreshKernel", "refreshSample",
                    "refreshSampleAndKernel", "executeQuery", "deleteKernel"]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", required=True)
    ap.add_argument("--flow", required=True, help="flow definition JSON file")
    ap.add_argument("--steps", default=",".join(SAVE_AND_DEPLOY))
    ap.add_argument("--iterations", type=int, default=1)
    ap.add_argument("--events", help="sample events file (JSON lines) for schema/LiveQuery steps")
    args = ap.parse_args(argv)
    ctx = {"client": args.url.rstrip("/"), "flow": json.load(open(args.flow, encoding="utf-8-sig")),
           "suffix": "x" + uuid.uuid4().hex[:6]}
    if args.events:
        ctx["events"] = [l for l in open(args.events).read().splitlines() if l.strip()]
    steps = [STEPS[s] for s in args.steps.split(",") if s]
    results = run_parallel("cli", steps, ctx, args.iterations)
    for r in results:
        print(json.dumps({"failed": r.failed, "elapsed_s": round(r.elapsed_s, 3),
                          "steps": [(s.description, s.success, round(s.elapsed_s, 3), s.exception)
                                    for s in r.step_results]}))
    raise SystemExit(1 if any(r.failed for r in results) else 0)


if __name__ == "__main__":
    main()
