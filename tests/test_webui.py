"""Website packages (dxa/service/webui, the reference's Website/Packages) driven under node against a live control
plane: page routes and node-side APIs, the flow designer (tabs, validity markers, rule condition preview, save and
reload round trip), flow list, jobs page, metrics dashboard data sources and widgets, home page."""
import json
import os
import shutil
import socket
import subprocess
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node") or shutil.which("nodejs")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def server(tmp_path, monkeypatch):
    monkeypatch.setenv("DXA_SUPERVISE", "0")
    for k in ("DXA_AUTH", "DXA_AUTH_JWKS", "DXA_AUTH_HS256_SECRET"):
        monkeypatch.delenv(k, raising=False)
    import uvicorn
    from dxa.service.app import create_app
    app = create_app(str(tmp_path / "cp"))
    port = _free_port()
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning"))
    t = threading.Thread(target=srv.run, daemon=True)
    t.start()
    for _ in range(200):
        if srv.started:
            break
        time.sleep(0.05)
    yield app, f"http://127.0.0.1:{port}"
    srv.should_exit = True
    t.join(timeout=10)


def test_website_routes(tmp_path, monkeypatch):
    from fastapi.testclient import TestClient
    from dxa.service.app import create_app
    monkeypatch.setenv("DXA_SUPERVISE", "0")
    monkeypatch.setenv("DXA_AUTH", "off")
    c = TestClient(create_app(str(tmp_path / "cp")))
    for path in ("/", "/home", "/config", "/config/new", "/config/edit/abc", "/dashboard", "/dashboard/abc", "/jobs"):
        r = c.get(path)
        assert r.status_code == 200 and '/dist/app.js' in r.text, path
    r = c.get("/dist/pipeline/flowDefinition.js")
    assert r.status_code == 200 and r.headers["content-type"].startswith("text/javascript")
    assert c.get("/dist/../app.py").status_code == 404
    assert c.get("/dist/nope.js").status_code == 404
    comp = c.get("/api/web-composition").json()
    assert {p["packageName"] for p in comp["pages"]} == {"home", "pipeline", "metrics", "jobs"}
    u = c.get("/api/user").json()
    assert u["isWriter"] is True
    fe = c.get("/api/functionenabled").json()
    assert fe["saveFlowButtonEnabled"] and fe["jobActionsEnabled"]


def test_website_reader_gets_no_write_switches(tmp_path, monkeypatch):
    from fastapi.testclient import TestClient
    from dxa.service.app import create_app
    monkeypatch.setenv("DXA_SUPERVISE", "0")
    monkeypatch.setenv("DXA_AUTH", "gateway")
    c = TestClient(create_app(str(tmp_path / "cp")))
    assert c.get("/api/user").status_code == 401
    r = c.get("/api/user", headers={"X-DXA-Roles": "DataXReader"}).json()
    assert r["isWriter"] is False
    assert c.get("/api/functionenabled", headers={"X-DXA-Roles": "DataXReader"}).json() == {}
    assert c.get("/api/functionenabled", headers={"X-DXA-Roles": "DataXWriter"}).json()["deployFlowButtonEnabled"]


def test_every_module_parses():
    if NODE is None:
        pytest.skip("node not installed")
    web = os.path.join(ROOT, "dxa", "service", "webui")
    files = [os.path.join(dp, f) for dp, _, fs in os.walk(web) for f in fs if f.endswith(".js")]
    assert len(files) >= 15
    for f in files:
        r = subprocess.run([NODE, "--check", f], capture_output=True, text=True)
        assert r.returncode == 0, (f, r.stderr)


def test_website_end_to_end_under_node(server):
    if NODE is None:
        pytest.skip("node not installed")
    app, base = server
    st = app.state.dxa
    # a flow with metric points for the dashboard: 3 batches of 2000 events, 1 s apart
    from dxa.flow.templates import default_flow
    flow = default_flow("metricflow")
    flow["gui"] = {"name": "metricflow", "displayName": "metricflow", "input": {"type": "local", "properties": {}}}
    st.store.upsert("flows", "metricflow", flow)
    now = int(time.time() * 1000)
    for i in range(3):
        t = now - 3000 + 1000 * i
        st.metrics.zadd("DATAX-metricflow:Input_DataXProcessedInput_Events_Count", t, json.dumps({"uts": t, "val": 2000}))
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "webui", "run_ui.mjs"), base, "metricflow", ROOT],
                       capture_output=True, text=True, timeout=120)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, (r.stdout, r.stderr)
    out = json.loads(lines[-1])
    assert r.returncode == 0 and "error" not in out, out.get("error") or r.stderr
    assert out["route_edit"] == ["FlowDefinitionPanel", "abc"] and out["route_new"] == "FlowDefinitionPanel"
    assert out["user"]["isWriter"] and out["n_functions"] > 20
    assert out["valid_onebox"] is True
    assert out["valid_eventhub_noconn"] is False and out["valid_eventhub_conn"] is True
    assert out["cond_err"] == "Value field must be a number when a numeric operator is used"
    assert out["list_before"] is False  # metricflow exists already
    assert out["tabs"] == ["info", "input", "referenceData", "functions", "query", "rules", "outputs", "scale", "schedule"]
    assert out["deploy_enabled_new"] is True
    assert out["input_invalid_kafka"] is True and out["deploy_enabled_kafka"] is False
    assert out["input_invalid_local"] is False
    assert out["rule_preview"] is True
    assert out["saved_path"] == "/config/edit/uiflow1"
    assert out["reloaded"] == {"name": "uiflow1", "type": "local", "rules": 1, "cond": "temperature",
                               "display": "UI Flow 1"}
    assert out["stored_condition"] == "temperature > 90"
    assert out["list_after"] and out["jobs_row"]
    assert "6,000" in out["dash_text"] and out["dash_svg_paths"] >= 1
    assert out["home"] is True
