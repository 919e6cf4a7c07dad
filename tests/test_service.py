"""Control-plane tests: REST routes (ApiResult shape), batch scheduling (ports ConfigHelperTest.cs and the slot
assertions of RuntimeConfigGenerationBatchTest.cs), metrics ingestion (ports MetricsIngestorTests.cs), LiveQuery
kernels, schema inference and job lifecycle with a real engine subprocess."""
import datetime as dt
import json
import os
import time

import pytest

from dxa.service import scheduler as S
from dxa.service.metrics_ingestor import generate_row, ingest_lines
from dxa.telemetry.metrics import MetricStore

from tests.fixtures import ref_path

SAMPLE = ref_path("DeploymentLocal/sample/HomeAutomationLocal.json")
BATCH = ref_path("Services/DataX.Config/DataX.Config.Test/Resource/batchFlow.json")

SCHEMA = json.dumps({"type": "struct", "fields": [
    {"name": "deviceId", "type": "long", "nullable": True, "metadata": {}},
    {"name": "deviceType", "type": "string", "nullable": True, "metadata": {}},
    {"name": "temp", "type": "double", "nullable": True, "metadata": {}}]})


def mini_flow(name="mini"):
    return {"name": name, "gui": {
        "name": name, "displayName": name,
        "input": {"type": "local", "mode": "streaming",
                  "properties": {"inputSchemaFile": SCHEMA, "normalizationSnippet": "Raw.*", "eventsPerBatch": "50",
                                 "windowDuration": "1"}},
        "process": {"queries": ["--DataXQuery--\nT1 = SELECT deviceType, COUNT(*) AS n FROM DataXProcessedInput "
                                "GROUP BY deviceType"], "functions": []},
        "outputs": [], "rules": []}}


@pytest.fixture()
def client(tmp_path, monkeypatch):
    from fastapi.testclient import TestClient
    from dxa.service.app import create_app
    monkeypatch.setenv("DXA_SECRETS_DIR", str(tmp_path / "secrets"))
    monkeypatch.setenv("DXA_SUPERVISE", "0")          # tests drive the supervisor by hand
    return TestClient(create_app(str(tmp_path / "root")))


# -- ConfigHelperTest.cs --------------------------------------------------------------------------------------------
def test_partition_increment():
    base = "wasbs://container@sa.blob.core.windows.net/path1/"
    assert S.partition_increment(base + "{yyyy/MM/dd/hh}") == 60
    assert S.partition_increment(base + "{yyyy-MM-dd-hh}") == 60
    assert S.partition_increment(base + "{yyyy/MM/dd/hh}/path2") == 60
    assert S.partition_increment(base + "{yyyy/MM/dd}") == 1440
    assert S.partition_increment(base + "{yyyy/MM}") == 43200
    assert S.partition_increment(base + "{yyyy}") == 518400


def test_normalize_translate():
    cur = dt.datetime(2019, 9, 10, 13, 5, 30)
    assert S.normalize_time(cur, "min") == dt.datetime(2019, 9, 10, 13, 5)
    assert S.normalize_time(cur, "min", dt.timedelta(minutes=5)) == dt.datetime(2019, 9, 10, 13, 0)
    assert S.normalize_time(cur, "hour") == dt.datetime(2019, 9, 10, 13, 0)
    assert S.normalize_time(cur, "hour", dt.timedelta(minutes=5)) == dt.datetime(2019, 9, 10, 13, 0)
    assert S.normalize_time(cur, "default") == dt.datetime(2019, 9, 10)
    assert S.translate_interval("10", "min") == dt.timedelta(minutes=10)
    assert S.translate_interval("10", "hour") == dt.timedelta(hours=10)
    assert S.translate_interval("10", "default") == dt.timedelta(days=10)
    assert S.translate_window("10", "min") == dt.timedelta(minutes=9, seconds=59, milliseconds=59)
    assert S.translate_window("10", "hour") == dt.timedelta(hours=9, minutes=59, seconds=59, milliseconds=59)
    assert S.translate_window("10", "default") == dt.timedelta(days=9, hours=23, minutes=59, seconds=59,
                                                               milliseconds=59)
    assert S.translate_delay("10", "hour") == dt.timedelta(hours=10)


def test_schedule_predicates():
    now = dt.datetime.utcnow()
    assert not S.should_schedule(True, False, now, now + dt.timedelta(days=1))
    assert not S.should_schedule(False, False, None, now)
    assert not S.should_schedule(False, True, now, None)
    assert S.should_schedule(False, False, now, None)
    assert S.should_schedule(False, True, now, now)
    assert not S.is_valid_recurring(now, now + dt.timedelta(days=1), None)
    assert not S.is_valid_recurring(now, now - dt.timedelta(days=2), now - dt.timedelta(days=1))
    assert S.is_valid_recurring(now, now - dt.timedelta(days=1), now + dt.timedelta(days=1))
    assert S.blob_partition_format("batching", "yyyy-MM-dd/HH") == "%1$ty-%1$tm-%1$td/%1$tH"
    assert S.blob_partition_format("streaming", "x") == "%1$tY/%1$tm/%1$td/%1$tH/${quarterBucket}/${minuteBucket}"


# -- RuntimeConfigGenerationBatchTest.cs ---------------------------------------------------------------------------
@pytest.mark.skipif(not os.path.exists(BATCH), reason="reference fixtures not mounted")
def test_batch_slots_match_reference():
    now = dt.datetime.utcnow().replace(microsecond=0)
    start, end = now - dt.timedelta(days=1), now + dt.timedelta(days=1)
    text = open(BATCH, encoding="utf-8-sig").read()
    text = text.replace("${startTime}", start.isoformat() + "Z").replace("${endTime}", end.isoformat() + "Z")
    flow = json.loads(text)
    slots = S.plan_batches(flow, now)
    re_slots = [s for s in slots if not s["isOneTime"]]
    ot_slots = [s for s in slots if s["isOneTime"]]
    assert len(re_slots) == 2 and len(ot_slots) == 3
    norm = start.replace(hour=0, minute=0, second=0)
    p = S._parse_time
    exp = norm
    for s in re_slots:
        a, b = p(s["processStartTime"]), p(s["processEndTime"])
        assert a == exp - dt.timedelta(days=2)
        assert b == exp + dt.timedelta(days=1, seconds=-1)
        assert (b - a).total_seconds() == 259199
        exp += dt.timedelta(days=1)
    exp = norm
    for s in ot_slots:
        a, b = p(s["processStartTime"]), p(s["processEndTime"])
        assert a == exp and (b - a).total_seconds() == 86399
        assert s["name"].startswith(flow["name"] + "-OneTime-")
        exp += dt.timedelta(days=1)
    gui = flow["gui"]
    assert gui["batchList"][1]["disabled"] is True                       # one-time disabled after scheduling
    assert gui["batchList"][0]["properties"]["lastProcessedTime"]        # recurring advanced
    # re-planning the recurring entry resumes after lastProcessedTime
    again = S.batch_slots(flow["name"], gui["batchList"][0], now)
    assert again["slots"] == []


# -- MetricsIngestorTests.cs ---------------------------------------------------------------------------------------
@pytest.mark.parametrize("line,length,tail", [
    ('{"val":0.998,"met":"sensor1","app":"MyFlow","uts":1542322572}', 47, '"val":0.998, "pivot1":""}'),
    ('{"val":0.998,"met":"sensor1","app":"MyFlow","uts":"2018-11-15T03:27:46.285Z"}', 47,
     '"val":0.998, "pivot1":""}'),
    ('{"Metric":0.998,"MetricName":"sensor1","Product":"MyFlow","EventTime":"2018-11-15T03:27:46.285Z",'
     '"Pivot1":"text"}', 51, '"val":0.998, "pivot1":"text"}'),
])
def test_metric_row(line, length, tail):
    key, content, score = generate_row(line, now_ms=1542322573123)
    assert key == "MyFlow:sensor1"
    assert content.startswith('{"uts":15') and len(content) == length and content.endswith(tail)
    assert score == 1542322573123


def test_ingest_lines_nx():
    st = MetricStore()
    r = ingest_lines(st, ['{"app":"a","met":"m","val":1}', "garbage", '{"app":"a","met":"m","val":2}'])
    assert r == {"messages": 3, "metrics": 2}
    assert len(st.zrangebyscore("a:m", 0, 1e18)) >= 1


# -- REST ----------------------------------------------------------------------------------------------------------
def test_flow_crud_and_codegen(client):
    f = mini_flow()
    r = client.post("/api/flow/save", json=f).json()
    assert r == {"error": False, "message": None, "result": {"name": "mini", "displayName": "mini"}}
    assert client.post("/api/flow/getall/min", json={}).json()["result"][0]["name"] == "mini"
    # gateway-shaped route works too
    got = client.post("/api/DataX.Flow/Flow.ManagementService/flow/get", json={"name": "mini"}).json()
    assert got["result"]["gui"]["name"] == "mini"
    gen = client.post("/api/flow/generateconfigs", json={"name": "mini"}).json()
    assert not gen["error"] and os.path.exists(gen["result"]["conf"])
    conf = open(gen["result"]["conf"]).read()
    assert "datax.job.name=mini" in conf
    jobs = client.post("/api/job/getall", json={}).json()["result"]
    assert [j["name"] for j in jobs] == ["mini"] and jobs[0]["state"] == "Idle"
    cg = client.post("/api/userqueries/codegen", json={"query": f["gui"]["process"]["queries"][0]}).json()
    assert "T1 = SELECT" in cg["result"]["code"]
    sch = client.post("/api/userqueries/schema", json={"query": f["gui"]["process"]["queries"][0],
                                                       "inputSchema": SCHEMA}).json()["result"]
    assert sch["T1"] == ["deviceType", "n"]
    assert client.post("/api/flow/get", json={"name": "nope"}).json()["error"] is True
    assert client.post("/api/flow/delete", json={"name": "mini"}).json()["result"] is True
    assert client.post("/api/flow/getall", json={}).json()["result"] == []


def test_flow_names_cannot_escape_the_runtime_root(client, tmp_path):
    victim = tmp_path / "victim"
    victim.mkdir()
    (victim / "keep.txt").write_text("x")
    for bad in (str(victim), "../victim", "..", "a/b", "mini.conf", ""):
        r = client.post("/api/flow/delete", json={"name": bad}).json()
        assert r["error"] is True, bad
        f = mini_flow()
        f["name"] = bad
        f["gui"]["name"] = bad
        if bad:
            assert client.post("/api/flow/save", json=f).json()["error"] is True, bad
    assert (victim / "keep.txt").exists()
    # a flow without a name gets its display name reduced to [a-z0-9] (FlowConfigBuilder.cs:66-75)
    f = mini_flow()
    f["name"] = ""
    f["gui"]["name"] = ""
    f["gui"]["displayName"] = "My IoT / Flow #2"
    assert client.post("/api/flow/save", json=f).json()["result"]["name"] == "myiotflow2"


def test_livequery_kernel(client):
    f = mini_flow()
    client.post("/api/flow/save", json=f)
    events = [json.dumps({"deviceId": i, "deviceType": "A" if i % 3 else "B", "temp": i * 0.5}) for i in range(30)]
    client.post("/api/inputdata/refreshsample", json={"name": "mini", "events": events})
    kid = client.post("/api/kernel", json={"flowName": "mini"}).json()["result"]
    r = client.post("/api/kernel/executequery", json={
        "kernelId": kid, "query": "--DataXQuery--\nT1 = SELECT deviceType, COUNT(*) AS n FROM DataXProcessedInput "
                                  "GROUP BY deviceType ORDER BY deviceType"}).json()
    assert r["result"] == ['{"deviceType":"A","n":20}', '{"deviceType":"B","n":10}']
    r = client.post("/api/kernel/executequery", json={"kernelId": kid, "query": "SELECT n FROM T1 WHERE n < 15"})
    assert r.json()["result"] == ['{"n":10}']
    assert client.post("/api/kernel/executequery", json={"kernelId": kid, "query": "CREATE TABLE acc (n long);"}
                       ).json()["result"] == ["done"]
    r = client.post("/api/kernel/executequery", json={
        "kernelId": kid, "query": "SELECT COUNT(*) AS n FROM DataXProcessedInput TIMEWINDOW('5 minutes') "
                                  "WITH UPSERT acc"}).json()
    assert r["result"] == ['{"n":30}']
    bad = client.post("/api/kernel/executequery", json={"kernelId": kid, "query": "SELECT nope FROM T1"}).json()
    assert bad["error"] is True
    assert len(client.post("/api/kernel/sampleinputfromquery", json={"kernelId": kid}).json()["result"]) == 30
    assert client.post("/api/kernel/delete", json={"kernelId": kid}).json()["result"] is True
    assert client.post("/api/kernel/executequery", json={"kernelId": kid, "query": "SELECT 1"}).json()["error"]


@pytest.mark.skipif(not os.path.exists(SAMPLE), reason="reference sample not mounted")
def test_livequery_generated_sample(client):
    flow = json.load(open(SAMPLE, encoding="utf-8-sig"))
    client.post("/api/flow/save", json=flow)
    kid = client.post("/api/kernel", json={"flowName": flow["name"]}).json()["result"]
    r = client.post("/api/kernel/executequery", json={
        "kernelId": kid, "query": "SELECT COUNT(*) AS n FROM DataXProcessedInput"}).json()
    assert r["result"] == ['{"n":200}']


def test_infer_schema_and_metrics(client):
    r = client.post("/api/inputdata/inferschema", json={"name": "x", "events": [{"a": 1, "b": {"c": "s"}},
                                                                                 {"a": 2.5}]}).json()
    sch = json.loads(r["result"]["Schema"])
    assert [f["name"] for f in sch["fields"]] == ["a", "b"] and sch["fields"][0]["type"] == "double"
    assert client.post("/api/data/upload", json=[{"app": "DATAX-x", "met": "m1", "val": 3}]).json() == "done"
    pts = client.get("/api/metrics/get", params={"m": "DATAX-x:m1"}).json()
    assert pts[-1]["val"] == 3.0
    r = client.post("/api/metrics/ingest", content='{"app":"p","met":"m","val":2}\nnot json',
                    headers={"content-type": "text/plain"}).json()
    assert r["result"] == {"messages": 2, "metrics": 1}
    assert client.get("/").status_code == 200


def test_auth_roles(tmp_path, monkeypatch):
    """Behind a trusted gateway (DXA_AUTH=gateway): roles from X-DXA-Roles (bearer tokens: tests/test_auth.py)."""
    from fastapi.testclient import TestClient
    from dxa.service.app import create_app
    monkeypatch.setenv("DXA_AUTH", "gateway")
    monkeypatch.setenv("DXA_SUPERVISE", "0")
    client = TestClient(create_app(str(tmp_path / "svc")))
    assert client.post("/api/flow/save", json=mini_flow()).status_code == 401
    assert client.post("/api/flow/save", json=mini_flow(), headers={"X-DXA-Roles": "DataXReader"}).status_code == 403
    assert client.post("/api/flow/save", json=mini_flow(), headers={"X-DXA-Roles": "DataXWriter"}).status_code == 200
    assert client.post("/api/flow/getall", json={}, headers={"X-DXA-Roles": "DataXReader"}).status_code == 200


@pytest.mark.timeout(300)
def test_job_lifecycle_runs_engine(client):
    client.post("/api/flow/save", json=mini_flow())
    client.post("/api/flow/generateconfigs", json={"name": "mini"})
    st = client.app.state.dxa
    job = st.jobs.upsert({"name": "mini", "args": {"maxBatches": "2", "realtime": "false"}})
    assert job["state"] == "Idle"
    r = client.post("/api/flow/startjobs", json={"name": "mini"}).json()
    assert not r["error"] and r["result"][0]["state"] == "Starting"
    deadline = time.time() + 240
    state = None
    while time.time() < deadline:
        state = client.post("/api/job/get", json={"name": "mini"}).json()["result"]["state"]
        if state in ("Success", "Error"):
            break
        time.sleep(0.5)
    log = open(st.jobs.get("mini")["log"]).read()
    assert state == "Success", log[-3000:]
    assert '"batches": 2' in log
    # restart then stop a long-running instance
    st.jobs.upsert({"name": "mini", "args": {"realtime": "true"}})
    client.post("/api/job/restart", json={"name": "mini"})
    time.sleep(1.0)
    r = client.post("/api/job/stop", json={"name": "mini"}).json()
    assert r["result"]["state"] == "Idle"


@pytest.mark.skipif(not os.path.exists(BATCH), reason="reference fixtures not mounted")
def test_schedulebatch_route_creates_slot_jobs(client, monkeypatch):
    now = dt.datetime.utcnow().replace(microsecond=0)
    text = open(BATCH, encoding="utf-8-sig").read()
    text = text.replace("${startTime}", (now - dt.timedelta(days=1)).isoformat() + "Z").replace(
        "${endTime}", (now + dt.timedelta(days=1)).isoformat() + "Z")
    flow = json.loads(text)
    st = client.app.state.dxa
    started = []
    monkeypatch.setattr(st.jobs, "restart", lambda name: started.append(name))
    assert not client.post("/api/flow/save", json=flow).json()["error"]
    r = client.post("/api/flow/schedulebatch", json={}).json()
    assert not r["error"], r
    names = r["result"][flow["name"]]
    assert len(names) == 5 and sorted(started) == sorted(names)
    job = st.jobs.get(names[0])
    assert job["app"] == "batch" and job["args"]["processStartTime"].endswith("Z")
    conf = open(job["confPath"]).read()
    assert "datax.job.input.default.blob.input0.path=" in conf
    assert "datax.job.input.default.blob.input0.partitionincrement=" in conf
    saved = client.post("/api/flow/get", json={"name": flow["name"]}).json()["result"]
    assert saved["gui"]["batchList"][1]["disabled"] is True


# -- ScenarioTester / DataXScenarios ---------------------------------------------------------------------------------
def test_scenario_runner_semantics():
    from dxa.service.scenarios import ScenarioResult, StepResult, scenario_from_json, step

    @step("stepOk")
    def ok(ctx):
        ctx["seq"] = ctx.get("seq", 0) + 1
        ctx["stepOk"] = ctx["seq"]
        return StepResult(True, "stepOk")

    @step("stepFail")
    def fail(ctx):
        ctx["seq"] = ctx.get("seq", 0) + 1
        ctx["stepFail"] = ctx["seq"]
        raise RuntimeError("boom")

    ctx = {}
    r = ScenarioResult("s", scenario_from_json("s", "[{'action':'stepFail'}, {'action':'stepOk'}]")).run(ctx)
    assert r.failed and ctx["stepFail"] == 1 and ctx["stepOk"] == 2          # later steps still run
    assert not ScenarioResult("s", [ok]).run({}).failed
    with pytest.raises(KeyError):
        scenario_from_json("s", "[{'action':'nope'}]")


def test_save_deploy_and_query_scenarios(client, monkeypatch):
    from dxa.service.scenarios import QUERY_AND_SCHEMA, SAVE_AND_DEPLOY, STEPS, run_parallel
    st = client.app.state.dxa
    started = []
    monkeypatch.setattr(st.jobs, "start", lambda name, *a, **k: started.append(name) or {"name": name})
    monkeypatch.setattr(st.jobs, "restart", lambda name: {"name": name})
    monkeypatch.setattr(st.jobs, "stop", lambda name, *a, **k: {"name": name})
    events = [json.dumps({"deviceId": i, "deviceType": "A", "temp": 1.5}) for i in range(10)]
    ctx = {"client": client, "flow": mini_flow("scn"), "events": events, "suffix": ""}
    res = run_parallel("deploy", [STEPS[s] for s in SAVE_AND_DEPLOY], ctx, 3)
    assert all(not r.failed for r in res), [(s.description, s.exception, s.result) for r in res
                                             for s in r.step_results]
    assert len(started) == 3
    res = run_parallel("query", [STEPS[s] for s in QUERY_AND_SCHEMA], ctx, 2)
    assert all(not r.failed for r in res), [(s.description, s.exception, s.result) for r in res
                                             for s in r.step_results]


@pytest.mark.timeout(300)
def test_supervisor_restarts_failed_job_from_checkpoint(client, tmp_path):
    """Fault injection fails the first attempt at batch 1; the supervisor restarts the job, which then completes
    (SURVEY §5 failure detection / recovery)."""
    from dxa.service.jobs import Supervisor
    client.post("/api/flow/save", json=mini_flow("flaky"))
    client.post("/api/flow/generateconfigs", json={"name": "flaky"})
    st = client.app.state.dxa
    marker = str(tmp_path / "fault.marker")
    st.jobs.upsert({"name": "flaky", "args": {"maxBatches": "3", "realtime": "false"},
                    "env": {"DXA_FAULT_INJECT": f"batch=1,once={marker}"}})

    def wait_final():
        t0 = time.time()
        while time.time() - t0 < 240:
            s = st.jobs.get("flaky")["state"]
            if s in ("Success", "Error", "Failed"):
                return s
            time.sleep(0.3)
        return None

    st.jobs.start("flaky")
    assert wait_final() == "Error" and os.path.exists(marker)
    sup = Supervisor(st.jobs, backoff_s=0.0)
    assert sup.check_once() == ["flaky"]
    assert wait_final() == "Success"
    log = open(st.jobs.get("flaky")["log"]).read()
    assert "injected fault at batch 1" in log and '"batches": 3' in log
    assert "Latency-Stage-parse" in log                       # stage timings are exported with batch metrics
    # a job that keeps failing is given up after max_restarts
    st.jobs.upsert({"name": "flaky", "env": {"DXA_FAULT_INJECT": "batch=0"}})
    sup2 = Supervisor(st.jobs, backoff_s=0.0, max_restarts=1)
    st.jobs.start("flaky")
    assert wait_final() == "Error"
    assert sup2.check_once() == ["flaky"]
    assert wait_final() == "Error"
    sup2.check_once()
    assert st.jobs.get("flaky")["state"] == "Failed"


def test_designer_shaped_flow_generates_and_runs(client, tmp_path):
    """A flow shaped exactly like the console designer builds it (blankFlow + a rule + a local output) saves,
    generates and runs."""
    g = {"name": "designed", "displayName": "designed", "owner": "me",
         "input": {"type": "local", "mode": "streaming", "properties": {
             "inputSchemaFile": SCHEMA, "normalizationSnippet": "Raw.*", "windowDuration": "1", "maxRate": "50",
             "timestampColumn": "", "watermarkValue": "0", "watermarkUnit": "second"}, "referenceData": []},
         "process": {"queries": ["--DataXQuery--\nT1 = ProcessRules(DataXProcessedInput);\n\nOUTPUT T1 TO Out1;"],
                     "functions": [], "jobconfig": {"jobNumGpus": "1"}},
         "outputs": [{"id": "Metrics", "type": "metric", "properties": {}},
                     {"id": "Out1", "type": "local", "properties": {"folder": str(tmp_path / "out"),
                                                                    "blobPartitionFormat": "yyyy/MM/dd/HH",
                                                                    "format": "json", "compressionType": "none"}}],
         "rules": [{"id": "hot", "type": "tag", "properties": {
             "_S_ruleId": "hot", "_S_ruleType": "SimpleRule", "_S_productId": "designed", "_S_ruleDescription": "hot",
             "_S_condition": "temp > 10", "_S_tagname": "Tag", "_S_tag": "Hot", "_S_severity": "Critical",
             "_S_isAlert": False, "_S_alertsinks": ["Metrics"], "schemaTableName": "DataXProcessedInput"}}],
         "batchList": []}
    assert not client.post("/api/flow/save", json={"name": "designed", "gui": g}).json()["error"]
    gen = client.post("/api/flow/generateconfigs", json={"name": "designed"}).json()
    assert not gen["error"], gen
    from dxa.config.settings import load_config, settings_from_arguments
    from dxa.engine.host import StreamingHost
    from dxa.engine.processor import Processor
    from dxa.io.sources import build_source
    d = load_config(settings_from_arguments([f"conf={gen['result']['conf']}"]))
    proc = Processor(d, "cpu")
    hist = StreamingHost(proc, build_source(d, "cpu", "local"), 1.0, max_batches=1, realtime=False).run()
    assert hist[-1]["Output_T1_Sink_InputEvents"] == 50
    files = [os.path.join(dp, f) for dp, _, fs in os.walk(tmp_path / "out") for f in fs]
    lines = [json.loads(l) for f in files for l in open(f).read().splitlines() if l.strip()]
    assert len(lines) == 50 and all("Rules" in r for r in lines)
    page = client.get("/").text
    assert "/dist/app.js" in page
