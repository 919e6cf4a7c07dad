"""Remote job clients (Livy / Databricks protocol) and the node-side Livy-compatible /batches endpoint.

Client tests follow the reference's LivyClient / DatabricksClient tests with a fake HTTP layer
(Services/DataX.Config/DataX.Config.LivyClient.Test/Mock/HttpClient.cs); the end-to-end test drives a real engine
job on a "node" control plane from a second "fleet" control plane through the Livy batch protocol."""
import json
import time

import pytest

from dxa.service import job_clients as J
from tests.test_service import client, mini_flow  # noqa: F401  (fixture)


class FakeHttp:
    def __init__(self, routes):
        self.routes = routes          # (method, url-suffix) → (status, body) or callable(body)
        self.calls = []

    def __call__(self, method, url, body=None):
        self.calls.append((method, url, body))
        for (m, suffix), resp in self.routes.items():
            if m == method and url.endswith(suffix):
                status, content = resp(body) if callable(resp) else resp
                return J.HttpResult(200 <= status < 300, status, content if isinstance(content, str)
                                    else json.dumps(content))
        return J.HttpResult(False, 404, "not found")


def test_connection_strings_and_states():
    assert J.parse_livy_connection("endpoint=https://h/livy;username=u;password=p=x") == {
        "endpoint": "https://h/livy", "username": "u", "password": "p=x"}
    assert J.parse_databricks_connection("endpoint=https://adb/api/2.0/;dbtoken=dapi1") == {
        "endpoint": "https://adb/api/2.0/", "dbtoken": "dapi1"}
    with pytest.raises(J.JobClientError):
        J.parse_livy_connection("endpoint=x")
    assert [J.parse_livy_state(s) for s in ("starting", "running", "dead", "success")] == \
        ["Starting", "Running", "Idle", "Success"]
    assert [J.parse_databricks_state(s) for s in ("PENDING", "RUNNING", "INTERNAL_ERROR", "TERMINATED", "SKIPPED")] \
        == ["Starting", "Running", "Error", "Idle", "Idle"]
    with pytest.raises(J.JobClientError):
        J.parse_livy_state("busy")


def test_livy_client_protocol():
    batch = {"id": 7, "state": "starting", "appInfo": {"sparkUiUrl": "http://rm/proxy/app_1"}, "log": ["a", "b"]}
    http = FakeHttp({("POST", "/batches"): (201, batch),
                     ("GET", "/batches/7"): (200, {**batch, "state": "running"}),
                     ("DELETE", "/batches/7"): (200, {"msg": "deleted"}),
                     ("GET", "/batches"): (200, {"sessions": [batch]})})
    c = J.LivyClient("endpoint=http://node:8998;username=u;password=p", http)
    r = c.submit({"file": "dxa.app", "args": ["conf=/x.conf"]})
    assert (r.job_id, r.state, r.note) == ("7", "Starting", "a\nb")
    assert r.links == {"App UI": "http://rm/proxy/app_1", "Logs": "http://rm/cluster/app/app_1"}
    assert json.loads(http.calls[0][2])["args"] == ["conf=/x.conf"]
    assert c.get(r.client_cache).state == "Running"
    assert c.stop(r.client_cache).state == "Idle"
    assert [b.job_id for b in c.get_all()] == ["7"]
    assert c.get({"id": 99}).state == "Idle"                      # 404 → reset to Idle


def test_databricks_client_protocol():
    run = {"job_id": 11, "run_id": 5, "state": {"life_cycle_state": "PENDING", "state_message": "waiting"}}
    states = iter(["TERMINATING", "TERMINATED"])
    http = FakeHttp({("POST", "jobs/create"): (200, {"job_id": 11}),
                     ("POST", "jobs/run-now"): (200, {"run_id": 5}),
                     ("GET", "jobs/runs/get?run_id=5"): lambda b: (200, {**run, "state": {
                         "life_cycle_state": next(states, "TERMINATED")}}),
                     ("POST", "jobs/runs/cancel"): (200, {}),
                     ("POST", "jobs/delete"): (200, {})})
    c = J.DatabricksClient("endpoint=https://adb/api/2.0;dbtoken=t", http)
    job = {"name": "j", "new_cluster": {"enableAutoscale": False, "num_workers": 2,
                                        "autoscale": {"min_workers": 1, "max_workers": 4}}}
    r = c.submit(job)
    sent = json.loads(http.calls[0][2])
    assert "autoscale" not in sent["new_cluster"] and sent["new_cluster"]["num_workers"] == 2
    assert http.calls[0][1] == "https://adb/api/2.0/jobs/create"
    assert r.state == "Idle" and r.client_cache["run_id"] == 5           # first poll: TERMINATING
    assert c.stop({"run_id": 5, "job_id": 11}).state == "Idle"
    assert [m for m, _, _ in http.calls].count("POST") == 4


def test_fleet_control_plane_runs_job_on_node_through_livy_protocol(client, tmp_path, monkeypatch):
    """Node: a control plane serving /batches (its JobManager runs the engine).  Fleet: a second JobManager whose job
    has a Livy client pointing at the node.  start → engine runs on the node → sync reports Success."""
    node = client
    node.post("/api/flow/save", json=mini_flow())
    node.post("/api/flow/generateconfigs", json={"name": "mini"})
    conf = node.app.state.dxa.jobs.store.get("sparkJobs", "mini")["confPath"]

    def via_testclient(method, url, body=None):
        path = url.split("://", 1)[1].split("/", 1)[1]
        r = node.request(method, "/" + path, content=body, headers={"Content-Type": "application/json"})
        return J.HttpResult(200 <= r.status_code < 300, r.status_code, r.text)

    from dxa.service.jobs import JobManager
    from dxa.service.store import DocumentStore
    fleet = JobManager(DocumentStore(str(tmp_path / "fleet.db")), str(tmp_path / "fleet_logs"))
    fleet.http = via_testclient
    fleet.upsert({"name": "remote-mini", "confPath": conf, "args": {"maxBatches": "2", "realtime": "false"},
                  "client": {"type": "livy", "connectionString": "endpoint=http://node:8998;username=u;password=p"}})
    job = fleet.start("remote-mini")
    assert job["state"] in ("Starting", "Running") and job["clientCache"]["id"] == 1
    deadline = time.time() + 240
    while time.time() < deadline:
        job = fleet.get("remote-mini")
        if job["state"] in ("Success", "Idle", "Error"):
            break
        time.sleep(0.5)
    assert job["state"] == "Success", job
    listed = node.get("/batches").json()
    assert listed["total"] == 1 and listed["sessions"][0]["state"] == "success"
    assert any('"batches": 2' in line for line in listed["sessions"][0]["log"])
    assert node.delete("/batches/1").status_code == 200 and node.get("/batches/1").status_code == 404
