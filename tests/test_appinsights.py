"""AppInsights transport: batch lifecycle events and exceptions reach a v2/track endpoint as Breeze envelopes
(reference: AppInsightLogger.scala:40-105, EventHubStreamingFactory.scala:88,100-115)."""
import json
import threading
from http.server import BaseHTTPRequestHandler, HTTPServer

import pytest


@pytest.fixture
def collector():
    got = []

    class H(BaseHTTPRequestHandler):
        def do_POST(self):
            body = self.rfile.read(int(self.headers["Content-Length"]))
            got.append((self.path, json.loads(body)))
            self.send_response(200)
            self.end_headers()
            self.wfile.write(b'{"itemsReceived":1,"itemsAccepted":1,"errors":[]}')

        def log_message(self, *a):
            pass

    srv = HTTPServer(("127.0.0.1", 0), H)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield f"http://127.0.0.1:{srv.server_port}/", got
    srv.shutdown()


def test_key_parsing():
    from dxa.telemetry.appinsights import DEFAULT_ENDPOINT, parse_key
    assert parse_key("abc-123") == ("abc-123", DEFAULT_ENDPOINT)
    assert parse_key("InstrumentationKey=k1;IngestionEndpoint=https://x.in.applicationinsights.azure.com/") == \
        ("k1", "https://x.in.applicationinsights.azure.com/")
    with pytest.raises(ValueError):
        parse_key("IngestionEndpoint=https://x/")


def test_sender_off_without_key(monkeypatch):
    from dxa.telemetry import appinsights as AI
    monkeypatch.delenv("DATAX_APPINSIGHTKEYREF", raising=False)
    assert AI.configure(None, app_name="x") is None
    AI.track_event("streaming/batch/begin", {"batchTime": "1 ms"})
    assert AI.EVENTS[-1]["event"] == "datax/streaming/batch/begin"
    assert AI.EVENTS[-1]["props"]["context.appname"] == "x"


def test_streaming_host_emits_lifecycle_and_exceptions(tmp_path, collector):
    url, got = collector
    from dxa.config.settings import SettingDictionary
    from dxa.engine.host import StreamingHost
    from dxa.engine.processor import Processor
    from dxa.io.sources import QueueSource
    from dxa.telemetry import appinsights as AI
    schema = tmp_path / "s.json"
    schema.write_text('{"type":"struct","fields":[{"name":"a","type":"long","nullable":true,"metadata":{}}]}')
    (tmp_path / "p.txt").write_text("Raw.*\n")
    (tmp_path / "t.txt").write_text("--DataXQuery--\nT = SELECT a, 1 / (a - 3) AS x FROM DataXProcessedInput\n")
    d = SettingDictionary({"datax.job.name": "aitest", "datax.job.input.default.blobschemafile": str(schema),
                           "datax.job.process.projection": str(tmp_path / "p.txt"),
                           "datax.job.process.transform": str(tmp_path / "t.txt"),
                           "datax.job.output.T.null.enabled": "true",
                           "DATAX_APPINSIGHTKEYREF": f"InstrumentationKey=00000000-1111;IngestionEndpoint={url}"})
    assert AI.configure(d) is not None
    proc = Processor(d, "cpu")
    src = QueueSource("cpu")
    src.push_many([b'{"a":1}', b'{"a":2}'])
    StreamingHost(proc, src, 0.001, max_batches=2, realtime=False, pipeline=False).run()
    AI.track_exception("ProcessDataFrame", "5 ms", ValueError("boom"))
    AI.shutdown()                                   # flushes the sender
    envs = [e for _path, batch in got for e in batch]
    assert all(p == "/v2/track" for p, _ in got)
    names = [e["data"]["baseData"].get("name") for e in envs if e["data"]["baseType"] == "EventData"]
    assert names.count("datax/streaming/batch/begin") == 2 and names.count("datax/streaming/batch/end") == 2
    assert "datax/error" in names
    ev = next(e for e in envs if e["data"]["baseType"] == "EventData")
    assert ev["iKey"] == "00000000-1111" and ev["name"] == "Microsoft.ApplicationInsights.000000001111.Event"
    props = ev["data"]["baseData"]["properties"]
    assert props["context.appname"] == "aitest" and props["batchTime"].endswith(" ms")
    exc = [e for e in envs if e["data"]["baseType"] == "ExceptionData"]
    assert exc and exc[0]["data"]["baseData"]["exceptions"][0]["typeName"] == "ValueError"
    assert exc[0]["data"]["baseData"]["properties"]["errorLocation"] == "ProcessDataFrame"
