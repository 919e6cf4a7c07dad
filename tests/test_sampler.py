"""Sampling the configured input for schema inference / LiveQuery (SchemaInferenceManager.cs:33-143,
KafkaMessageBus.cs:80-190, BlobMessageBus.cs:30-60) against the in-process Kafka broker and local blob folders."""
import json
import os
import threading
import time

import pytest

from dxa.service import sampler as S
from tests.kafka_fake import FakeBroker


@pytest.fixture()
def broker():
    b = FakeBroker(["iot"], partitions=2)
    yield b
    b.close()


def _produce_later(port, delay=0.4):
    from dxa.io import kafka as K

    def go():
        time.sleep(delay)
        c = K.KafkaClient(f"127.0.0.1:{port}")
        for p in range(2):
            c.produce("iot", p, [json.dumps({"deviceId": p * 10 + i, "temp": 20.5 + i,
                                             "loc": {"lat": 1.5, "home": "h"}}).encode() for i in range(5)])
    t = threading.Thread(target=go)
    t.start()
    return t


def test_kafka_sampling_starts_at_the_end(broker):
    from dxa.io import kafka as K
    c = K.KafkaClient(f"127.0.0.1:{broker.port}")
    c.produce("iot", 0, [b'{"old": 1}'])                   # before the sample window: not sampled (Latest)
    t = _produce_later(broker.port)
    evs = S.sample_kafka(f"127.0.0.1:{broker.port}", ["iot"], 1.5)
    t.join()
    assert len(evs) == 10 and all("old" not in e["Raw"] for e in evs)
    sp = evs[0]["SystemProperties"]
    assert sp["Topic"] == "iot" and sp["Partition"] in ("0", "1") and int(sp["UnixTimestampMs"]) > 0


def test_inferschema_route_samples_kafka_and_saves(broker, tmp_path, monkeypatch):
    from fastapi.testclient import TestClient
    from dxa.service.app import create_app
    monkeypatch.setenv("DXA_SUPERVISE", "0")
    app = create_app(str(tmp_path / "svc"))
    client = TestClient(app)
    t = _produce_later(broker.port)
    r = client.post("/api/inputdata/inferschema", json={
        "name": "flow1", "userName": "ann", "inputType": "kafka", "inputMode": "streaming",
        "eventhubConnectionString": f"127.0.0.1:{broker.port}", "eventhubNames": "iot", "seconds": 2}).json()
    t.join()
    assert not r["error"], r
    schema = json.loads(r["result"]["Schema"]) if isinstance(r["result"].get("Schema"), str) else r["result"]
    text = json.dumps(schema)
    assert "deviceId" in text and "temp" in text and "lat" in text
    files = os.listdir(tmp_path / "svc" / "samples")
    assert len(files) == 1 and files[0].startswith("flow1-")
    lines = (tmp_path / "svc" / "samples" / files[0]).read_bytes().decode().split("\r\n")
    assert len([l for l in lines if l]) == 10 and json.loads(lines[0])["Raw"].startswith("{")
    assert len(app.state.dxa.samples["flow1"]) == 10


def test_blob_sampling_newest_documents(tmp_path):
    old = tmp_path / "in" / "2020" / "01" / "a.json"
    new = tmp_path / "in" / "2020" / "02" / "b.json"
    for p, tag in ((old, "old"), (new, "new")):
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text("\n".join(json.dumps({"tag": tag, "i": i}) for i in range(300)) + "\n")
    os.utime(old, (1, 1))
    evs = S.sample_input({"inputMode": "batching",
                          "batchInputs": [{"properties": {"path": str(tmp_path / "in" / "{yyyy}" / "{MM}")}}]})
    assert len(evs) == S.MAX_BLOB_DOCS
    assert all(json.loads(e["Raw"])["tag"] == "new" for e in evs[:300])
    assert evs[0]["Properties"]["Length"] == str(len(evs[0]["Raw"]))


def test_unknown_input_type_is_an_error():
    with pytest.raises(S.SampleError):
        S.sample_input({"inputType": "carrierpigeon"})
