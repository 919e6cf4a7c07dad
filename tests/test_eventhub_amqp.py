"""Event Hubs / IoT Hub direct AMQP input (EventHubStreamingFactory.scala:23-118, EventhubCheckpointer.scala:13-74)
against an in-process AMQP 1.0 fake (tests/amqp_fake.py)."""
import json
import time
import uuid

import pytest

from dxa.io import amqp as A
from dxa.io.eventhub import EARLIEST, LATEST, EventHubSource, build_eventhub_source, selector
from tests.amqp_fake import FakeEventHub


@pytest.fixture
def hub():
    h = FakeEventHub(partitions=2)
    yield h
    h.close()


def _decoded(raw):
    buf = raw.buf.cpu().numpy().tobytes()
    offs = raw.offs.cpu().tolist()
    return [buf[offs[i]:offs[i + 1]] for i in range(raw.n)]


def _wait_batch(src, bt, want, tries=20):
    got, raws = [], []
    for k in range(tries):
        raw = src.next_batch(bt + k)
        raws.append((bt + k, raw))
        got += _decoded(raw)
        if len(got) >= want:
            break
    return got, raws


def test_codec_roundtrip():
    vals = [None, True, False, A.UInt(0), A.UInt(7), A.UInt(70000), A.ULong(0), A.ULong(3), A.ULong(1 << 40), -5,
            1 << 40, 2.5, "héllo", "x" * 300, A.Symbol("sym"), b"\x00\x01", b"y" * 400, A.Timestamp(1700000000123),
            uuid.UUID(int=12345), [1, "a", None], {"k": 1, A.Symbol("s"): [2, 3]}, A.UShort(9), A.UByte(200),
            A.Described(A.ULong(0x70), [True])]
    for v in vals:
        enc = A.encode(v)
        dec, i = A.decode(enc)
        assert i == len(enc)
        assert dec == v and type(dec) is type(v) or (isinstance(v, tuple))


def test_codec_array():
    # array8 of smalluint: 0xe0 size count ctor values...
    enc = bytes([0xe0, 5, 3, 0x52, 1, 2, 3])
    dec, i = A.decode(enc)
    assert dec == [1, 2, 3] and i == len(enc)


def test_message_roundtrip():
    m = A.encode_message(b'{"a":1}', {"x-opt-sequence-number": 4}, {"p": "q"})
    d = A.decode_message(m)
    assert d["body"] == b'{"a":1}' and d["annotations"]["x-opt-sequence-number"] == 4 and d["app"] == {"p": "q"}


def test_connection_string():
    cs = A.parse_eventhub_connection("Endpoint=sb://ns.servicebus.windows.net/;SharedAccessKeyName=k;"
                                     "SharedAccessKey=v=;EntityPath=hub1")
    assert cs == {"host": "ns.servicebus.windows.net", "port": "5671", "tls": "1", "keyname": "k", "key": "v=",
                  "entity": "hub1"}
    with pytest.raises(A.AmqpError):
        A.parse_eventhub_connection("HostName=x;SharedAccessKey=y")


def test_selector_expressions():
    assert selector(12, LATEST) == "amqp.annotation.x-opt-sequence-number >= '12'"
    assert selector(None, EARLIEST) == "amqp.annotation.x-opt-offset > '-1'"
    assert selector(None, LATEST) == "amqp.annotation.x-opt-offset > '@latest'"
    assert selector(None, 1700000000000) == "amqp.annotation.x-opt-enqueued-time > '1700000000000'"


def test_sasl_rejects_bad_key(hub):
    with pytest.raises(A.AmqpError):
        A.AmqpConnection("127.0.0.1", hub.port, use_tls=False, username="RootManageSharedAccessKey",
                         password="wrong", timeout=5)


def test_management_partitions(hub):
    conn = A.AmqpConnection("127.0.0.1", hub.port, use_tls=False, username=hub.key_name, password=hub.key,
                            timeout=5)
    try:
        assert A.management_partitions(conn, "iot") == ["0", "1"]
    finally:
        conn.close()


def test_source_reads_from_start_with_properties(hub):
    for i in range(5):
        hub.send(i % 2, json.dumps({"i": i}).encode(), {"deviceKind": "t"})
    src = EventHubSource(hub.connection_string, "cpu", start=EARLIEST, rank=0, world=1, wait_s=0.3)
    try:
        got, raws = _wait_batch(src, 1_000_000, 5)
        assert sorted(json.loads(g)["i"] for g in got) == list(range(5))
        raw = next(r for _bt, r in raws if r.n)
        props = raw.properties.to_pylist()
        assert props[0] == {"deviceKind": "t"}
        sp = raw.system_properties.to_pylist()
        assert {"x-opt-sequence-number", "x-opt-offset", "x-opt-enqueued-time", "x-opt-partition-id"} <= set(sp[0])
    finally:
        src.close()


def test_source_latest_skips_existing_and_maxrate(hub):
    hub.send(0, b'{"old":1}')
    src = EventHubSource(hub.connection_string, "cpu", start=LATEST, max_rate=3, rank=0, world=1, wait_s=0.3)
    try:
        raw = src.next_batch(1)
        assert raw.n == 0
        assert src.pending == {}                   # nothing known yet → nothing to checkpoint
        src.commit(1)
        for i in range(8):
            hub.send(0, json.dumps({"n": i}).encode())
        time.sleep(0.2)
        raw = src.next_batch(2)
        assert 0 < raw.n <= 3                      # maxRatePerPartition
        got = [json.loads(g)["n"] for g in _decoded(raw)]
        assert got == list(range(raw.n))
    finally:
        src.close()


def test_checkpoint_restore_and_flush(hub, tmp_path):
    for i in range(6):
        hub.send(0, json.dumps({"n": i}).encode())
        hub.send(1, json.dumps({"n": 100 + i}).encode())
    ck = str(tmp_path / "ck")
    src = EventHubSource(hub.connection_string, "cpu", start=EARLIEST, max_rate=4, checkpoint_dir=ck, rank=0,
                         world=1, wait_s=0.3)
    try:
        got, raws = _wait_batch(src, 5_000_000, 8)
        for bt, _r in raws:
            src.commit(bt)
    finally:
        src.close()
    lines = open(tmp_path / "ck" / "offsets.txt").read().split()
    last = {ln.split(",")[2]: int(ln.split(",")[4]) for ln in lines}
    assert last == {"0": 4, "1": 4}
    # restart: continue at the committed sequence numbers (at-least-once, no gap)
    src = EventHubSource(hub.connection_string, "cpu", start=EARLIEST, checkpoint_dir=ck, rank=0, world=1,
                         wait_s=0.3)
    try:
        got, _ = _wait_batch(src, 6_000_000, 4)
        assert sorted(json.loads(g)["n"] for g in got) == [4, 5, 104, 105]
    finally:
        src.close()
    # flushexistingcheckpoints: the checkpoint is ignored → starts from `start`
    src = EventHubSource(hub.connection_string, "cpu", start=EARLIEST, checkpoint_dir=ck, flush_existing=True,
                         rank=0, world=1, wait_s=0.3)
    try:
        got, _ = _wait_batch(src, 7_000_000, 12)
        assert len(got) == 12
    finally:
        src.close()


def test_start_enqueue_time(hub):
    for i in range(4):
        hub.send(0, json.dumps({"n": i}).encode(), enqueued_ms=1_000 * (i + 1))
    src = EventHubSource(hub.connection_string, "cpu", start=2_500, rank=0, world=1, wait_s=0.3)
    try:
        got, _ = _wait_batch(src, 1, 2)
        assert [json.loads(g)["n"] for g in got] == [2, 3]
    finally:
        src.close()


def test_partitions_split_over_ranks(hub):
    hub.send(0, b'{"p":0}')
    hub.send(1, b'{"p":1}')
    seen = []
    for r in range(2):
        src = EventHubSource(hub.connection_string, "cpu", start=EARLIEST, rank=r, world=2, wait_s=0.3)
        try:
            assert src.parts == [str(r)]
            got, _ = _wait_batch(src, 1, 1)
            seen += [json.loads(g)["p"] for g in got]
        finally:
            src.close()
    assert sorted(seen) == [0, 1]


def test_build_source_eventhub_kind(hub, tmp_path):
    from dxa.config.settings import SettingDictionary
    from dxa.io.sources import build_source
    hub.send(1, b'{"v":1}')
    d = SettingDictionary({
        "datax.job.input.default.eventhub.connectionstring": hub.connection_string,
        "datax.job.input.default.eventhub.consumergroup": "$Default",
        "datax.job.input.default.eventhub.checkpointdir": str(tmp_path / "ck"),
        "datax.job.input.default.eventhub.startenqueuetime": "0",
        "datax.job.input.default.eventhub.maxrate": "100",
        "datax.job.input.default.blobschemafile": json.dumps({"type": "struct", "fields": [
            {"name": "v", "type": "long", "nullable": True, "metadata": {}}]}),
    })
    src = build_source(d, "cpu")
    try:
        assert isinstance(src, EventHubSource)
        got, _ = _wait_batch(src, 1, 1)
        assert got == [b'{"v":1}']
    finally:
        src.close()


def test_sampler_eventhub_amqp(hub):
    import threading
    from dxa.service import sampler as S

    def later():
        time.sleep(0.6)
        hub.send(0, b'{"s":1}', {"a": "b"})
    threading.Thread(target=later, daemon=True).start()
    out = S.sample_input({"inputType": "iothub", "inputMode": "streaming",
                          "eventhubConnectionString": hub.connection_string, "eventhubNames": "iot",
                          "seconds": 2})
    assert [json.loads(o["Raw"]) for o in out] == [{"s": 1}]
    assert out[0]["Properties"] == {"a": "b"} and out[0]["SystemProperties"]["x-opt-partition-id"] == "0"
