"""Kafka protocol client, native record-batch codec, Kafka source (rank partition assignment, max rate, offsets
checkpoint + restore) and the simulated producer — against the in-process fake broker."""
import json
import os

import pytest
import torch

from dxa.io import kafka as K
from tests.kafka_fake import FakeBroker


def test_crc32c_known_vector():
    assert K.crc32c(b"123456789") == 0xE3069283


def test_batch_roundtrip():
    vals = [b'{"a":1}', b"", b'{"b":"xyz"}'] + [b"x" * 300]
    batch = K.encode_batch(vals, timestamp_ms=1)
    buf, offs, recoffs, nxt = K.decode_records(batch, 0)
    got = [bytes(buf[offs[i]:offs[i + 1]]) for i in range(len(vals))]
    assert got == vals and recoffs.tolist() == [0, 1, 2, 3] and nxt == 4
    assert (buf[int(offs[-1]):] == 0).all() and len(buf) == int(offs[-1]) + 16
    # records below the fetch offset are dropped; a truncated trailing batch is ignored
    buf, offs, recoffs, nxt = K.decode_records(batch + batch[:30], 2)
    assert recoffs.tolist() == [2, 3]
    bad = bytearray(batch)
    bad[-1] ^= 0xFF
    with pytest.raises(K.KafkaError):
        K.decode_records(bytes(bad), 0)


@pytest.fixture()
def broker():
    b = FakeBroker(["iot"], partitions=3)
    yield b
    b.close()


def _produce(broker, n_per_part):
    c = K.KafkaClient(f"127.0.0.1:{broker.port}")
    for p in range(3):
        for chunk in range(2):
            c.produce("iot", p, [json.dumps({"p": p, "i": chunk * 1000 + i}).encode()
                                 for i in range(n_per_part // 2)])
    return c


def test_client_metadata_offsets_fetch(broker):
    c = _produce(broker, 10)
    assert c.metadata(["iot"]) == {"iot": [0, 1, 2]}
    assert c.list_offset("iot", 1, K.EARLIEST) == 0 and c.list_offset("iot", 1, K.LATEST) == 10
    recs, hw = c.fetch("iot", 2, 7)
    _, offs, recoffs, nxt = K.decode_records(recs, 7)
    assert hw == 10 and recoffs.tolist() == [7, 8, 9] and nxt == 10


def test_kafka_source_batches_checkpoint_restore(broker, tmp_path):
    from dxa.ops.jsonparse import ParsePlan, parse
    from dxa.engine.types import StructField, StructType
    _produce(broker, 10)
    ck = str(tmp_path / "ck")
    src = K.KafkaSource(K.KafkaClient(f"127.0.0.1:{broker.port}"), ["iot"], "cpu", ck, max_rate=4)
    raw = src.next_batch(1_000_000)
    assert raw.n == 12                                            # 3 partitions x max_rate 4
    col, ok = parse(raw.buf, raw.offs, ParsePlan(StructType((StructField("p", "long"), StructField("i", "long")))))
    assert sorted(col.child("p").data.tolist()) == [0] * 4 + [1] * 4 + [2] * 4
    # the read cursor runs ahead of the commits (prefetch): the next batch is the next 4 per partition
    raw2 = src.next_batch(2_000_000)
    assert raw2.n == 12
    col2, _ = parse(raw2.buf, raw2.offs, ParsePlan(StructType((StructField("p", "long"), StructField("i", "long")))))
    assert sorted(col2.child("i").data.tolist()) == sorted([4, 1000, 1001, 1002] * 3)
    src.commit(1_000_000)
    lines = open(os.path.join(ck, "offsets.txt")).read().splitlines()
    assert sorted(lines) == ["1000,iot,0,0,4", "1000,iot,1,0,4", "1000,iot,2,0,4"]
    src.commit(2_000_000)
    lines = open(os.path.join(ck, "offsets.txt")).read().splitlines()
    assert sorted(lines) == ["2000,iot,0,4,8", "2000,iot,1,4,8", "2000,iot,2,4,8"]
    assert src.next_batch(3_000_000).n == 6                       # 10 - 8 = 2 left per partition; not committed
    # a restarted source resumes from the checkpoint: batch 3 was never committed, so it is read again
    src2 = K.KafkaSource(K.KafkaClient(f"127.0.0.1:{broker.port}"), ["iot"], "cpu", ck, max_rate=4)
    assert src2.next_batch(4_000_000).n == 6
    src2.commit(4_000_000)
    assert src2.next_batch(5_000_000).n == 0
    src2.commit(5_000_000)
    assert sorted(open(os.path.join(ck, "offsets.txt")).read().splitlines()) == [
        "5000,iot,0,10,10", "5000,iot,1,10,10", "5000,iot,2,10,10"]


class _DeferredProcessor:
    """Stub processor with pipelined outputs: batch t's completion callback fires while batch t+1 is processed."""

    def __init__(self):
        self.on_batch_complete = None
        self.seen = []
        self._pending = None

    def process_batch(self, raw, bt, interval_us, when=None):
        from dxa.ops.jsonparse import ParsePlan, parse
        from dxa.engine.types import StructField, StructType
        if raw.n:
            col, _ = parse(raw.buf, raw.offs, ParsePlan(StructType((StructField("p", "long"),
                                                                    StructField("i", "long")))))
            self.seen += list(zip(col.child("p").data.tolist(), col.child("i").data.tolist()))
        if self._pending is not None:
            self.on_batch_complete(*self._pending)
        self._pending = (bt, {"n": float(raw.n)})
        return {}

    def drain(self):
        if self._pending is not None:
            self.on_batch_complete(*self._pending)
            self._pending = None


def test_pipelined_host_delivers_every_kafka_record_once(broker, tmp_path):
    from dxa.engine.host import StreamingHost
    _produce(broker, 8)
    ck = str(tmp_path / "ck")
    src = K.KafkaSource(K.KafkaClient(f"127.0.0.1:{broker.port}"), ["iot"], "cpu", ck, max_rate=3)
    proc = _DeferredProcessor()
    host = StreamingHost(proc, src, interval_s=1.0, max_batches=4, realtime=False, pipeline=True)
    host.run()
    expected = sorted((p, c * 1000 + i) for p in range(3) for c in range(2) for i in range(4))
    assert sorted(proc.seen) == expected                          # 24 records, none twice, none skipped
    assert [m["n"] for m in host.history] == [9.0, 9.0, 6.0, 0.0]
    # the checkpoint holds the last committed batch's own ranges, and a restart has nothing left to read
    last = sorted(open(os.path.join(ck, "offsets.txt")).read().splitlines())
    assert [ln.split(",")[1:] for ln in last] == [["iot", str(p), "8", "8"] for p in range(3)]
    src2 = K.KafkaSource(K.KafkaClient(f"127.0.0.1:{broker.port}"), ["iot"], "cpu", ck, max_rate=3)
    assert src2.next_batch(0).n == 0


def test_rank_partition_assignment(broker):
    _produce(broker, 4)
    a = K.KafkaSource(K.KafkaClient(f"127.0.0.1:{broker.port}"), ["iot"], "cpu", rank=0, world=2)
    b = K.KafkaSource(K.KafkaClient(f"127.0.0.1:{broker.port}"), ["iot"], "cpu", rank=1, world=2)
    assert a.parts == [("iot", 0), ("iot", 2)] and b.parts == [("iot", 1)]
    assert a.next_batch(0).n + b.next_batch(0).n == 12


def test_sasl_plain_and_eventhub_settings():
    b = FakeBroker(["hub"], partitions=1, sasl_password="Endpoint=sb://x/;EntityPath=hub")
    try:
        c = K.KafkaClient(f"127.0.0.1:{b.port}", sasl=("$ConnectionString", "Endpoint=sb://x/;EntityPath=hub"))
        assert c.metadata(["hub"]) == {"hub": [0]}
        with pytest.raises(K.KafkaError):
            K.KafkaClient(f"127.0.0.1:{b.port}", sasl=("$ConnectionString", "wrong")).metadata(["hub"])
    finally:
        b.close()
    es = K.eventhub_kafka_settings("Endpoint=sb://myns.servicebus.windows.net/;SharedAccessKeyName=k;"
                                   "SharedAccessKey=s;EntityPath=telemetry")
    assert es["bootstrap"] == "myns.servicebus.windows.net:9093" and es["topic"] == "telemetry"
    assert es["sasl"][0] == "$ConnectionString" and es["use_ssl"]


def test_simulated_producer(broker):
    from dxa.simulate.kafka_producer import program_from_schema_text, run
    schema = json.dumps({"type": "struct", "fields": [
        {"name": "v", "type": "double", "nullable": False, "metadata": {"minValue": 1.0, "maxValue": 2.0}}]})
    c = K.KafkaClient(f"127.0.0.1:{broker.port}")
    sent = run(c, ["iot"], program_from_schema_text(schema), rate=5, seconds=0.01)
    assert sent == 5
    total = sum(c.list_offset("iot", p, K.LATEST) for p in range(3))
    assert total == 5


def test_build_source_from_settings(broker, tmp_path):
    from dxa.config.settings import SettingDictionary
    from dxa.io.sources import build_source
    _produce(broker, 2)
    d = SettingDictionary({"datax.job.input.default.kafka.bootstrapservers": f"127.0.0.1:{broker.port}",
                           "datax.job.input.default.kafka.topics": "iot",
                           "datax.job.input.default.kafka.checkpointdir": str(tmp_path / "k")})
    src = build_source(d, "cpu")                  # auto.offset.reset defaults to latest, as the reference
    assert isinstance(src, K.KafkaSource) and src.next_batch(0).n == 0
    d = SettingDictionary(dict(d.dict, **{"datax.job.input.default.kafka.autooffsetreset": "earliest",
                                          "datax.job.input.default.kafka.checkpointdir": str(tmp_path / "k2")}))
    assert build_source(d, "cpu").next_batch(0).n == 6


@pytest.mark.gpu
@pytest.mark.parametrize("compression", ["lz4", "none"])
def test_kafka_source_device_decode_matches_host(broker, tmp_path, compression):
    """The GPU ingest (batch headers planned on the host, records decompressed and framed on the device, values
    parsed in place) delivers the same records and commit ranges as the host decoder."""
    import torch
    from dxa.engine.types import StructField, StructType
    from dxa.ops.jsonparse import ParsePlan, parse
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = K.KafkaClient(f"127.0.0.1:{broker.port}")
    for p in range(3):
        for chunk in range(3):
            c.produce("iot", p, [json.dumps({"p": p, "i": chunk * 1000 + i}).encode() for i in range(50)],
                      compression=compression)
    schema = StructType((StructField("p", "long"), StructField("i", "long")))
    got = {}
    for mode in ("device", "host"):
        src = K.KafkaSource(K.KafkaClient(f"127.0.0.1:{broker.port}"), ["iot"], "cuda:0", str(tmp_path / mode),
                            max_rate=70, device_decode=(mode == "device"),
                            check_crcs="device" if mode == "device" else "host")
        rows = []
        for bt in (1, 2, 3):
            raw = src.next_batch(bt * 1_000_000)
            assert (raw.ends is not None) == (mode == "device")
            col, ok = parse(raw.buf, raw.offs, ParsePlan(schema), raw.ends)
            assert bool(ok.all())
            rows.append(sorted(zip(col.child("p").data.tolist(), col.child("i").data.tolist())))
            src.commit(bt * 1_000_000)
        src.check() if mode == "device" else None
        got[mode] = (rows, sorted(open(os.path.join(tmp_path / mode, "offsets.txt")).read().splitlines()))
    assert got["device"] == got["host"]
    assert [len(r) for r in got["device"][0]] == [210, 210, 30]


@pytest.mark.gpu
def test_kafka_device_batches_survive_next_decode(broker, tmp_path):
    """A batch's device buffers are recorded on the consumer stream: work queued on it behind a long kernel still
    reads batch 1's bytes after the batch is dropped and batch 2 decodes (the caching allocator must not hand batch
    1's memory to batch 2's decode stream)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = K.KafkaClient(f"127.0.0.1:{broker.port}")
    for p in range(3):
        c.produce("iot", p, [json.dumps({"p": p, "i": i, "pad": "x" * (i % 50)}).encode() for i in range(400)],
                  compression="lz4")
    src = K.KafkaSource(K.KafkaClient(f"127.0.0.1:{broker.port}"), ["iot"], "cuda:0", max_rate=200,
                        device_decode=True)
    raw1 = src.next_batch(1_000_000)
    torch.cuda.synchronize()
    want = raw1.buf.cpu().clone()
    torch.cuda._sleep(200_000_000)                 # the consumer stream is busy for a while ...
    late = raw1.buf.clone()                        # ... so this copy of batch 1 runs after batch 2's decode
    del raw1
    raw2 = src.next_batch(2_000_000)
    torch.cuda.synchronize()
    assert torch.equal(late.cpu(), want)
    assert raw2.n == 600
    src.verify(1_000_000)
    src.verify(2_000_000)


@pytest.mark.gpu
def test_kafka_device_decode_failure_is_reported(broker):
    """A corrupt LZ4 block that passes the host plan fails on the device; ``verify`` (called by the streaming host
    before commit) raises instead of committing malformed rows."""
    import torch
    from dxa.io import kafka_device as KD
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    vals = [json.dumps({"i": i, "s": "abc" * 20}).encode() for i in range(200)]
    rs = bytearray(K.encode_batch(vals, 1, "lz4", level=9))
    plan = KD.plan_fetch(bytes(rs), 0, verify_crc=False)
    # point the first block's first match far before the output start: the decoder must flag it
    off = int(plan.k_comp_off[0])
    stored = bool(plan.k_stored[0])
    if stored:
        pytest.skip("first block stored uncompressed")
    tok = rs[off]
    lit = tok >> 4
    p = off + 1
    if lit == 15:
        while rs[p] == 255:
            p += 1
        lit += rs[p]
        p += 1
    p += lit
    rs[p:p + 2] = (0xFFFF).to_bytes(2, "little")
    staging = torch.zeros(len(rs) + 64, dtype=torch.uint8).pin_memory()
    staging[:len(rs)] = torch.frombuffer(bytearray(rs), dtype=torch.uint8)
    dec = KD.DeviceRecordDecoder(torch.device("cuda:0"))
    raw, ev = dec.decode(staging, plan)
    torch.cuda.current_stream().wait_event(ev)
    assert raw.status.failed() > 0
    with pytest.raises(KD.DecodeError):
        dec.check()


def test_start_position_from_enqueue_time(broker):
    """startenqueuetime (EventHubStreamingFactory.scala:47-64): 0 → start, >0 → epoch seconds, <0 → now-relative,
    unset → autooffsetreset (latest by default); resolved with ListOffsets by timestamp."""
    assert K.start_position("0") == K.EARLIEST and K.start_position(None) == K.LATEST
    assert K.start_position(None, "earliest") == K.EARLIEST
    assert K.start_position("1700000000") == 1_700_000_000_000
    assert K.start_position("-60", now_ms=10_000_000) == 10_000_000 - 60_000
    c = K.KafkaClient(f"127.0.0.1:{broker.port}")
    for k, ts in enumerate((1_000_000, 2_000_000, 3_000_000)):
        c.produce("iot", 0, [json.dumps({"k": k, "i": i}).encode() for i in range(5)], timestamp_ms=ts)
    assert c.list_offset("iot", 0, 2_000_000) == 5
    assert c.list_offset("iot", 0, 2_500_000) == 10
    assert c.list_offset("iot", 0, 9_000_000) == 15            # past the end: the log end
    src = K.KafkaSource(K.KafkaClient(f"127.0.0.1:{broker.port}"), ["iot"], "cpu", start=K.start_position("2000"))
    assert src.fetch_pos[("iot", 0)] == 5 and src.next_batch(0).n == 10


def test_records_per_batch_follows_the_producer_estimator():
    """batch.size bounds a batch's estimated *compressed* size (MemoryRecordsBuilder.hasRoomFor): with LZ4 on
    SimulatedData JSON (~3.3x) a 16 KiB batch holds ~84 records, not 16 KiB / 608 B = 26."""
    from dxa.io import kafka as K
    from dxa.models import iot
    from dxa.simulate.datagen import generate
    buf, offs = generate(iot.program(), 20000, torch.device("cpu"), seed=3, row0=0, base_ms=1_700_000_000_000)
    per, ratio = K.records_per_batch(buf.numpy(), offs.numpy(), sample=8000)
    avg = float(offs[-1]) / 20000
    assert 0.25 < ratio < 0.4
    # the fixed point: the estimated compressed batch fills batch.size
    assert abs(per * avg * ratio * 1.05 - K.KAFKA_BATCH_SIZE) < avg * ratio * 1.05 * 2
    per_none, ratio_none = K.records_per_batch(buf.numpy(), offs.numpy(), compression="none", sample=8000)
    assert ratio_none > 1.0 and per_none < 27
