"""Sampling a flow's configured input for schema inference and LiveQuery (the reference's IMessageBus
implementations: Services/DataX.Flow/DataX.Flow.SchemaInference/SchemaGenerator.cs:19-157,
Kafka/KafkaMessageBus.cs:80-190, Eventhub/EventhubMessageBus.cs, Blob/BlobMessageBus.cs).

* ``kafka`` / ``kafkaeventhub`` / ``events`` / ``iothub`` inputs: a consumer over the in-tree Kafka client (Event Hubs
  and IoT Hub through their Kafka endpoint, SASL PLAIN with ``$ConnectionString``) that starts at the END of every
  partition (AutoOffsetReset.Latest, KafkaMessageBus.cs:88) and collects what arrives during ``seconds``;
* ``batching`` inputs: the most recently modified blobs under each batch input's path, up to 500 documents
  (BlobMessageBus.cs:30-60);
* ``local``: events rendered by the schema-driven generator.

Each sampled event becomes an ``EventRaw`` (``{"Raw", "Properties", "SystemProperties"}`` with the reference's
Topic / Partition / Offset / UtcDateTime / UnixTimestampMs system properties); the sample file is the events' JSON
joined by CRLF (``EventsData.EventsJson``), saved as ``<samples>/<flowId>-<hash(user)>.json``.
"""
from __future__ import annotations

import datetime as _dt
import hashlib
import json
import os
import time
from typing import Any, Dict, List, Optional, Tuple

DEFAULT_SECONDS = 30
MAX_BLOB_DOCS = 500


class SampleError(Exception):
    pass


def _event_raw(raw: str, props: Dict[str, str], sysprops: Dict[str, str]) -> Dict[str, Any]:
    return {"Raw": raw, "Properties": props, "SystemProperties": sysprops}


def sample_kafka(servers: str, topics: List[str], seconds: float, sasl=None, use_ssl: bool = False,
                 max_events: int = 100_000, poll_s: float = 0.2) -> List[Dict[str, Any]]:
    """Events produced to ``topics`` during the next ``seconds`` (consumer starts at each partition's end)."""
    from ..io import kafka as K
    client = K.KafkaClient(servers, use_ssl=use_ssl, sasl=sasl)
    try:
        meta = client.metadata(topics)
        pos = {(t, p): client.list_offset(t, p, K.LATEST) for t in topics for p in meta.get(t, [])}
        out: List[Dict[str, Any]] = []
        deadline = time.monotonic() + seconds
        while time.monotonic() < deadline and len(out) < max_events:
            got_any = False
            for (t, p), cur in list(pos.items()):
                recs, _hw = client.fetch(t, p, cur, max_wait_ms=int(poll_s * 1000))
                if not recs:
                    continue
                vals, offs, recoffs, nxt = K.decode_records(recs, cur, pad=0)
                for i in range(len(recoffs)):
                    raw = bytes(vals[offs[i]:offs[i + 1]]).decode("utf-8", "replace")
                    off = int(recoffs[i])
                    now = time.time()
                    out.append(_event_raw(raw, {"HeadersCount": "0"}, {
                        "Topic": t, "Partition": str(p), "Offset": str(off),
                        "UtcDateTime": _dt.datetime.utcfromtimestamp(now).strftime("%m/%d/%Y %I:%M:%S %p"),
                        "UnixTimestampMs": str(int(now * 1000))}))
                    got_any = True
                pos[(t, p)] = max(cur, nxt)
            if not got_any:
                time.sleep(poll_s)
        return out
    finally:
        client.close()


def sample_eventhub_amqp(conn: str, hub: Optional[str], seconds: float,
                         max_events: int = 100_000) -> List[Dict[str, Any]]:
    """Events arriving on every partition of the hub during ``seconds`` (AMQP receiver at the end of the stream)."""
    from ..io.eventhub import LATEST, EventHubSource
    src = EventHubSource(conn, "cpu", start=LATEST, rank=0, world=1, hub=hub, wait_s=0.2)
    out: List[Dict[str, Any]] = []
    try:
        deadline = time.monotonic() + seconds
        while time.monotonic() < deadline and len(out) < max_events:
            src.conn.pump(min(0.2, max(0.01, deadline - time.monotonic())))
            for p, link in src.links.items():
                for m in link.drain():
                    ann = {str(k): str(v) for k, v in m["annotations"].items()}
                    out.append(_event_raw(m["body"].decode("utf-8", "replace"),
                                          {str(k): str(v) for k, v in (m["app"] or {}).items()},
                                          dict(ann, **{"x-opt-partition-id": p})))
        return out
    finally:
        src.close()


def sample_blobs(paths: List[str], max_docs: int = MAX_BLOB_DOCS) -> List[Dict[str, Any]]:
    """The newest documents (lines of the most recently modified files) under each batch input path; ``{…}`` date
    tokens in a path match any folder name."""
    import re
    from ..io import fs
    out: List[Dict[str, Any]] = []
    for path in paths:
        pattern = re.sub(r"\{[^}]*\}", "*", path)       # a batch path names folders: every file below them
        files = fs.list_matching(pattern.rstrip("/") + "/**") if "*" in pattern else fs.list_matching(pattern)

        def mtime(f):
            try:
                return os.path.getmtime(f)
            except OSError:
                return 0.0
        files.sort(key=mtime, reverse=True)
        docs: List[str] = []
        for f in files:
            for line in fs.read_text(f).splitlines():
                if line.strip():
                    docs.append(line)
                    if len(docs) >= max_docs:
                        break
            if len(docs) >= max_docs:
                break
        for d in docs:
            n = str(len(d))
            out.append(_event_raw(d, {"Length": n}, {"Length": n}))
    return out


def sample_local(schema_json: str, n: int = 100) -> List[Dict[str, Any]]:
    from ..engine.types import schema_from_json
    from ..simulate.datagen import compile_spark, render_cpu
    prog = compile_spark(schema_from_json(schema_json))
    base = int(time.time() * 1000)
    return [_event_raw(render_cpu(prog, i, 1, base, 0).decode(), {}, {}) for i in range(n)]


def sample_input(q: Dict[str, Any], seconds: Optional[int] = None) -> List[Dict[str, Any]]:
    """An InteractiveQueryObject (``inputType``, ``inputMode``, ``eventhubConnectionString``, ``eventhubNames``,
    ``batchInputs``, ``inputSchema``, ``seconds``) → sampled EventRaw dicts."""
    from ..config.secrets import resolve
    from ..io import kafka as K
    secs = seconds if seconds is not None else int(q.get("seconds") or 0)
    secs = secs if secs > 0 else DEFAULT_SECONDS
    mode = (q.get("inputMode") or "streaming").lower()
    kind = (q.get("inputType") or "").lower()
    if mode == "batching":
        paths = []
        for b in q.get("batchInputs") or []:
            props = b.get("properties") or b
            if props.get("path"):
                paths.append(resolve(props["path"]))
        return sample_blobs(paths)
    if kind in ("kafka", "kafkaeventhub", "events", "eventhub", "iothub"):
        conn = resolve(q.get("eventhubConnectionString") or "")
        names = [t.strip() for t in (q.get("eventhubNames") or "").split(",") if t.strip()]
        if kind == "kafka":
            return sample_kafka(conn, names, secs)
        if kind in ("events", "eventhub", "iothub"):          # EventhubMessageBus: AMQP from the end
            return sample_eventhub_amqp(conn, names[0] if names else None, secs)
        es = K.eventhub_kafka_settings(conn)
        topics = [es["topic"]] if es.get("topic") else names
        return sample_kafka(es["bootstrap"], topics, secs, sasl=es["sasl"], use_ssl=True)
    if kind == "local":
        if not q.get("inputSchema"):
            raise SampleError("local input: no inputSchema to generate sample events from")
        return sample_local(q["inputSchema"] if isinstance(q["inputSchema"], str) else json.dumps(q["inputSchema"]))
    raise SampleError(f"cannot sample input type '{kind}'")


def events_json(events: List[Dict[str, Any]]) -> str:
    """``EventsData.EventsJson``: each EventRaw serialised, CRLF-terminated."""
    return "".join(json.dumps(e) + "\r\n" for e in events)


def save_sample(root: str, flow_id: str, user: str, events: List[Dict[str, Any]]) -> str:
    """``<root>/<flowId>-<hash(user)>.json`` (SchemaGenerator.SaveSample)."""
    from ..io import fs
    h = hashlib.sha256((user or "").encode()).hexdigest()[:16]
    path = os.path.join(root, f"{flow_id}-{h}.json")
    fs.write_atomic(path, events_json(events))
    return path
