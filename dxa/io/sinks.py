"""Output operators: ``datax.job.output.<name>.<sink>.*`` → sink writers with the reference's metric names.

Reference: DataProcessing/datax-host/src/main/scala/datax/sink/OutputManager.scala:22-160 (operators, per-sink flag
columns, ``to_json(struct(*))``, ``Sink_InputEvents`` / ``Sink_<S>_All|Filtered`` metrics), BlobSinker.scala:30-226
(folder templating with ``%1$tY``… / ``${quarterBucket}`` / ``${minuteBucket}`` / ``${target}``, gzip by default),
EventHubStreamPoster.scala (200-event chunks, newline-joined), HttpPoster.scala (200-event JSON arrays),
CosmosDBSinker.scala, SqlSinker.scala.

Cloud targets are real clients (Blob / Event Hubs / Cosmos DB REST, SQL Server over TDS — ``dxa.io.tds``).  The
single-node stand-ins are opt-in only: blob → local/mounted folder; eventhub → a local spool folder per hub;
cosmosdb ``local:`` → JSON document folder per database/collection; sql ``sqlite:///path`` or ``local:`` → SQLite;
plus ``file``, ``console``, ``memory`` and ``null``.  A connection string that is neither fails at job start.
"""
from __future__ import annotations

import datetime as _dt
import gzip
import json
import os
import re
import threading
import time
import uuid
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from ..config.secrets import resolve
from ..engine.column import Table
from ..engine.serialize import table_to_json_lines
from . import fs

SINK_PREFIX = "Sink_"
_pool = ThreadPoolExecutor(max_workers=8, thread_name_prefix="dxa-output")       # one task per output
_sink_pool = ThreadPoolExecutor(max_workers=8, thread_name_prefix="dxa-sink")    # per-sink fan-out inside one


def java_time_format(fmt: str, ts: _dt.datetime) -> str:
    """Subset of ``String.format(fmt, timestamp)`` used in DataX folder templates (``%1$tY/%1$tm/%1$td/%1$tH``…)."""
    table = {"Y": f"{ts.year:04d}", "m": f"{ts.month:02d}", "d": f"{ts.day:02d}", "H": f"{ts.hour:02d}",
             "M": f"{ts.minute:02d}", "S": f"{ts.second:02d}", "y": f"{ts.year % 100:02d}", "j": f"{ts.timetuple().tm_yday:03d}",
             "L": f"{ts.microsecond // 1000:03d}", "e": str(ts.day), "k": str(ts.hour)}
    return re.sub(r"%(?:1\$)?t([A-Za-z])", lambda m: table.get(m.group(1), m.group(0)), fmt)


def blob_folder(fmt: Optional[str], ts: _dt.datetime, target: Optional[str] = None) -> Optional[str]:
    if not fmt:
        return None
    quarter = ["00", "15", "30", "45"][min(3, round(ts.minute / 15))]
    minute_bucket = ts.strftime("%H%M%S")
    out = java_time_format(fmt, ts)
    out = out.replace("${quarterBucket}", quarter).replace("${minuteBucket}", minute_bucket)
    out = out.replace("${target}", target or "UNKNOWN")
    return out.rstrip("/") + "/"


_eh_senders: Dict[str, object] = {}


def eventhub_send(conn: str, payload: bytes, hub: str = "default", properties: Optional[Dict[str, str]] = None):
    """Send one event: an Event Hubs connection string (``Endpoint=sb://…;SharedAccessKey…``) → REST send
    (``io/azure.EventHubSender``, the reference's EventHubSenderPool); ``http(s)://`` → POST; anything else → spool
    file under DXA_FS_ROOT."""
    from . import azure
    if azure.is_eventhub_connection(conn):
        sender = _eh_senders.get(conn)
        if sender is None:
            sender = _eh_senders.setdefault(conn, azure.EventHubSender(conn, hub))
        sender.send(payload, properties)
        return
    if conn.startswith("http://") or conn.startswith("https://"):
        import urllib.request
        urllib.request.urlopen(urllib.request.Request(conn, data=payload, method="POST"), timeout=5).read()
        return
    m = re.search(r"EntityPath=([^;]+)", conn)
    name = m.group(1) if m else hub
    root = os.environ.get("DXA_FS_ROOT", ".dxa_fs")
    path = os.path.join(root, "eventhub", name, f"{int(time.time() * 1000)}-{uuid.uuid4().hex[:8]}.bin")
    fs.write_atomic(path, payload)


@dataclass
class Sink:
    name: str                                  # metric name component, e.g. "Blobs"
    write: Callable[[List[str], Table, _dt.datetime, str], int]
    filter_expr: Optional[str] = None
    as_json: bool = True
    # grouped sinks (blob): rows are split by the string value of ``group_expr`` (a single "main" group without
    # one) and ``write`` is called once per configured group as write(lines, group, ts, target)
    groups: Optional[List[str]] = None
    group_expr: Optional[str] = None
    # the sink writes gzip files: a device-rendered payload used only by this sink is compressed on the GPU and
    # crosses PCIe compressed (JsonLines.gz)
    gzip: bool = False


DEFAULT_OUTPUT_GROUP = "main"                # BlobSinker.scala:32


def _joined(lines):
    """Newline-joined documents; a blob-backed ``JsonLines`` yields a zero-copy buffer (no per-line objects)."""
    data = getattr(lines, "data", None)
    return data() if data is not None else "\n".join(lines)


def _chunks(xs, n):
    for i in range(0, len(xs), n):
        yield xs[i:i + n]


def _blob_sink(d, output_name) -> Optional[Sink]:
    groups = {g: sd.get("folder") for g, sd in d.group_by_sub_namespace("group.").items()}
    if not groups:
        return None
    compression = (d.get("compressiontype") or "gzip").lower()
    fmt = (d.get("format") or "json").lower()
    group_eval = d.get("groupevaluation")

    def write(lines, group, ts, target):
        """One group's rows into its folder (BlobSinker.sinkDataGroups, :128-157); unknown groups are dropped."""
        folder = groups.get(group)
        if folder is None or not len(lines):
            return 0
        folder = blob_folder(resolve(folder), ts, target)
        suffix = ".json" + (".gz" if compression != "none" else "")
        path = folder + f"part-{uuid.uuid4().hex[:12]}{suffix}"
        timeout = float(os.environ.get("DATAX_BlobWriterTimeout", 10))
        gz = getattr(lines, "gz", None) if compression != "none" else None
        if gz is not None:                   # compressed on the GPU before the D2H (ops/deflate.py)
            fs.write_with_timeout(path, memoryview(gz), timeout_s=timeout, gzipped=True)
        else:
            fs.write_with_timeout(path, _joined(lines), timeout_s=timeout, gzip_it=compression != "none")
        return len(lines)
    return Sink("Blobs", write, groups=sorted(groups), group_expr=group_eval, gzip=compression != "none")


def _eventhub_sink(d, output_name) -> Optional[Sink]:
    conn = d.get("connectionstring")
    if not conn:
        return None
    compression = (d.get("compressiontype") or "gzip").lower()
    props = dict(d.sub_dictionary("appendproperty.").items()) or None

    def write(lines, table, ts, target):
        c = resolve(conn)
        for chunk in _chunks(lines, 200):
            payload = "\n".join(chunk).encode()
            if compression != "none":
                payload = fs.gzip_parallel(payload)
            eventhub_send(c, payload, output_name, props)
        return len(lines)
    return Sink("EventHub", write, d.get("filter"))


def _http_sink(d, output_name) -> Optional[Sink]:
    ep = d.get("endpoint")
    if not ep:
        return None
    headers = {k: v for k, v in d.sub_dictionary("header.").items()}

    def write(lines, table, ts, target):
        from ..telemetry.metrics import http_post_json
        for chunk in _chunks(lines, 200):
            http_post_json(resolve(ep), chunk, headers)
        return len(lines)
    return Sink("HttpPost", write, d.get("filter"))


def _local_scheme(conn: str) -> Optional[str]:
    """``local:`` / ``local:<sub folder>`` — an explicit request for the single-node stand-in of a cloud sink."""
    return conn[len("local:"):].strip("/") if conn.lower().startswith("local:") else None


def _cosmos_sink(d, output_name) -> Optional[Sink]:
    conn_ref = d.get("connectionstring")
    if not conn_ref:
        return None
    db = d.get("database") or "db"
    coll = d.get("collection") or output_name
    from . import azure
    conn = resolve(conn_ref)
    local = _local_scheme(conn)
    if local is None and not azure.is_cosmos_connection(conn):
        # a production string that does not parse must not silently turn into local files
        raise ValueError(f"output '{output_name}': cosmosdb.connectionstring is neither a Cosmos DB connection "
                         "string (AccountEndpoint=…;AccountKey=…) nor an explicit 'local:' target")

    def write(lines, table, ts, target):
        if local is None:
            # document upserts through the REST API (CosmosDBSinker's upsert mode)
            client = azure.CosmosClient(conn)
            for line in lines:
                doc = json.loads(line)
                doc.setdefault("id", str(uuid.uuid4()))
                client.upsert(db, coll, doc)
            return len(lines)
        root = os.environ.get("DXA_FS_ROOT", ".dxa_fs")
        folder = os.path.join(root, "cosmosdb", local, db, coll) if local else os.path.join(root, "cosmosdb", db,
                                                                                            coll)
        os.makedirs(folder, exist_ok=True)
        for line in lines:
            doc = json.loads(line)
            doc.setdefault("id", str(uuid.uuid4()))
            fs.write_atomic(os.path.join(folder, doc["id"] + ".json"), json.dumps(doc))
        return len(lines)
    return Sink("CosmosDB", write, d.get("filter"))


def _opt(d, key):
    """Setting lookup tolerant of the reference's camelCase keys (``trustServerCertificate``)."""
    v = d.get(key)
    if v is None:
        low = key.lower()
        for k, val in d.items():
            if k.lower() == low:
                return val
    return v


def _sql_sink(d, output_name) -> Optional[Sink]:
    """SqlSinker (SqlSinker.scala:19-107): SQL Server / Azure SQL over TDS (``jdbc:sqlserver://…`` or ADO.NET
    strings; ``usebulkinsert`` → bulk load), SQLite for ``sqlite:///path``, a local SQLite file for ``local:``.
    Anything else fails at job start."""
    conn_ref = d.get("connectionstring")
    if not conn_ref:
        return None
    table_name = d.get("table") or output_name
    conn = resolve(conn_ref)
    lock = threading.Lock()
    from . import tds
    if tds.is_sqlserver_connection(conn) or (_opt(d, "url") and tds.is_sqlserver_connection(resolve(_opt(d, "url")))):
        def sec(key):
            v = _opt(d, key)
            return resolve(v) if v else None
        writer = tds.SqlServerWriter(
            conn, table_name, write_mode=d.get("writemode") or "append", url=sec("url"),
            database=_opt(d, "databasename"), user=sec("user"), password=sec("password"),
            encrypt=_opt(d, "encrypt"), trust_server_certificate=_opt(d, "trustServerCertificate"),
            host_name_in_certificate=_opt(d, "hostNameInCertificate"),
            connect_timeout=float(d.get("connectiontimeout") or 30), query_timeout=float(d.get("querytimeout") or 30),
            bulk=(d.get("usebulkinsert") or "false").lower() == "true",
            bulk_batch=int(d.get("bulkcopybatchsize") or 2000),
            table_lock=(d.get("usebulkcopytablelock") or "false").lower() == "true")

        def write_tds(lines, table, ts, target):
            if table.length == 0:
                return 0
            cols = table.names
            types = [c.dtype for c in table.columns]
            rows = [[json.dumps(v, default=str) if isinstance(v, (dict, list)) else v for v in
                     (r[c] for c in cols)] for r in table.to_pylist()]
            with lock:
                return writer.write(cols, types, rows)
        return Sink("SqlSink", write_tds, d.get("filter"), as_json=False)
    local = _local_scheme(conn)
    if conn.startswith("sqlite:///"):
        path = conn[len("sqlite:///"):]
    elif local is not None:
        path = os.path.join(os.environ.get("DXA_FS_ROOT", ".dxa_fs"), "sql", (local or "sql") + ".db")
    else:
        raise ValueError(f"output '{output_name}': sql.connectionstring is not a SQL Server connection string "
                         "(jdbc:sqlserver://… or Server=…), a sqlite:/// path or an explicit 'local:' target")

    def write(lines, table, ts, target):
        import sqlite3
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        rows = table.to_pylist()
        if not rows:
            return 0
        cols = table.names
        with lock, sqlite3.connect(path) as db:
            db.execute(f'CREATE TABLE IF NOT EXISTS "{table_name}" (' + ",".join(f'"{c}"' for c in cols) + ")")
            db.executemany(f'INSERT INTO "{table_name}" VALUES (' + ",".join("?" * len(cols)) + ")",
                           [[_sql_val(r[c]) for c in cols] for r in rows])
        return len(rows)
    return Sink("SqlSink", write, d.get("filter"), as_json=False)


def _sql_val(v):
    if isinstance(v, (dict, list)):
        return json.dumps(v, default=str)
    if isinstance(v, (_dt.datetime, _dt.date)):
        return v.isoformat()
    return v


MEMORY_SINKS: Dict[str, List[str]] = {}


def _file_sink(d, output_name) -> Optional[Sink]:
    path = d.get("path")
    if not path:
        return None

    def write(lines, table, ts, target):
        p = fs.local_path(java_time_format(path, ts))
        p.parent.mkdir(parents=True, exist_ok=True)
        with open(p, "ab") as f:
            if len(lines):
                d = _joined(lines)
                f.write(d.encode("utf-8") if isinstance(d, str) else d)
                f.write(b"\n")
        return len(lines)
    return Sink("File", write, d.get("filter"))


def _console_sink(d, output_name) -> Optional[Sink]:
    def write(lines, table, ts, target):
        for l in lines[: int(d.get("maxrows") or 20)]:
            print(f"[{output_name}] {l}")
        return len(lines)
    return Sink("Console", write, d.get("filter"))


def _memory_sink(d, output_name) -> Optional[Sink]:
    def write(lines, table, ts, target):
        MEMORY_SINKS.setdefault(output_name, []).extend(lines)
        return len(lines)
    return Sink("Memory", write, d.get("filter"))


def _null_sink(d, output_name) -> Optional[Sink]:
    return Sink("Null", lambda lines, table, ts, target: len(lines), d.get("filter"))


SINK_FACTORIES: Dict[str, Callable] = {
    "blob": _blob_sink, "eventhub": _eventhub_sink, "httppost": _http_sink, "cosmosdb": _cosmos_sink,
    "sql": _sql_sink, "file": _file_sink, "console": _console_sink, "memory": _memory_sink, "null": _null_sink,
}


def register_sink(kind: str, factory: Callable):
    SINK_FACTORIES[kind.lower()] = factory


# sinks that never block on I/O: a batch's outputs writing only to these finish on one output thread, one after
# another (a thread per output then only adds wake-ups and GIL hand-offs against the batch thread)
LOCAL_SINKS = frozenset({"Null", "Memory", "Console"})


class OutputOperator:
    def __init__(self, name: str, sinks: List[Sink], processed_schema_path: Optional[str] = None):
        self.name = name
        self.sinks = sinks
        self.processed_schema_path = processed_schema_path
        self._schema_written = False

    @property
    def local(self) -> bool:
        return all(s.name in LOCAL_SINKS for s in self.sinks)

    def stage(self, table: Table, ctx=None) -> "StagedOutput":
        """Device-side half of an output (runs on the batch's thread/stream): drop internal columns, evaluate
        per-sink filters, and start the async D2H copies of what each sink will serialize."""
        from ..config.settings import NAME_PREFIX
        from ..ops import serialize as native_ser
        internal = f"__{NAME_PREFIX}_"
        keep = [i for i, n in enumerate(table.names) if not n.startswith(internal)]
        t = Table([table.names[i] for i in keep], [table.columns[i] for i in keep], table.length, table.device)
        if self.processed_schema_path and not self._schema_written:
            from ..engine.types import to_json_obj
            fs.write_atomic(self.processed_schema_path, json.dumps(to_json_obj(t.schema()), indent=2))
            self._schema_written = True
        st = StagedOutput(self, t.length)
        if t.length == 0:
            return st
        native = native_ser.available()

        def capture(sub, compress=False):
            if native:
                return native_ser.stage_table(sub, compress=compress)
            return table_to_json_lines(sub)            # pure-Python fallback renders eagerly

        whole = None
        for s in self.sinks:
            sub = t
            if s.groups is not None:                 # per-sink payloads: compressed on the device for gzip blobs
                st.items.append((s, self._split_groups(s, t, ctx, lambda sub: capture(sub, s.gzip))))
                continue
            if s.filter_expr:
                from ..engine.expr import EvalContext, Scope, evaluate, predicate_mask
                from ..sql.parser import parse_expression
                m = predicate_mask(evaluate(parse_expression(s.filter_expr), Scope.of_table(t), ctx or EvalContext()))
                sub = t.take(m.nonzero().flatten())
                payload = capture(sub) if s.as_json else _HostRows(sub)
            elif s.as_json:
                if whole is None:
                    whole = capture(t)
                payload = whole
            else:
                payload = _HostRows(t)
            st.items.append((s, payload))
        return st

    @staticmethod
    def _split_groups(s: Sink, t: Table, ctx, capture) -> Dict[str, Any]:
        """Rows of a grouped sink by group name: the flag column is a string expression (BlobSinker.scala:175-183,
        ``rows.groupBy(flagColumn)``); without one every row belongs to "main".  One host read of the distinct group
        names; each group is a row subset captured for serialization."""
        if not s.group_expr:
            return {DEFAULT_OUTPUT_GROUP: capture(t)}
        from ..engine.column import materialize
        from ..engine.expr import EvalContext, Scope, evaluate
        from ..ops import groupby as G
        from ..sql.parser import parse_expression
        col = materialize(evaluate(parse_expression(s.group_expr), Scope.of_table(t), ctx or EvalContext()))
        if hasattr(col, "materialize") and not hasattr(col, "take"):
            col = col.materialize()
        groups = G.group_rows([col])
        names = col.take(groups.rep).to_pylist()
        out = {}
        for k, name in enumerate(names):
            if name is None or str(name) not in s.groups:
                continue
            idx = (groups.gid == k).nonzero().flatten()
            out[str(name)] = capture(t.take(idx))
        return out

    def output(self, table: Table, partition_time: _dt.datetime, ctx=None, target: Optional[str] = None
               ) -> Dict[str, int]:
        return self.stage(table, ctx).finish(partition_time, target)


class _HostRows:
    """Rows of a (sub)table materialised on the host for sinks that take rows rather than JSON (SQL)."""

    def __init__(self, t: Table):
        self.names = list(t.names)
        self.rows = t.to_pylist()
        self.length = len(self.rows)

    def to_pylist(self):
        return self.rows


class StagedOutput:
    def __init__(self, op: OutputOperator, n: int):
        self.op = op
        self.n = n
        self.items: List = []

    def payloads(self) -> List[Any]:
        """Every captured payload (a grouped sink contributes one per group)."""
        out = []
        for _, p in self.items:
            out.extend(p.values() if isinstance(p, dict) else [p])
        return out

    def finish(self, partition_time: _dt.datetime, target: Optional[str] = None) -> Dict[str, int]:
        """Host-side half: render JSON (waits only for this output's D2H copies) and write every sink."""
        metrics = {f"{SINK_PREFIX}InputEvents": self.n}
        # the key set must not depend on the data: ranks all-reduce the batch metrics as one vector
        for s in self.op.sinks:
            if s.groups is not None:             # BlobSinker: <Sink>_Events_<group>, <Sink>_Count_<group> (files)
                for g in s.groups:
                    metrics[f"{SINK_PREFIX}{s.name}_Events_{g}"] = 0
                    metrics[f"{SINK_PREFIX}{s.name}_Count_{g}"] = 0
            else:
                metrics[f"{SINK_PREFIX}{s.name}_{'Filtered' if s.filter_expr else 'All'}"] = 0
        if self.n == 0:
            return metrics
        rendered = {}

        def lines_of(payload):
            if isinstance(payload, _HostRows):
                return None, payload
            key = id(payload)
            if key not in rendered:
                rendered[key] = payload.render() if hasattr(payload, "render") else payload
            return rendered[key], None

        def run(item):
            s, payload = item
            if s.groups is not None:
                out = {}
                for g, p in payload.items():
                    lines, _ = lines_of(p)
                    cnt = s.write(lines, g, partition_time, target)
                    out[f"{SINK_PREFIX}{s.name}_Events_{g}"] = cnt
                    out[f"{SINK_PREFIX}{s.name}_Count_{g}"] = 1 if cnt else 0
                return out
            lines, rows = lines_of(payload)
            cnt = s.write(lines if lines is not None else [], rows, partition_time, target)
            return {f"{SINK_PREFIX}{s.name}_{'Filtered' if s.filter_expr else 'All'}": cnt}

        if len(self.items) == 1:
            metrics.update(run(self.items[0]))
        else:
            for s, payload in self.items:        # render shared payloads once, before fanning out
                if s.groups is None:
                    lines_of(payload)
            for r in _sink_pool.map(run, self.items):
                for k, v in r.items():
                    metrics[k] = metrics.get(k, 0) + v
        return metrics


def build_outputs(d) -> List[OutputOperator]:
    from ..config.settings import OUTPUT_PREFIX
    ops = []
    for name, sub in d.group_by_sub_namespace(OUTPUT_PREFIX).items():
        if name == "default":
            continue
        sinks = []
        for kind, sd in sub.group_by_sub_namespace().items():
            f = SINK_FACTORIES.get(kind.lower())
            if f is None:
                continue
            s = f(sd, name)
            if s is not None:
                sinks.append(s)
        if not sinks:
            raise ValueError(f"no sink is defined for output '{name}'!")
        ops.append(OutputOperator(name, sinks, sub.get("processedschemapath")))
    return ops
