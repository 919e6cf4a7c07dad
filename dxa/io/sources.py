"""Streaming sources: each produces one ``RawBatch`` (device byte buffer + record offsets) per micro-batch.

Reference inputs: EventHub / IoT Hub direct streams, Kafka direct streams, the onebox local
generator (DataProcessing/datax-host/src/main/scala/datax/input/LocalStreamingSource.scala:17-39), blob batches
(BlobBatchingHost) and blob-pointer events (BlobPointerInput.scala).

Here:
* ``LocalGeneratorSource`` — schema-driven synthetic events rendered straight into HBM by the GPU generator;
* ``FileSource``           — newline-delimited JSON files (optionally gzip), framed on the device;
* ``BlobPointerSource``    — events carrying ``{"BlobPath": …}``, whose files are read and framed;
* ``SocketSource``         — a TCP listener receiving newline-delimited events (netcat-style ingest);
* ``QueueSource``          — an in-process queue (the REST ingest endpoint and tests push into it);
* ``PartitionedReplaySource`` — a set of per-partition byte streams with offsets, checkpointed in the reference's
  ``offsets.txt`` format (``batchTimeMs,name,partition,fromSeq,untilSeq``, EventhubCheckpointer.scala:16-73).
EventHub / Kafka client libraries are not part of this environment; those input kinds are rejected with a clear
error at job start (the conf keys are still generated and parsed).
"""
from __future__ import annotations

import datetime as _dt
import gzip
import json
import os
import queue
import re
import socket
import threading
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..engine.processor import RawBatch
from ..ops.jsonparse import frame_records
from . import fs


class SourceError(Exception):
    pass


class Source:
    name = "source"
    # metric names this source may attach to a batch (RawBatch.source_metrics); the processor zero-fills the absent
    # ones so every rank all-reduces the same key set
    metric_names: Tuple[str, ...] = ()

    def next_batch(self, batch_time_us: int) -> Optional[RawBatch]:
        raise NotImplementedError

    def commit(self, batch_time_us: int):
        pass

    def close(self):
        pass


class OffsetTrackedSource(Source):
    """Partitioned source whose reads run ahead of its commits.

    ``StreamingHost(pipeline=True)`` fetches batch t+1 while batch t is still being processed, so the read cursor
    (``fetch_pos``) and the committed position (``pos``) are distinct: ``next_batch`` advances ``fetch_pos`` at once and
    records that batch's ``(start, end)`` ranges under its batch time; ``commit(bt)`` pops exactly those ranges and
    checkpoints them (reference ``EventhubCheckpointer.scala:59-60`` writes one line per partition of the committed
    batch).  A restart resumes from ``pos`` (the checkpoint), so uncommitted prefetched batches are re-read
    (at-least-once)."""

    def _init_offsets(self, positions: Dict, ckpt: Optional["Checkpointer"], hub_of=None):
        self.pos = dict(positions)           # committed
        self.fetch_pos = dict(positions)     # next record to read
        self._inflight: "Dict[int, Dict]" = {}
        self._lock = threading.Lock()
        self.ckpt = ckpt
        self._hub_of = hub_of or (lambda key: key)

    def _record_batch(self, batch_time_us: int, ranges: Dict):
        with self._lock:
            for k, (_s, e) in ranges.items():
                self.fetch_pos[k] = e
            self._inflight[batch_time_us] = ranges

    @property
    def pending(self) -> Dict:
        """Ranges of the oldest uncommitted batch (for inspection)."""
        with self._lock:
            return dict(self._inflight[min(self._inflight)]) if self._inflight else {}

    def commit(self, batch_time_us: int):
        with self._lock:
            ranges = self._inflight.pop(batch_time_us, None)
            if ranges is None:
                return
            for k, (_s, e) in ranges.items():
                prev = self.pos.get(k)
                self.pos[k] = e if prev is None else max(prev, e)
            if self.ckpt:
                self.ckpt.write(batch_time_us // 1000,
                                [(*self._hub_of(k), s, e) for k, (s, e) in ranges.items()])


def _to_device_batch(records: Sequence[bytes], device, file_info=None) -> RawBatch:
    buf, offs = frame_records(list(records), device=device, pin=torch.device(device).type == "cuda")
    return RawBatch(buf, offs, len(records), file_info=file_info, source_bytes=int(offs[-1].item()) if records
                    else 0)


class LocalGeneratorSource(Source):
    """Synthetic events from a SimulatedData/DataGenerator schema, rendered on the device.

    ``events_per_batch`` is the JOB's rate, as the reference's single local receiver (LocalStreamingSource.scala:
    31-37): with W ranks, rank r renders rows ``[row + off_r, row + off_r + n_r)`` of the same counter-based stream
    (``n_r`` = its share), so the W ranks together produce exactly the events one rank would, never duplicates."""
    name = "local"

    def __init__(self, schema, events_per_batch: int, device, seed: int = 1, simulated: bool = False,
                 rank: Optional[int] = None, world: Optional[int] = None):
        from .. import parallel as P
        from ..simulate.datagen import compile_simulated, compile_spark
        self.prog = compile_simulated(schema) if simulated else compile_spark(schema)
        self.n = int(events_per_batch)
        self.device = torch.device(device)
        self.seed = seed
        self.row = 0
        self.rank = P.rank() if rank is None else rank
        self.world = P.world() if world is None else world
        base, extra = divmod(self.n, self.world)
        self.n_mine = base + (1 if self.rank < extra else 0)
        self.offset = self.rank * base + min(self.rank, extra)

    def next_batch(self, batch_time_us: int) -> Optional[RawBatch]:
        from ..simulate.datagen import generate
        buf, offs = generate(self.prog, self.n_mine, self.device, seed=self.seed, row0=self.row + self.offset,
                             base_ms=batch_time_us // 1000, step_us=0)
        self.row += self.n
        return RawBatch(buf, offs, self.n_mine)


class QueueSource(Source):
    """Events pushed by producers (REST ingest, tests); each batch drains what has arrived."""
    name = "queue"

    def __init__(self, device, max_batch: int = 10_000_000):
        self.q: "queue.Queue[bytes]" = queue.Queue()
        self.device = torch.device(device)
        self.max_batch = max_batch

    def push(self, record: bytes | str):
        self.q.put(record.encode() if isinstance(record, str) else record)

    def push_many(self, records):
        for r in records:
            self.push(r)

    def next_batch(self, batch_time_us: int) -> Optional[RawBatch]:
        recs = []
        while len(recs) < self.max_batch:
            try:
                recs.append(self.q.get_nowait())
            except queue.Empty:
                break
        return _to_device_batch(recs, self.device)


class SocketSource(QueueSource):
    """TCP listener: each connection streams newline-delimited JSON events."""
    name = "socket"

    def __init__(self, device, host: str = "127.0.0.1", port: int = 9999, rank: Optional[int] = None):
        """With W ranks each rank is one receiver: rank r listens on ``port + r`` (port 0: any free port), so
        producers spread their connections over the ranks the way Spark spreads receivers over executors."""
        from .. import parallel as P
        super().__init__(device)
        rank = P.rank() if rank is None else rank
        self.sock = socket.create_server((host, port + rank if port else 0))
        self.port = self.sock.getsockname()[1]
        self._stop = False
        threading.Thread(target=self._accept, daemon=True).start()

    def _accept(self):
        while not self._stop:
            try:
                conn, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(conn,), daemon=True).start()

    def _serve(self, conn):
        with conn, conn.makefile("rb") as f:
            for line in f:
                line = line.strip()
                if line:
                    self.push(line)

    def close(self):
        self._stop = True
        self.sock.close()


class FileSource(Source):
    """New files appearing under a folder or glob pattern (local or ``wasbs://``), newline-delimited JSON
    (gzip-aware).  Each batch takes the files not yet processed; framing runs on the device.  With W ranks a file is
    read by exactly one rank (``fs.owned_by_rank``: stable hash of its path), as Spark spreads input files over
    executors."""
    name = "file"

    def __init__(self, pattern: str, device, max_files_per_batch: int = 1000, rank: Optional[int] = None,
                 world: Optional[int] = None):
        from .. import parallel as P
        self.pattern = pattern
        self.device = torch.device(device)
        self.seen = set()
        self.max_files = max_files_per_batch
        self.rank = P.rank() if rank is None else rank
        self.world = P.world() if world is None else world

    def _list(self) -> List[str]:
        return fs.owned_by_rank(fs.list_matching(self.pattern), self.rank, self.world)

    def next_batch(self, batch_time_us: int) -> Optional[RawBatch]:
        files = [p for p in self._list() if p not in self.seen][: self.max_files]
        data = bytearray()
        for p in files:
            self.seen.add(p)
            b = fs.read_bytes(p)
            data += b
            if b and not b.endswith(b"\n"):
                data += b"\n"
        return frame_bytes(bytes(data), self.device, file_info={"inputPath": ";".join(files)} if files else None)


def frame_bytes(data: bytes, device, file_info=None) -> RawBatch:
    device = torch.device(device)
    if device.type == "cuda":
        from ..ops.jsonparse import frame_lines_gpu
        host = torch.frombuffer(bytearray(data + b"\0" * 16), dtype=torch.uint8)
        buf = host.pin_memory().to(device, non_blocking=True)
        offs = frame_lines_gpu(buf, len(data))
        return RawBatch(buf, offs, int(offs.shape[0]) - 1, file_info=file_info, source_bytes=len(data))
    recs = [l for l in data.split(b"\n") if l.strip()]
    return _to_device_batch(recs, device, file_info)


_SA_REGEX = r"wasbs?://[\w-]+@([\w\d]+)\.blob\.core\.windows\.net/.*"


def _java_time_pattern(fmt: str) -> str:
    out = fmt
    for j, p in (("yyyy", "%Y"), ("MM", "%m"), ("dd", "%d"), ("HH", "%H"), ("mm", "%M"), ("ss", "%S"),
                 ("SSS", "%f")):
        out = out.replace(j, p)
    return out.replace("'", "")


class BlobPointerSource(Source):
    """Events of the form ``{"BlobPath": "<path>"}`` (BlobPointerInput.scala:28-162): each pointed-to blob's lines
    become rows of the batch, with a per-row ``FileInternal`` (input path, file time, output file name, target,
    rule index prefix).

    With ``datax.job.input.default.source.<id>.target`` sources configured, a path is in scope only when the source
    id extracted by ``sourceidregex`` (default: the storage account of a ``wasbs://`` URL) names one of them; its
    file time comes from ``filetimeregex`` (group 1; ``filetimeformat`` or ``yyyy-MM-dd HH:mm:ss`` after '_'→':'
    and 'T'→' '), its output file name from ``blobpathregex`` (groups joined by '-'); out-of-scope paths are dropped
    (BlobPointerInput.filterPathGroups).  Without sources, every path (optionally filtered by ``path_regex``) is
    read.  Per batch: ``InputBlobs`` and ``Latency-Blobs`` (now − earliest file time)."""
    name = "blobpointer"
    metric_names = ("InputBlobs", "Latency-Blobs")

    def __init__(self, inner: Source, device, path_regex: Optional[str] = None, settings=None):
        self.inner = inner
        self.device = torch.device(device)
        self.rx = re.compile(path_regex) if path_regex else None
        self.sources: Dict[str, Dict[str, Optional[str]]] = {}
        self.source_id_rx = re.compile(_SA_REGEX)
        self.blob_path_rx = self.file_time_rx = None
        self.file_time_fmt = None
        if settings is not None:
            from ..config import settings as S
            inp = settings.sub_dictionary(S.INPUT_PREFIX)
            for sid, sub in inp.group_by_sub_namespace("source.").items():
                self.sources[sid] = {"target": sub.get("target"), "catalogprefix": sub.get("catalogprefix")}
            if inp.get("sourceidregex"):
                self.source_id_rx = re.compile(inp.get("sourceidregex"))
            if inp.get("blobpathregex"):
                self.blob_path_rx = re.compile(inp.get("blobpathregex"))
            if inp.get("filetimeregex"):
                self.file_time_rx = re.compile(inp.get("filetimeregex"))
            self.file_time_fmt = inp.get("filetimeformat")
        self.last_metrics: Dict[str, float] = {}

    def file_internal(self, path: str) -> Optional[Dict[str, str]]:
        """FileInternal of one path, or None when it is out of scope."""
        if not self.sources:
            return {"inputPath": path}
        m = self.source_id_rx.search(path)
        src = self.sources.get(m.group(1)) if m else None
        if src is None:
            return None
        info = {"inputPath": path, "target": src.get("target") or "", "ruleIndexPrefix": src.get("catalogprefix") or ""}
        if self.file_time_rx is not None:
            t = self.file_time_rx.search(path)
            if t:
                try:
                    txt = t.group(1)
                    ts = (_dt.datetime.strptime(txt, _java_time_pattern(self.file_time_fmt)) if self.file_time_fmt
                          else _dt.datetime.fromisoformat(txt.replace("_", ":").replace("T", " ")))
                    info["fileTime"] = ts.strftime("%Y-%m-%d %H:%M:%S")
                except ValueError:
                    log_warn(f"cannot parse the file time of {path}")
        if self.blob_path_rx is not None:
            m2 = self.blob_path_rx.search(path)
            if m2 is None:
                raise SourceError(f"blobpathregex does not match blob path '{path}'")
            info["outputFileName"] = "-".join(g or "" for g in m2.groups())
        return info

    def next_batch(self, batch_time_us: int) -> Optional[RawBatch]:
        b = self.inner.next_batch(batch_time_us)
        if b is None or b.n == 0:
            return b
        data = b.buf.cpu().numpy().tobytes()
        offs = b.offs.cpu().tolist()
        ends = b.ends.cpu().tolist() if b.ends is not None else None
        files: List[Tuple[str, Dict[str, str]]] = []
        seen = set()
        dropped = 0
        for i in range(b.n):
            try:
                p = json.loads(data[offs[i]:(ends[i] if ends else offs[i + 1])])["BlobPath"]
            except Exception:  # noqa: BLE001
                continue
            if (self.rx is not None and not self.rx.search(p)) or p in seen:
                continue
            seen.add(p)
            info = self.file_internal(p)
            if info is None:
                dropped += 1
                continue
            files.append((p, info))
        if dropped:
            log_warn(f"Found out-of-scope paths count={dropped}")
        blob = bytearray()
        rows: List[Tuple[Dict[str, str], int]] = []
        for p, info in files:
            x = fs.read_bytes(p)
            if x and not x.endswith(b"\n"):
                x += b"\n"
            blob += x
            rows.append((info, sum(1 for line in x.split(b"\n")[:-1] if len(line) >= 1)))
        times = [_dt.datetime.fromisoformat(i["fileTime"]) for i, _ in rows if i.get("fileTime")]
        self.last_metrics = {"InputBlobs": float(len(files))}
        if times:
            self.last_metrics["Latency-Blobs"] = (_dt.datetime.utcnow() - min(times)).total_seconds()
        raw = frame_bytes(bytes(blob), self.device, file_info={"inputPath": ";".join(p for p, _ in files)})
        if rows and sum(r for _i, r in rows) == raw.n:
            raw.file_rows = rows
        raw.source_metrics = dict(self.last_metrics)
        return raw


def log_warn(msg: str):
    import logging
    logging.getLogger("dxa.sources").warning(msg)


class PartitionedReplaySource(OffsetTrackedSource):
    """Partitioned event log with sequence numbers and reference-format offset checkpoints.

    ``partitions``: name → list of event payloads (an in-memory or file-backed log).  ``max_rate`` caps events per
    partition per batch (the reference's ``maxRatePerPartition``)."""
    name = "replay"

    def __init__(self, partitions: Dict[str, Sequence[bytes]], device, checkpoint_dir: Optional[str] = None,
                 max_rate: Optional[int] = None, hub: str = "replay", flush_existing: bool = False):
        self.device = torch.device(device)
        self.max_rate = max_rate
        self.hub = hub
        from .. import parallel as P
        # partition → rank: rank r reads the partitions at positions ≡ r (mod W) of the sorted partition list, and
        # checkpoints them in its own offsets file
        names = sorted(partitions)
        mine = [p for i, p in enumerate(names) if i % P.world() == P.rank()]
        self.parts = {p: partitions[p] for p in mine}
        ckpt = Checkpointer(checkpoint_dir) if checkpoint_dir else None
        pos = {p: 0 for p in self.parts}
        if ckpt and not flush_existing:
            for (name, part), until in ckpt.restore().items():
                if name == hub and part in pos:
                    pos[part] = until
        self._init_offsets(pos, ckpt, hub_of=lambda p: (self.hub, p))

    def next_batch(self, batch_time_us: int) -> Optional[RawBatch]:
        recs = []
        ranges = {}
        for p, log in self.parts.items():
            start = self.fetch_pos[p]
            end = len(log) if self.max_rate is None else min(len(log), start + self.max_rate)
            recs.extend(log[start:end])
            ranges[p] = (start, end)
        self._record_batch(batch_time_us, ranges)
        return _to_device_batch(recs, self.device)


class Checkpointer:
    """``offsets.txt`` (+ ``.old`` backup) — the reference's EventhubCheckpointer format
    (``batchTimeMs,ehName,partition,fromSeq,untilSeq``, EventhubCheckpointer.scala:16-73).

    With W ranks every rank owns a disjoint set of partitions and writes its own file, ``<folder>/rank-<r>/
    offsets.txt`` (ranks never overwrite each other's lines); ``restore`` reads the single-rank file and every
    rank's file and keeps, per (hub, partition), the line of the latest batch — so a restart at any world size finds
    every partition's committed position, whichever rank wrote it."""

    def __init__(self, folder: str, rank: Optional[int] = None, world: Optional[int] = None):
        from .. import parallel as P
        rank = P.rank() if rank is None else rank
        world = P.world() if world is None else world
        self.root = str(fs.local_path(folder))
        sub = self.root if world <= 1 else os.path.join(self.root, f"rank-{rank}")
        self.path = os.path.join(sub, "offsets.txt")

    def write(self, batch_ms: int, ranges):
        os.makedirs(os.path.dirname(self.path), exist_ok=True)
        if os.path.exists(self.path):
            os.replace(self.path, self.path + ".old")
        lines = [f"{batch_ms},{name},{part},{s},{e}" for name, part, s, e in ranges]
        fs.write_atomic(self.path, "\n".join(lines) + "\n")

    def _files(self) -> List[str]:
        out = []
        cands = [os.path.join(self.root, "offsets.txt")]
        if os.path.isdir(self.root):
            cands += [os.path.join(self.root, d, "offsets.txt") for d in sorted(os.listdir(self.root))
                      if d.startswith("rank-")]
        for c in cands:
            if os.path.exists(c):
                out.append(c)
            elif os.path.exists(c + ".old"):
                out.append(c + ".old")
        return out

    def restore(self) -> Dict[Tuple[str, str], int]:
        best: Dict[Tuple[str, str], Tuple[int, int]] = {}
        for path in self._files():
            for line in open(path):
                parts = line.strip().split(",")
                if len(parts) != 5:
                    continue
                key, ms, until = (parts[1], parts[2]), int(parts[0]), int(parts[4])
                if key not in best or ms >= best[key][0]:
                    best[key] = (ms, until)
        return {k: v[1] for k, v in best.items()}


def build_source(settings, device, kind: Optional[str] = None) -> Source:
    """Source from a job's settings (``datax.job.input.default.*``)."""
    from ..config import settings as S
    from ..engine.types import schema_from_json
    d = settings
    inp = d.sub_dictionary(S.INPUT_PREFIX)
    if kind is None:
        if inp.get("local.schemafile") or inp.get("local.eventsperbatch"):
            kind = "local"
        elif inp.get("file.pattern"):
            kind = "file"
        elif inp.get("socket.port"):
            kind = "socket"
        elif inp.get("eventhub.connectionstring"):
            kind = "eventhub"                # AMQP unless eventhub.protocol=kafka (the Kafka endpoint)
        elif inp.get("kafka.bootstrapservers") or inp.get("kafka.topics"):
            kind = "kafka"
        else:
            kind = "queue"
    if kind == "local":
        from ..config.secrets import resolve
        path = resolve(inp.get("local.schemafile") or inp.get_string("blobschemafile"))
        text = path if path.lstrip().startswith("{") else fs.read_text(path)
        obj = json.loads(text)
        simulated = isinstance(obj, dict) and "dataSchema" in obj
        schema = obj["dataSchema"][0]["fields"] if simulated else schema_from_json(text)
        return LocalGeneratorSource(schema, int(inp.get("local.eventsperbatch") or 100), device,
                                    int(inp.get("local.seed") or 1), simulated)
    if kind == "file":
        return FileSource(inp.get_string("file.pattern"), device)
    if kind == "socket":
        return SocketSource(device, inp.get("socket.host") or "127.0.0.1", int(inp.get("socket.port") or 9999))
    if kind == "queue":
        return QueueSource(device)
    if kind in ("blob", "blobpointer"):
        # BlobStreamingApp: the stream carries {"BlobPath": …} pointer events (BlobPointerInput.scala)
        inner_kind = "eventhub" if inp.get("eventhub.connectionstring") else (
            "kafka" if (inp.get("kafka.bootstrapservers") or inp.get("kafka.topics")) else "queue")
        return BlobPointerSource(build_source(settings, device, inner_kind), device, settings=settings)
    if kind in ("eventhub", "iothub") and (inp.get("eventhub.protocol") or "amqp").lower() == "amqp":
        # the direct AMQP stream (EventHubStreamingFactory); IoT Hub's built-in endpoint is Event Hub-compatible
        from .. import parallel as P
        from .eventhub import build_eventhub_source
        return build_eventhub_source(inp, device, P.rank(), P.world())
    if kind in ("kafka", "eventhub", "kafkaeventhub", "iothub"):
        from .. import parallel as P
        from .kafka import build_kafka_source
        return build_kafka_source(inp, device, "eventhub" if kind in ("eventhub", "iothub", "kafkaeventhub")
                                  else "kafka", P.rank(), P.world())
    raise SourceError(f"unknown input kind '{kind}'")
