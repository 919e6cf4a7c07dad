"""Kafka wire-protocol client + streaming source + producer — no client library needed.

The reference reads Kafka through Spark's direct stream (DataProcessing/datax-host/.../input/KafkaStreamingFactory
.scala:22-94, KafkaInputSetting.scala:14-142) and Event Hubs through the Event Hubs Spark connector
(EventHubStreamingFactory.scala:23-118); its test producer sends generated JSON (app/KafkaProducer.scala:19-95).
Here one small client speaks the Kafka protocol directly (Metadata v1, ListOffsets v1, Fetch v4, Produce v3,
SaslHandshake v1 + SaslAuthenticate v0 for SASL/PLAIN over TLS) — which also covers Azure Event Hubs through its
Kafka endpoint (``<namespace>.servicebus.windows.net:9093``, user ``$ConnectionString``).

Record batches are decoded natively (``host_kafka.cpp``) straight into a padded value buffer + offsets, i.e. the
layout the GPU JSON parser consumes after one H2D copy.  Partitions are spread over ranks (partition index mod world
size — one source partition per GPU rank, like one RDD partition per Kafka partition), offsets are checkpointed in the
reference's ``offsets.txt`` format and committed only after the batch's outputs are written.
"""
from __future__ import annotations

import ctypes
import socket
import ssl
import struct
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .sources import Checkpointer, OffsetTrackedSource, RawBatch, Source, SourceError

API_PRODUCE, API_FETCH, API_LIST_OFFSETS, API_METADATA = 0, 1, 2, 3
API_SASL_HANDSHAKE, API_SASL_AUTH = 17, 36
EARLIEST, LATEST = -2, -1


class KafkaError(SourceError):
    pass


# -- native codec ------------------------------------------------------------------------------------------------------
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        from ..ops.serialize import lib
        L = lib()
        L.dxa_crc32c.restype = ctypes.c_uint32
        L.dxa_crc32c.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.dxa_kafka_count.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.dxa_kafka_extract.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.dxa_kafka_encode.restype = ctypes.c_void_p
        L.dxa_kafka_encode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_int32, ctypes.c_void_p]
        L.dxa_kafka_encode_stream.restype = ctypes.c_void_p
        L.dxa_kafka_encode_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int64] * 4 + \
            [ctypes.c_int32] * 4 + [ctypes.c_void_p]
        L.dxa_kafka_encode_lz4.restype = ctypes.c_void_p
        L.dxa_kafka_encode_lz4.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                           ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
        _LIB = L
    return _LIB


def _codec_fns():
    L = _lib()
    if not hasattr(L, "_codecs_bound"):
        p, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        for name, args in (("dxa_snappy_compress", [p, i64, p, i64, i32]), ("dxa_snappy_decompress", [p, i64, p, i64]),
                           ("dxa_snappy_length", [p, i64]), ("dxa_zstd_decompress", [p, i64, p, i64]),
                           ("dxa_zstd_bound", [p, i64]), ("dxa_zstd_compress", [p, i64, p, i64, i32, i32]),
                           ("dxa_zstd_compress_bound", [i64])):
            f = getattr(L, name)
            f.argtypes, f.restype = args, i64
        L._codecs_bound = True
    return L


def snappy_compress(data: bytes, xerial: bool = True) -> bytes:
    """snappy-java's xerial stream (what Java producers write) or one raw block."""
    L = _codec_fns()
    cap = 256 + len(data) * 2
    out = ctypes.create_string_buffer(cap)
    n = L.dxa_snappy_compress(data, len(data), out, cap, int(xerial))
    if n < 0:
        raise KafkaError("snappy compress failed")
    return out.raw[:n]


def snappy_decompress(data: bytes) -> bytes:
    """xerial stream or raw block → bytes (the host decoder of codec 2)."""
    L = _codec_fns()
    m = L.dxa_snappy_length(data, len(data))
    if m < 0:
        raise KafkaError("malformed snappy payload")
    out = ctypes.create_string_buffer(max(1, m))
    if L.dxa_snappy_decompress(data, len(data), out, m) != m:
        raise KafkaError("malformed snappy payload")
    return out.raw[:m]


def zstd_compress(data: bytes, level: int = 3, content_size: bool = False,
                  checksum: bool = False) -> bytes:
    """One zstd frame from the system libzstd (the producer side: Kafka's zstd-jni stream omits the content size)."""
    L = _codec_fns()
    cap = L.dxa_zstd_compress_bound(len(data))
    if cap < 0:
        raise KafkaError("libzstd is not installed")
    out = ctypes.create_string_buffer(cap)
    n = L.dxa_zstd_compress(data, len(data), out, cap, level, int(content_size) | (int(checksum) << 1))
    if n < 0:
        raise KafkaError("zstd compress failed")
    return out.raw[:n]


def zstd_decompress(data: bytes) -> bytes:
    """Frames → bytes with this package's decoder (host_zstd.cpp, RFC 8878; no libzstd involved)."""
    L = _codec_fns()
    bound = L.dxa_zstd_bound(data, len(data))
    if bound < 0:
        raise KafkaError("malformed zstd frame")
    out = ctypes.create_string_buffer(max(1, bound))
    m = L.dxa_zstd_decompress(data, len(data), out, bound)
    if m < 0:
        raise KafkaError(f"malformed zstd frame (error {m})")
    return out.raw[:m]


def crc32c(data: bytes) -> int:
    return int(_lib().dxa_crc32c(data, len(data)))


CODECS = {"none": 0, "gzip": 1, "snappy": 2, "lz4": 3, "zstd": 4}
ZSTD_DEFAULT_LEVEL = 3            # Kafka's compression.zstd.level default (zstd's own default)


def encode_batch(values: Sequence[bytes], timestamp_ms: Optional[int] = None, compression: str = "none",
                 level: int = 1, block_size: int = 64 * 1024) -> bytes:
    """One v2 record batch holding ``values`` (null keys); ``compression`` none / gzip / snappy / lz4 / zstd
    (``level``: Kafka's compression.lz4.level or compression.zstd.level; ``block_size``: the LZ4 frame block size).
    snappy is snappy-java's xerial stream (what the Java producer writes); zstd needs the system libzstd."""
    vals = b"".join(values)
    offs = np.zeros(len(values) + 1, dtype=np.int64)
    if values:
        offs[1:] = np.cumsum([len(v) for v in values])
    return encode_batch_arrays(np.frombuffer(vals, np.uint8), offs, timestamp_ms, compression, level, block_size)


def encode_batch_arrays(vals: np.ndarray, offs: np.ndarray, timestamp_ms: Optional[int] = None,
                        compression: str = "none", level: int = 1, block_size: int = 64 * 1024) -> bytes:
    """``encode_batch`` over a values buffer + int64 offsets [n+1] (no per-record Python objects)."""
    vals = np.ascontiguousarray(vals)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    n = int(offs.shape[0]) - 1
    out_len = ctypes.c_int64(0)
    L = _lib()
    ptr = L.dxa_kafka_encode_lz4(vals.ctypes.data, offs.ctypes.data, n,
                                 int(time.time() * 1000) if timestamp_ms is None else timestamp_ms,
                                 CODECS[compression.lower()], level, block_size, ctypes.byref(out_len))
    if not ptr:
        raise KafkaError(f"record batch encode failed ({compression})")
    try:
        return ctypes.string_at(ptr, out_len.value)
    finally:
        L.dxa_host_free(ptr)


def encode_stream(vals: np.ndarray, offs: np.ndarray, per_batch: int, base_offset: int = 0,
                  timestamp_ms: Optional[int] = None, compression: str = "lz4", level: int = 9,
                  block_size: int = 64 * 1024, threads: int = 16) -> np.ndarray:
    """A producer's record batches of ``per_batch`` records each, back to back as a Fetch response carries them
    (base offsets from ``base_offset``) → uint8 array.  ``vals`` + int64 ``offs`` [n+1] hold the record values."""
    vals = np.ascontiguousarray(vals)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    n = int(offs.shape[0]) - 1
    out_len = ctypes.c_int64(0)
    L = _lib()
    ptr = L.dxa_kafka_encode_stream(vals.ctypes.data, offs.ctypes.data, n, per_batch, base_offset,
                                    int(time.time() * 1000) if timestamp_ms is None else timestamp_ms,
                                    CODECS[compression.lower()], level, block_size, threads, ctypes.byref(out_len))
    if not ptr:
        raise KafkaError(f"record batch stream encode failed ({compression})")
    try:
        return np.frombuffer(ctypes.string_at(ptr, out_len.value), dtype=np.uint8).copy()
    finally:
        L.dxa_host_free(ptr)


KAFKA_BATCH_SIZE = 16384          # producer batch.size default (bytes)
_RATIO_FACTOR = 1.05               # CompressionRatioEstimator.COMPRESSION_RATIO_ESTIMATION_FACTOR


def records_per_batch(vals: np.ndarray, offs: np.ndarray, batch_size: int = KAFKA_BATCH_SIZE,
                      compression: str = "lz4", level: int = 9, block_size: int = 64 * 1024,
                      rounds: int = 4, sample: int = 20000) -> Tuple[int, float]:
    """How many records a Java producer puts in one record batch: the accumulator closes a batch when its *estimated
    compressed* size would pass ``batch.size`` (MemoryRecordsBuilder.hasRoomFor: uncompressed bytes × the topic's
    learned compression ratio × 1.05).  The ratio estimate starts at 1.0 and converges to the observed one, so the
    fixed point is iterated on a sample of the records → (records per batch, compressed/uncompressed ratio)."""
    n = int(offs.shape[0]) - 1
    m = min(n, sample)
    avg = float(offs[m] - offs[0]) / max(1, m)
    ratio = 1.0
    per = 1
    for _ in range(rounds):
        per = max(1, int(batch_size / (avg * ratio * _RATIO_FACTOR)))
        enc = encode_stream(vals, offs[:m + 1], per, compression=compression, level=level, block_size=block_size)
        ratio = enc.nbytes / float(offs[m] - offs[0])
    return per, ratio


_ERRS = {-2: "unsupported message format (magic != 2)", -3: "CRC mismatch", -4: "gzip decode failed",
         -5: "unsupported compression codec", -6: "record batch decompression failed (lz4 / snappy / zstd)"}


def decode_records(record_set: bytes, min_offset: int, pad: int = 16, verify_crc: bool = True
                   ) -> Tuple[np.ndarray, np.ndarray, np.ndarray, int]:
    """Record set bytes → (values uint8 [bytes+pad], value offsets int64 [n+1], record offsets int64 [n],
    next fetch offset)."""
    L = _lib()
    n = ctypes.c_int64(0)
    nb = ctypes.c_int64(0)
    nxt = ctypes.c_int64(0)
    rc = L.dxa_kafka_count(record_set, len(record_set), min_offset, ctypes.byref(n), ctypes.byref(nb),
                           ctypes.byref(nxt), 1 if verify_crc else 0)
    if rc:
        raise KafkaError(f"record batch decode failed: {_ERRS.get(rc, rc)}")
    vals = np.zeros(nb.value + pad, dtype=np.uint8)
    offs = np.zeros(n.value + 1, dtype=np.int64)
    recoffs = np.zeros(max(1, n.value), dtype=np.int64)
    rc = L.dxa_kafka_extract(record_set, len(record_set), min_offset, vals.ctypes.data, offs.ctypes.data,
                             recoffs.ctypes.data, ctypes.byref(nxt))
    if rc:
        raise KafkaError(f"record batch decode failed: {_ERRS.get(rc, rc)}")
    return vals, offs, recoffs[:n.value], nxt.value


# -- protocol primitives ----------------------------------------------------------------------------------------------
class _W:
    def __init__(self):
        self.b = bytearray()

    def i8(self, v):
        self.b += struct.pack(">b", v)
        return self

    def i16(self, v):
        self.b += struct.pack(">h", v)
        return self

    def i32(self, v):
        self.b += struct.pack(">i", v)
        return self

    def i64(self, v):
        self.b += struct.pack(">q", v)
        return self

    def str(self, s: Optional[str]):
        if s is None:
            return self.i16(-1)
        e = s.encode()
        self.i16(len(e))
        self.b += e
        return self

    def bytes(self, v: Optional[bytes]):
        if v is None:
            return self.i32(-1)
        self.i32(len(v))
        self.b += v
        return self

    def array(self, items, fn):
        if items is None:
            return self.i32(-1)
        self.i32(len(items))
        for it in items:
            fn(self, it)
        return self


class _R:
    def __init__(self, b: bytes):
        self.b = memoryview(b)
        self.p = 0

    def _take(self, fmt, n):
        v = struct.unpack_from(fmt, self.b, self.p)[0]
        self.p += n
        return v

    def i8(self):
        return self._take(">b", 1)

    def i16(self):
        return self._take(">h", 2)

    def i32(self):
        return self._take(">i", 4)

    def i64(self):
        return self._take(">q", 8)

    def str(self):
        n = self.i16()
        if n < 0:
            return None
        s = bytes(self.b[self.p:self.p + n]).decode()
        self.p += n
        return s

    def bytes(self):
        n = self.i32()
        if n < 0:
            return None
        v = bytes(self.b[self.p:self.p + n])
        self.p += n
        return v

    def array(self, fn):
        n = self.i32()
        return [] if n < 0 else [fn(self) for _ in range(n)]


class Connection:
    def __init__(self, host: str, port: int, client_id: str = "dxa", use_ssl: bool = False,
                 sasl: Optional[Tuple[str, str]] = None, timeout: float = 30.0):
        s = socket.create_connection((host, port), timeout=timeout)
        if use_ssl:
            s = ssl.create_default_context().wrap_socket(s, server_hostname=host)
        self.sock = s
        self.client_id = client_id
        self.corr = 0
        self.lock = threading.Lock()
        if sasl is not None:
            self._sasl_plain(*sasl)

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass

    def _recv_exact(self, n):
        out = bytearray()
        while len(out) < n:
            chunk = self.sock.recv(min(1 << 20, n - len(out)))
            if not chunk:
                raise KafkaError("connection closed by broker")
            out += chunk
        return bytes(out)

    def request(self, api_key: int, version: int, body: bytes) -> _R:
        with self.lock:
            self.corr += 1
            hdr = _W().i16(api_key).i16(version).i32(self.corr).str(self.client_id).b
            msg = bytes(hdr) + body
            self.sock.sendall(struct.pack(">i", len(msg)) + msg)
            size = struct.unpack(">i", self._recv_exact(4))[0]
            resp = self._recv_exact(size)
        r = _R(resp)
        if r.i32() != self.corr:
            raise KafkaError("correlation id mismatch")
        return r

    def _sasl_plain(self, user: str, password: str):
        r = self.request(API_SASL_HANDSHAKE, 1, bytes(_W().str("PLAIN").b))
        err = r.i16()
        if err:
            raise KafkaError(f"SASL handshake failed (error {err}; mechanisms {r.array(_R.str)})")
        token = b"\0" + user.encode() + b"\0" + password.encode()
        r = self.request(API_SASL_AUTH, 0, bytes(_W().bytes(token).b))
        err = r.i16()
        msg = r.str()
        if err:
            raise KafkaError(f"SASL authentication failed: {msg or err}")


def parse_bootstrap(servers: str) -> List[Tuple[str, int]]:
    out = []
    for hp in servers.split(","):
        hp = hp.strip()
        if hp:
            h, _, p = hp.rpartition(":")
            out.append((h, int(p)))
    return out


def eventhub_kafka_settings(conn: str) -> Dict[str, object]:
    """Event Hubs connection string → Kafka endpoint settings (SASL_SSL PLAIN, ``$ConnectionString``)."""
    parts = dict(p.split("=", 1) for p in conn.split(";") if "=" in p)
    host = parts["Endpoint"].split("://", 1)[-1].strip("/")
    return {"bootstrap": f"{host}:9093", "topic": parts.get("EntityPath"), "use_ssl": True,
            "sasl": ("$ConnectionString", conn)}


class KafkaClient:
    """Metadata-aware client: one connection per broker, requests routed to partition leaders."""

    def __init__(self, bootstrap: str, client_id: str = "dxa", use_ssl: bool = False,
                 sasl: Optional[Tuple[str, str]] = None):
        self.bootstrap = parse_bootstrap(bootstrap)
        self.client_id, self.use_ssl, self.sasl = client_id, use_ssl, sasl
        self.conns: Dict[Tuple[str, int], Connection] = {}
        self.brokers: Dict[int, Tuple[str, int]] = {}
        self.leaders: Dict[Tuple[str, int], int] = {}

    def _conn(self, addr) -> Connection:
        c = self.conns.get(addr)
        if c is None:
            c = self.conns[addr] = Connection(addr[0], addr[1], self.client_id, self.use_ssl, self.sasl)
        return c

    def _any(self) -> Connection:
        last = None
        for addr in list(self.conns) + self.bootstrap:
            try:
                return self._conn(addr)
            except OSError as e:
                last = e
        raise KafkaError(f"no reachable bootstrap broker: {last}")

    def close(self):
        for c in self.conns.values():
            c.close()
        self.conns.clear()

    def metadata(self, topics: Optional[List[str]] = None) -> Dict[str, List[int]]:
        body = _W().array(topics, lambda w, t: w.str(t)).b
        r = self._any().request(API_METADATA, 1, bytes(body))
        brokers = r.array(lambda r: (r.i32(), r.str(), r.i32(), r.str()))
        self.brokers = {nid: (h, p) for nid, h, p, _ in brokers}
        r.i32()                                             # controller id
        out = {}

        def part(r):
            err, pid, leader = r.i16(), r.i32(), r.i32()
            r.array(_R.i32)
            r.array(_R.i32)
            return err, pid, leader

        for _ in range(r.i32()):
            err, name, _internal = r.i16(), r.str(), r.i8()
            parts = r.array(part)
            if err:
                raise KafkaError(f"metadata error {err} for topic {name}")
            out[name] = sorted(p for _, p, _ in parts)
            for _, p, leader in parts:
                self.leaders[(name, p)] = leader
        return out

    def _leader(self, topic, partition) -> Connection:
        if (topic, partition) not in self.leaders:
            self.metadata([topic])
        nid = self.leaders[(topic, partition)]
        return self._conn(self.brokers[nid])

    def list_offset(self, topic: str, partition: int, when: int = LATEST) -> int:
        """EARLIEST (-2), LATEST (-1), or a timestamp in ms → the first offset whose record timestamp is at or after
        it (the end of the log when there is none: the broker answers -1)."""
        off = self._list_offset(topic, partition, when)
        if off < 0 and when >= 0:
            return self._list_offset(topic, partition, LATEST)
        return off

    def _list_offset(self, topic: str, partition: int, when: int) -> int:
        body = _W().i32(-1).array([topic], lambda w, t: w.str(t).array(
            [partition], lambda w2, p: w2.i32(p).i64(when))).b
        r = self._leader(topic, partition).request(API_LIST_OFFSETS, 1, bytes(body))
        for _ in range(r.i32()):
            r.str()
            for _ in range(r.i32()):
                _p, err, _ts, off = r.i32(), r.i16(), r.i64(), r.i64()
                if err:
                    raise KafkaError(f"list offsets error {err}")
                return off
        raise KafkaError("empty ListOffsets response")

    def fetch(self, topic: str, partition: int, offset: int, max_bytes: int = 64 << 20,
              max_wait_ms: int = 100) -> Tuple[bytes, int]:
        """→ (record set bytes, high watermark)."""
        body = _W().i32(-1).i32(max_wait_ms).i32(1).i32(max_bytes).i8(0).array(
            [topic], lambda w, t: w.str(t).array([partition], lambda w2, p: w2.i32(p).i64(offset).i32(max_bytes))).b
        r = self._leader(topic, partition).request(API_FETCH, 4, bytes(body))
        r.i32()                                             # throttle
        for _ in range(r.i32()):
            r.str()
            for _ in range(r.i32()):
                _p, err, hw, _lso = r.i32(), r.i16(), r.i64(), r.i64()
                r.array(lambda r: (r.i64(), r.i64()))
                recs = r.bytes() or b""
                if err == 1:                                # OFFSET_OUT_OF_RANGE
                    raise KafkaError(f"offset {offset} out of range for {topic}/{partition}")
                if err:
                    raise KafkaError(f"fetch error {err} for {topic}/{partition}")
                return recs, hw
        return b"", offset

    def produce(self, topic: str, partition: int, values: Sequence[bytes], acks: int = 1,
                compression: str = "none", timestamp_ms: Optional[int] = None) -> int:
        batch = encode_batch(values, timestamp_ms, compression=compression)
        body = _W().str(None).i16(acks).i32(30000).array(
            [topic], lambda w, t: w.str(t).array([partition], lambda w2, p: w2.i32(p).bytes(batch))).b
        r = self._leader(topic, partition).request(API_PRODUCE, 3, bytes(body))
        for _ in range(r.i32()):
            r.str()
            for _ in range(r.i32()):
                _p, err, base, _t = r.i32(), r.i16(), r.i64(), r.i64()
                if err:
                    raise KafkaError(f"produce error {err}")
                return base
        return -1


class KafkaSource(OffsetTrackedSource):
    """Direct Kafka / Event Hubs (Kafka endpoint) stream.  Each rank owns partitions ``i % world == rank``; a batch
    fetches up to ``max_rate`` records per partition from the read cursor, which runs ahead of the committed
    position while the host prefetches; ``commit(bt)`` (called after batch bt's outputs are written) advances the
    committed positions by exactly that batch's ranges and writes them to ``offsets.txt``."""
    name = "kafka"

    def __init__(self, client: KafkaClient, topics: List[str], device, checkpoint_dir: Optional[str] = None,
                 max_rate: Optional[int] = None, start: int = EARLIEST, flush_existing: bool = False,
                 rank: int = 0, world: int = 1, max_fetches: int = 64, device_decode: Optional[bool] = None,
                 check_crcs="host"):
        self.client = client
        # consumer check.crcs: "host" (default; the planner / host decoder checks), "device" (kafka_crc_kernel on
        # the GPU ingest path), or off (False / "false")
        self.check_crcs = {True: "host", False: "off", "true": "host", "false": "off"}.get(check_crcs, check_crcs)
        self.verify_crc = self.check_crcs != "off"
        self._status: Dict[int, object] = {}
        self.topics = topics
        self.device = torch.device(device)
        self.max_rate = max_rate
        self.max_fetches = max_fetches
        # record batches decompressed and framed on the GPU (dxa.io.kafka_device); host decoding otherwise
        self.device_decode = (self.device.type == "cuda") if device_decode is None else device_decode
        self._decoder = None
        ckpt = Checkpointer(checkpoint_dir, rank, world) if checkpoint_dir else None
        meta = client.metadata(topics)
        all_parts = [(t, p) for t in topics for p in meta.get(t, [])]
        self.parts = [tp for i, tp in enumerate(all_parts) if i % world == rank]
        restored = {} if (ckpt is None or flush_existing) else ckpt.restore()
        pos: Dict[Tuple[str, int], int] = {}
        for t, p in self.parts:
            got = restored.get((t, str(p)))
            pos[(t, p)] = got if got is not None else client.list_offset(t, p, start)
        self._init_offsets(pos, ckpt, hub_of=lambda tp: (tp[0], str(tp[1])))

    def next_batch(self, batch_time_us: int) -> Optional[RawBatch]:
        if self.device_decode:
            got = self._next_batch_device(batch_time_us)
            if got is not None:
                return got
        return self._next_batch_host(batch_time_us)

    def _next_batch_device(self, batch_time_us: int) -> Optional[RawBatch]:
        """Fetch, plan batch headers on the host, decode on the GPU.  None (cursor untouched) when a fetched
        record set needs the host decoder — the batch is then fetched again on the host path."""
        from . import kafka_device as KD
        sets, plans = [], []
        ranges: Dict[Tuple[str, int], Tuple[int, int]] = {}
        pos = 0
        for tp in self.parts:
            start = self.fetch_pos[tp]
            cur, got = start, 0
            for _ in range(self.max_fetches):
                recs, hw = self.client.fetch(tp[0], tp[1], cur)
                if not recs:
                    break
                try:
                    plan = KD.plan_fetch(recs, cur, self.check_crcs == "host")
                except KD.Unsupported:
                    return None
                if self.max_rate is not None:
                    plan = KD.trim(plan, self.max_rate - got)
                n, nxt = plan.nrec, plan.next_offset
                if n:
                    sets.append(recs)
                    plans.append((plan, pos))
                    pos += len(recs)
                got += n
                cur = max(cur, nxt)
                if cur >= hw or (self.max_rate is not None and got >= self.max_rate):
                    break
            ranges[tp] = (start, cur)
        staging = torch.empty(pos + 64, dtype=torch.uint8, pin_memory=True)
        sn = staging.numpy()
        for recs, (_, at) in zip(sets, plans):
            sn[at:at + len(recs)] = np.frombuffer(recs, dtype=np.uint8)
        if self._decoder is None:
            self._decoder = KD.DeviceRecordDecoder(self.device, track=False,
                                                   verify_crc=self.check_crcs == "device")
        raw, done = self._decoder.decode(staging, KD.merge(plans))
        cur_stream = torch.cuda.current_stream(self.device)
        cur_stream.wait_event(done)
        # the batch's tensors were allocated on the decode stream but are read on the consumer's stream (parse,
        # string views, outputs): without record_stream the caching allocator could hand their memory to the next
        # decode while this batch's kernels still read it
        for t in (raw.buf, raw.offs, raw.ends):
            if t is not None:
                t.record_stream(cur_stream)
        self._record_batch(batch_time_us, ranges)
        with self._lock:
            self._status[batch_time_us] = raw.status
        return raw

    def verify(self, batch_time_us: int):
        """Raise ``DecodeError`` if batch ``batch_time_us`` failed to decode on the device.  The streaming host calls
        this before ``commit`` — a corrupt batch fails the job without committing its offsets (the host decoder
        raises ``KafkaError`` for the same data); the status was copied to pinned memory behind the decode, so this
        reads one word."""
        with self._lock:
            st = self._status.pop(batch_time_us, None)
        if st is not None and st.failed():
            from .kafka_device import DecodeError
            raise DecodeError(f"Kafka batch {batch_time_us}: record batches failed to decode on the device")

    def check(self):
        """Check every decoded batch not yet verified (tests, shutdown)."""
        with self._lock:
            pending, self._status = self._status, {}
        bad = [bt for bt, st in pending.items() if st is not None and st.failed()]
        if bad:
            from .kafka_device import DecodeError
            raise DecodeError(f"Kafka batches {bad}: record batches failed to decode on the device")

    def _next_batch_host(self, batch_time_us: int) -> Optional[RawBatch]:
        vals_list, offs_list = [], []
        ranges: Dict[Tuple[str, int], Tuple[int, int]] = {}
        for tp in self.parts:
            start = self.fetch_pos[tp]
            cur, got = start, 0
            for _ in range(self.max_fetches):
                recs, hw = self.client.fetch(tp[0], tp[1], cur)
                if not recs:
                    break
                vals, offs, recoffs, nxt = decode_records(recs, cur, pad=0, verify_crc=self.verify_crc)
                n = len(recoffs)
                if self.max_rate is not None and got + n > self.max_rate:
                    n = self.max_rate - got
                    nxt = int(recoffs[n - 1]) + 1 if n > 0 else cur
                    vals, offs = vals[: offs[n]], offs[: n + 1]
                if n:
                    vals_list.append(vals[: offs[n]])
                    offs_list.append(offs[: n + 1])
                got += n
                cur = max(cur, nxt)
                if cur >= hw or (self.max_rate is not None and got >= self.max_rate):
                    break
            ranges[tp] = (start, cur)
        self._record_batch(batch_time_us, ranges)
        return _raw_from_parts(vals_list, offs_list, self.device)

    def close(self):
        self.client.close()


def _raw_from_parts(vals_list, offs_list, device) -> RawBatch:
    total = sum(int(o[-1]) for o in offs_list)
    n = sum(len(o) - 1 for o in offs_list)
    buf = np.zeros(total + 16, dtype=np.uint8)
    offs = np.zeros(n + 1, dtype=np.int64)
    pos = rows = 0
    for v, o in zip(vals_list, offs_list):
        k = len(o) - 1
        buf[pos:pos + int(o[-1])] = v[: int(o[-1])]
        offs[rows:rows + k + 1] = o + pos
        pos += int(o[-1])
        rows += k
    tb, to = torch.from_numpy(buf), torch.from_numpy(offs)
    if device.type == "cuda":
        tb = tb.pin_memory().to(device, non_blocking=True)
        to = to.pin_memory().to(device, non_blocking=True)
    return RawBatch(tb, to, n, source_bytes=total)


def start_position(start_enqueue_time: Optional[str], auto_offset_reset: Optional[str] = None,
                   now_ms: Optional[int] = None) -> int:
    """The reference's starting position (EventHubStreamingFactory.scala:47-64; KafkaInputSetting.scala:91):
    ``startenqueuetime`` unset → ``autooffsetreset`` (default "latest": end of stream); 0 → start of stream;
    < 0 → now + that many seconds; > 0 → that epoch second.  Returns EARLIEST / LATEST or a timestamp in ms, which
    ``KafkaClient.list_offset`` resolves per partition (ListOffsets by timestamp: the first record at or after it)."""
    import time as _time
    if start_enqueue_time not in (None, ""):
        v = int(str(start_enqueue_time).strip())
        if v == 0:
            return EARLIEST
        if v < 0:
            return (int(_time.time() * 1000) if now_ms is None else now_ms) + v * 1000
        return v * 1000
    return EARLIEST if (auto_offset_reset or "latest").strip().lower() == "earliest" else LATEST


def build_kafka_source(inp, device, kind: str, rank: int = 0, world: int = 1) -> KafkaSource:
    """From ``datax.job.input.default.{kafka|eventhub}.*`` settings."""
    from ..config.secrets import resolve
    if kind == "eventhub":
        conn = resolve(inp.get_string("eventhub.connectionstring"))
        es = eventhub_kafka_settings(conn)
        client = KafkaClient(es["bootstrap"], use_ssl=True, sasl=es["sasl"])
        topics = [es["topic"]] if es["topic"] else [t.strip() for t in (inp.get("eventhub.name") or "").split(",")]
        ckpt = inp.get("eventhub.checkpointdir")
        rate = inp.get("eventhub.maxrate")
        flush = (inp.get("eventhub.flushexistingcheckpoints") or "false").lower() == "true"
    else:
        servers = resolve(inp.get("kafka.bootstrapservers") or inp.get_string("kafka.connectionstring"))
        sasl = None
        if inp.get("kafka.sasl.username"):
            sasl = (inp.get("kafka.sasl.username"), resolve(inp.get("kafka.sasl.password") or ""))
        client = KafkaClient(servers, use_ssl=(inp.get("kafka.ssl") or "false").lower() == "true", sasl=sasl)
        topics = [t.strip() for t in inp.get_string("kafka.topics").split(",") if t.strip()]
        ckpt = inp.get("kafka.checkpointdir")
        rate = inp.get("kafka.maxrate")
        flush = (inp.get("kafka.flushexistingcheckpoints") or "false").lower() == "true"
    crcs = (inp.get(f"{kind}.checkcrcs") or "true").lower()          # true (host) | device | auto | false
    if crcs == "auto":
        # per rank from the node's planner threads and host memory budget (affinity.crc_placement)
        import os
        from ..parallel.affinity import crc_placement, host_threads
        lw = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        crcs = crc_placement(lr, lw, host_threads(lr, lw))
    start = start_position(inp.get(f"{kind}.startenqueuetime"), inp.get(f"{kind}.autooffsetreset"))
    return KafkaSource(client, topics, device, ckpt, int(rate) if rate else None, start=start,
                       flush_existing=flush, rank=rank, world=world, check_crcs=crcs)
