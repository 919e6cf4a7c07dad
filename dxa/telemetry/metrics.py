"""Per-batch metric emission with the reference's wire formats
(DataProcessing/datax-host/src/main/scala/datax/telemetry/MetricLogger.scala:14-100):

* Redis sorted sets: ``ZADD <app>:<metric> <nowMs> {"uts":<batchMs>, "val":<v>}``
* EventHub / JSON lines: ``{"app":"<app>", "met":"<metric>","uts":<batchMs>, "val":<v>}``
* HTTP POST (onebox ``/api/data/upload``): a JSON array of those objects.

Sinks are configured by ``datax.job.process.metric.{redis,eventhub,httppost}`` (MetricsHandler.scala:11-33); we
add ``file`` (JSON lines) and an in-process ``MetricStore`` (the Redis-compatible store behind our metrics REST API).
"""
from __future__ import annotations

import bisect
from dataclasses import dataclass
import json
import socket
import threading
import time
import urllib.request
from typing import Dict, Iterable, List, Optional, Tuple

from ..config.secrets import resolve


def _num(v: float) -> str:
    if isinstance(v, float) and v.is_integer() and abs(v) < 1e15:
        return repr(float(v))
    return repr(v)


class MetricStore:
    """In-process sorted-set store (Redis ZADD / ZRANGEBYSCORE semantics) shared by the engine and the REST API."""

    _instance: Optional["MetricStore"] = None

    def __init__(self):
        self._sets: Dict[str, List[Tuple[float, str]]] = {}
        self._lock = threading.Lock()

    @classmethod
    def default(cls) -> "MetricStore":
        if cls._instance is None:
            cls._instance = MetricStore()
        return cls._instance

    def zadd(self, key: str, score: float, member: str, nx: bool = False):
        with self._lock:
            s = self._sets.setdefault(key, [])
            if nx and any(m == member for _, m in s):
                return 0
            bisect.insort(s, (float(score), member))
            if len(s) > 100_000:
                del s[: len(s) - 100_000]
            return 1

    def zrangebyscore(self, key: str, lo: float, hi: float) -> List[Tuple[float, str]]:
        with self._lock:
            s = self._sets.get(key, [])
            i = bisect.bisect_left(s, (float(lo), ""))
            out = []
            for sc, m in s[i:]:
                if sc > hi:
                    break
                out.append((sc, m))
            return out

    def keys(self, pattern: str = "*") -> List[str]:
        import fnmatch
        with self._lock:
            return [k for k in self._sets if fnmatch.fnmatch(k, pattern)]


@dataclass
class RedisServerConf:
    name: str
    host: str
    port: int
    key: Optional[str]
    timeout: int
    use_ssl: bool
    is_cluster: bool


def parse_redis_connection_string(conn: str) -> Optional[RedisServerConf]:
    """``<host>:<port>,password=<p>,ssl=True|False,cluster=True|False,timeout=<ms>`` with the reference's defaults
    (ssl and cluster on, 3000 ms) — RedisBase.scala:32-58."""
    if not conn:
        return None
    parts = conn.split(",")
    hp = parts[0].strip().split(":")
    if len(hp) != 2:
        raise ValueError("Malformed format of host and port in redis connection string")
    opts = {}
    for p in parts[1:]:
        pos = p.find("=")
        if pos <= 0:
            raise ValueError("Malformed format of parts in redis connection string")
        opts[p[:pos].strip()] = p[pos + 1:]

    def flag(k):
        return opts.get(k, "True").strip().lower() == "true"
    return RedisServerConf(hp[0], hp[0], int(hp[1]), opts.get("password"), int(opts.get("timeout", "3000")),
                           flag("ssl"), flag("cluster"))


class RedisClient:
    """Minimal RESP client (``host:port,password=…,ssl=…``, reference RedisBase.scala:32-58)."""

    def __init__(self, conn: str, timeout: Optional[float] = None):
        conf = parse_redis_connection_string(conn)
        self.conf = conf
        self.host, self.port = conf.host, conf.port
        self.password = conf.key
        self.use_ssl = conf.use_ssl
        self.timeout = timeout if timeout is not None else conf.timeout / 1000.0
        self._sock = None
        self._lock = threading.Lock()

    def _connect(self):
        s = socket.create_connection((self.host, self.port), timeout=self.timeout)
        if self.use_ssl:
            import ssl
            s = ssl.create_default_context().wrap_socket(s, server_hostname=self.host)
        self._sock = s
        self._file = s.makefile("rb")
        if self.password:
            self._cmd("AUTH", self.password)

    def _cmd(self, *args):
        payload = b"*%d\r\n" % len(args) + b"".join(
            b"$%d\r\n%s\r\n" % (len(a), a) for a in (x if isinstance(x, bytes) else str(x).encode() for x in args))
        self._sock.sendall(payload)
        return self._reply()

    def _reply(self):
        line = self._file.readline()
        t, rest = line[:1], line[1:-2]
        if t == b"+":
            return rest.decode()
        if t == b"-":
            raise RuntimeError(rest.decode())
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            if n < 0:
                return None
            data = self._file.read(n + 2)[:-2]
            return data.decode()
        if t == b"*":
            return [self._reply() for _ in range(int(rest))]
        raise RuntimeError(f"bad redis reply {line!r}")

    def command(self, *args):
        with self._lock:
            if self._sock is None:
                self._connect()
            return self._cmd(*args)

    def zadd(self, key, score, member):
        return self.command("ZADD", key, score, member)


def http_post_json(url: str, items: List, headers: Optional[Dict[str, str]] = None, timeout: float = 5.0,
                   retries: int = 0) -> int:
    body = ("[" + ",".join(i if isinstance(i, str) else json.dumps(i) for i in items) + "]").encode()
    h = {"Content-Type": "application/json"}
    h.update(headers or {})
    last = None
    for _ in range(retries + 1):
        try:
            req = urllib.request.Request(url, data=body, headers=h, method="POST")
            with urllib.request.urlopen(req, timeout=timeout) as r:
                return r.status
        except Exception as e:  # noqa: BLE001 — best-effort telemetry
            last = e
    raise last


class MetricLogger:
    def __init__(self, app: str, redis: Optional[str] = None, eventhub: Optional[str] = None,
                 http_endpoint: Optional[str] = None, file_path: Optional[str] = None,
                 store: Optional[MetricStore] = None):
        self.app = app
        self.redis = RedisClient(resolve(redis)) if redis else None
        self.eventhub = resolve(eventhub) if eventhub else None
        self.http = http_endpoint or None
        self.file = file_path
        self.store = store
        self.errors = 0
        self.sent: List[Dict] = []

    @staticmethod
    def from_settings(d, store: Optional[MetricStore] = None) -> "MetricLogger":
        from ..config.settings import PROCESS_PREFIX
        sub = d.sub_dictionary(PROCESS_PREFIX + "metric.")
        return MetricLogger(d.metric_app_name(), sub.get("redis") or None, sub.get("eventhub") or None,
                            sub.get("httppost") or None, sub.get("file") or None, store)

    def lines(self, metrics: Iterable[Tuple[str, float]], ts_ms: int) -> List[str]:
        return [f'{{"app":"{self.app}", "met":"{k}","uts":{ts_ms}, "val":{_num(float(v))}}}' for k, v in metrics]

    def send_batch_metrics(self, metrics: Dict[str, float], ts_ms: int):
        items = list(metrics.items())
        now = int(time.time() * 1000)
        self.sent = [{"app": self.app, "met": k, "uts": ts_ms, "val": v} for k, v in items]
        try:
            if self.store is not None:
                for k, v in items:
                    self.store.zadd(f"{self.app}:{k}", now, f'{{"uts":{ts_ms}, "val":{_num(float(v))}}}')
            if self.redis is not None:
                for k, v in items:
                    self.redis.zadd(f"{self.app}:{k}", now, f'{{"uts":{ts_ms}, "val":{_num(float(v))}}}')
            full = self.lines(items, ts_ms)
            if self.eventhub:
                from ..io.sinks import eventhub_send
                eventhub_send(self.eventhub, "\n".join(full).encode(), "metrics")
            if self.http:
                http_post_json(self.http, full)
            if self.file:
                from ..io import fs
                p = fs.local_path(self.file)
                p.parent.mkdir(parents=True, exist_ok=True)
                with open(p, "a") as f:
                    f.write("\n".join(full) + "\n")
        except Exception:  # noqa: BLE001 — metrics must never take the engine down
            self.errors += 1
