"""Metrics ingestion into the dashboard store.

* ``ingest_lines`` — the reference's DataX.Metrics.Ingestor (Helper/IngestorEventProcessor.cs:61-200): each line is a
  JSON metric (``app``/``product``, ``met``/``metricname``, ``val``/``metric``, ``uts``/``eventtime``, ``pivot1``);
  it becomes ``ZADD NX <product>:<metric> <server-ms> {"uts":<server-ms>, "val":<v>, "pivot1":"<p>"}`` (server time
  on purpose, to avoid client clock skew).
* ``ingest_items`` — the onebox website's ``/api/data/upload`` cache (Website/util/localCache.js:9-40): default
  metrics (``app``/``met``/``val``) and custom metrics (``Product``/``MetricName``/``Metric``/``Pivot1``), stamped with
  the server time; a bounded ring of the raw items is kept for inspection.
* ``EventQueueIngestor`` — a background thread that drains a metrics queue (the reference reads Event Hubs).
"""
from __future__ import annotations

import json
import queue
import threading
import time
from typing import Any, Dict, Iterable, List, Optional

from ..telemetry.metrics import MetricStore, _num

CACHE_SIZE = 10_000


def generate_row(line: str, now_ms: Optional[int] = None):
    """(key, content, score) for one metric line, or None when the line is not a JSON object."""
    try:
        obj = json.loads(line)
    except ValueError:
        return None
    if not isinstance(obj, dict):
        return None
    item: Dict[str, Any] = {}
    for k, v in obj.items():
        kl = k.lower()
        if kl in ("eventtime", "uts"):
            item["time"] = v
        elif kl in ("metricname", "met"):
            item["name"] = v
        elif kl in ("metric", "val"):
            item["val"] = v
        elif kl in ("product", "app"):
            item["product"] = v
        elif kl == "pivot1":
            item["pivot"] = v
    now_ms = int(time.time() * 1000) if now_ms is None else now_ms
    val = item.get("val")
    val_s = json.dumps(val) if isinstance(val, (int, float)) else str(val)
    pivot = "" if item.get("pivot") is None else str(item.get("pivot"))
    content = '{"uts":' + str(now_ms) + ', "val":' + val_s + ', "pivot1":"' + pivot + '"}'
    return f"{item.get('product')}:{item.get('name')}", content, now_ms


def ingest_lines(store: MetricStore, lines: Iterable[str]) -> Dict[str, int]:
    messages = metrics = 0
    for line in lines:
        messages += 1
        row = generate_row(line)
        if row is not None:
            key, content, score = row
            store.zadd(key, score, content, nx=True)
            metrics += 1
    return {"messages": messages, "metrics": metrics}


def ingest_items(store: MetricStore, items: List[Any], cache: Optional[List[Dict[str, Any]]] = None):
    now = int(time.time() * 1000)
    for it in items:
        if isinstance(it, str):
            try:
                it = json.loads(it)
            except ValueError:
                continue
        if not isinstance(it, dict):
            continue
        it = dict(it)
        it["uts"] = now
        if it.get("Product"):
            key = f"{it['Product']}:{it.get('MetricName')}"
            content = json.dumps({"uts": now, "val": it.get("Metric"), "pivot1": it.get("Pivot1")})
        else:
            key = f"{it.get('app')}:{it.get('met')}"
            v = it.get("val")
            content = '{"uts":' + str(now) + ', "val":' + (_num(float(v)) if isinstance(v, (int, float))
                                                          else json.dumps(v)) + "}"
        it["MetricName"] = key
        store.zadd(key, now, content)
        if cache is not None:
            cache.append(it)
    if cache is not None and len(cache) > CACHE_SIZE:
        del cache[:len(cache) - CACHE_SIZE]


class EventQueueIngestor(threading.Thread):
    """Drains newline-delimited metric messages from a queue into the store."""

    def __init__(self, store: MetricStore, q: "queue.Queue[bytes]"):
        super().__init__(daemon=True, name="dxa-metrics-ingestor")
        self.store, self.q = store, q
        self._stop = threading.Event()
        self.stats = {"messages": 0, "metrics": 0}

    def run(self):
        while not self._stop.is_set():
            try:
                msg = self.q.get(timeout=0.2)
            except queue.Empty:
                continue
            text = msg.decode("utf-8", "replace") if isinstance(msg, (bytes, bytearray)) else str(msg)
            r = ingest_lines(self.store, text.splitlines())
            for k in self.stats:
                self.stats[k] += r[k]

    def stop(self):
        self._stop.set()
