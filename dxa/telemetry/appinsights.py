"""Application Insights telemetry: batch lifecycle events and exceptions (the reference's AppInsightLogger,
DataProcessing/datax-host/src/main/scala/datax/telemetry/AppInsightLogger.scala:18-108).

* The instrumentation key comes from the ``DATAX_APPINSIGHTKEYREF`` job argument / environment variable
  (JobArgument.scala:15), resolved through the secret store (``keyvault://…``, ``secretscope://…`` or a literal); it
  may be a bare key or a connection string ``InstrumentationKey=…;IngestionEndpoint=https://…/``.  Without a key the
  sender is OFF (AppInsightLogger.scala:32-34) and events only go to the local sinks below.
* Every event / exception carries the context properties ``context.appname``, ``context.appid`` and
  ``context.executorid`` (AppInsightLogger.scala:84-105; the executor id is the GPU rank here).
* Envelopes are the Breeze ``v2/track`` schema (``Microsoft.ApplicationInsights.<ikey>.Event`` with ``EventData`` /
  ``ExceptionData``), batched by a background sender thread and POSTed as a JSON array — a slow or unreachable
  endpoint never blocks a micro-batch; a failed POST is retried up to 3 times, then dropped and counted.
* Local sinks (always on): a bounded in-process ring (REST API, tests) and JSON lines appended to
  ``$DXA_TELEMETRY_FILE``.

Event names follow the reference: ``datax/streaming/batch/begin|end`` (EventHubStreamingFactory.scala:88,115;
KafkaStreamingFactory.scala:75,91), ``datax/localstreaming/batch/…`` (LocalStreamingFactory.scala:32,48),
``datax/batch/app/begin`` and ``datax/batch/end`` (BlobBatchingHost.scala:74,104), ``datax/error``
(CommonProcessorFactory.scala:384-394).
"""
from __future__ import annotations

import datetime as _dt
import json
import logging
import os
import queue
import threading
import time
import traceback
from collections import deque
from typing import Dict, List, Optional

log = logging.getLogger("dxa.appinsights")

EVENTS = deque(maxlen=1000)
_lock = threading.Lock()
DEFAULT_ENDPOINT = "https://dc.services.visualstudio.com/"
SDK_VERSION = "dxa-py:1.0"


def _root() -> str:
    from ..config.settings import ROOT
    return ROOT


class _Sender:
    """Background batching sender for ``<endpoint>/v2/track``."""

    def __init__(self, ikey: str, endpoint: str, flush_s: float = 1.0, max_batch: int = 256):
        self.ikey = ikey
        self.url = endpoint.rstrip("/") + "/v2/track"
        self.q: "queue.Queue[Optional[dict]]" = queue.Queue(maxsize=10_000)
        self.flush_s = flush_s
        self.max_batch = max_batch
        self.sent = 0
        self.dropped = 0
        self._t = threading.Thread(target=self._run, name="dxa-appinsights", daemon=True)
        self._t.start()

    def submit(self, env: dict):
        try:
            self.q.put_nowait(env)
        except queue.Full:
            self.dropped += 1

    def _post(self, batch: List[dict]) -> bool:
        import urllib.request
        body = json.dumps(batch, default=str).encode("utf-8")
        req = urllib.request.Request(self.url, data=body, method="POST",
                                     headers={"Content-Type": "application/json"})
        for attempt in range(3):
            try:
                with urllib.request.urlopen(req, timeout=10) as r:
                    if 200 <= r.status < 300:
                        return True
            except Exception as e:  # noqa: BLE001 — telemetry must never fail the job
                log.debug("appinsights POST failed (attempt %d): %s", attempt + 1, e)
            time.sleep(0.2 * (attempt + 1))
        return False

    def _run(self):
        stop = False
        while not stop:
            batch = []
            try:
                item = self.q.get(timeout=self.flush_s)
                if item is None:
                    stop = True
                else:
                    batch.append(item)
                while len(batch) < self.max_batch:
                    item = self.q.get_nowait()
                    if item is None:
                        stop = True
                        break
                    batch.append(item)
            except queue.Empty:
                pass
            if batch:
                if self._post(batch):
                    self.sent += len(batch)
                else:
                    self.dropped += len(batch)

    def close(self, timeout: float = 5.0):
        self.q.put(None)
        self._t.join(timeout)


_sender: Optional[_Sender] = None
_context: Dict[str, str] = {}


def parse_key(value: str):
    """Bare instrumentation key or connection string → (ikey, endpoint)."""
    if "=" in value:
        parts = dict(p.split("=", 1) for p in value.split(";") if "=" in p)
        norm = {k.strip().lower(): v.strip() for k, v in parts.items()}
        ikey = norm.get("instrumentationkey")
        if not ikey:
            raise ValueError("AppInsights connection string has no InstrumentationKey")
        return ikey, norm.get("ingestionendpoint") or DEFAULT_ENDPOINT
    return value.strip(), DEFAULT_ENDPOINT


def configure(settings=None, app_name: Optional[str] = None, executor_id: Optional[str] = None,
              key: Optional[str] = None, endpoint: Optional[str] = None):
    """Turn the sender on when a key (or ``DATAX_APPINSIGHTKEYREF``) resolves; set the context properties."""
    global _sender
    from ..config.secrets import resolve
    ref = key
    if ref is None:
        ref = (settings.get("DATAX_APPINSIGHTKEYREF") if settings is not None else None) or \
            os.environ.get("DATAX_APPINSIGHTKEYREF")
    app = app_name or (settings.job_name() if settings is not None else None) or f"{_root()}_Unknown_App"
    from .. import parallel as P
    _context.clear()
    _context.update({"context.appname": app, "context.appid": f"{app}-{os.getpid()}",
                     "context.executorid": str(executor_id if executor_id is not None else P.rank())})
    if _sender is not None:
        _sender.close()
        _sender = None
    if not ref:
        log.warning("AI Key is not found, AppInsight Sender is OFF")
        return None
    try:
        value = resolve(ref)
    except Exception:  # noqa: BLE001
        value = None
    if not value:
        log.warning("AI KeyRef is not found at %s, AppInsight Sender is OFF", ref)
        return None
    ikey, ep = parse_key(value)
    _sender = _Sender(ikey, endpoint or os.environ.get("DXA_APPINSIGHTS_ENDPOINT") or ep)
    log.warning("AI Key is set, AppInsight Sender is ON")
    return _sender


def shutdown():
    global _sender
    if _sender is not None:
        _sender.close()
        _sender = None


def _envelope(kind: str, base_type: str, base_data: dict) -> dict:
    ikey = _sender.ikey if _sender is not None else ""
    return {
        "name": f"Microsoft.ApplicationInsights.{ikey.replace('-', '')}.{kind}",
        "time": _dt.datetime.utcnow().strftime("%Y-%m-%dT%H:%M:%S.%fZ"),
        "iKey": ikey,
        "tags": {"ai.cloud.role": _context.get("context.appname", ""),
                 "ai.cloud.roleInstance": _context.get("context.executorid", ""),
                 "ai.internal.sdkVersion": SDK_VERSION},
        "data": {"baseType": base_type, "baseData": dict(ver=2, **base_data)},
    }


def _local(e: dict):
    with _lock:
        EVENTS.append(e)
    path = os.environ.get("DXA_TELEMETRY_FILE")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(e, default=str) + "\n")


def _merge(props: Optional[Dict[str, str]]) -> Dict[str, str]:
    out = dict(_context)
    if props:
        out.update({k: str(v) for k, v in props.items()})
    return out


def track_event(name: str, properties: Optional[Dict[str, str]] = None,
                measurements: Optional[Dict[str, float]] = None):
    """``name`` without a leading product root gets ``datax/`` prepended (ProductConstant.ProductRoot)."""
    if not name.startswith(_root() + "/"):
        name = f"{_root()}/{name}"
    props = _merge(properties)
    meas = {k: float(v) for k, v in (measurements or {}).items() if isinstance(v, (int, float))}
    _local({"ts": time.time(), "event": name, "props": props, "measurements": meas})
    if _sender is not None:
        _sender.submit(_envelope("Event", "EventData", {"name": name, "properties": props, "measurements": meas}))


def track_exception(location: str, batch_time=None, exc: Optional[BaseException] = None,
                    properties: Optional[Dict[str, str]] = None, measurements: Optional[Dict[str, float]] = None):
    """The reference's error pair: a ``datax/error`` event with location, message and the top 10 stack frames,
    then the exception itself (CommonProcessorFactory.scala:384-394)."""
    import sys
    if exc is None:
        exc = sys.exc_info()[1]
    msg = str(exc) if exc is not None else ""
    stack = "".join(traceback.format_exception(type(exc), exc, exc.__traceback__, limit=10)) if exc is not None \
        else traceback.format_exc(limit=10)
    props = {"errorLocation": location, "errorMessage": msg, "errorStackTrace": stack,
             "batchTime": str(batch_time)}
    if properties:
        props.update(properties)
    track_event("error", props, None)
    xprops = _merge({k: v for k, v in props.items() if k != "errorStackTrace"})
    meas = {k: float(v) for k, v in (measurements or {}).items()}
    _local({"ts": time.time(), "exception": type(exc).__name__ if exc is not None else "Error", "message": msg,
            "props": xprops, "measurements": meas})
    if _sender is not None:
        _sender.submit(_envelope("Exception", "ExceptionData", {
            "exceptions": [{"id": 1, "outerId": 0, "typeName": type(exc).__name__ if exc is not None else "Error",
                            "message": msg, "hasFullStack": True, "stack": stack}],
            "properties": xprops, "measurements": meas}))
