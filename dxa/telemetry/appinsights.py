"""Batch telemetry events / exceptions (the reference's AppInsightLogger, DataProcessing/datax-host/src/main/scala/
datax/telemetry/AppInsightLogger.scala:18-108).  Events are appended as JSON lines to ``$DXA_TELEMETRY_FILE`` (if set)
and kept in a bounded in-process ring for the REST API."""
from __future__ import annotations

import json
import os
import threading
import time
import traceback
from collections import deque

EVENTS = deque(maxlen=1000)
_lock = threading.Lock()


def track_event(name: str, props=None, measurements=None):
    e = {"ts": time.time(), "event": name, "props": props or {}, "measurements": measurements or {}}
    with _lock:
        EVENTS.append(e)
    path = os.environ.get("DXA_TELEMETRY_FILE")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(e, default=str) + "\n")


def track_exception(location: str, batch_time=None):
    track_event("datax/error", {"errorLocation": location, "batchTime": str(batch_time),
                                "errorStackTrace": traceback.format_exc(limit=10)})
