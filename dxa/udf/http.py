"""HTTP function UDF (the reference's Azure Function UDF: AzureFunctionHandler.scala:14-65 and
datax-utility/.../AzureFunctionCaller.scala:21-103 — GET/POST, ≤3 string params, 5 retries, pooled clients).

Distinct argument tuples of a batch are found on the device (the group-by hash kernels: ``ops.groupby.group_rows``),
only their representative rows come to the host, and each is called once, concurrently (20 workers) — a batch of a
million rows with a handful of distinct keys costs a handful of requests and a handful of host values.  The results
are scattered back by group id on the device.

Every call of a batch shares one deadline (``budget_s``, default 30 s): retries back off exponentially (0.1 s, 0.2 s,
…) but never past it, so five retries against a dead endpoint cannot stall a micro-batch by 5 × timeout per key —
an argument tuple whose calls run out of budget yields null, as an exhausted retry loop does in the reference."""
from __future__ import annotations

import json
import time
import urllib.parse
import urllib.request
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

_pool = ThreadPoolExecutor(max_workers=20, thread_name_prefix="dxa-http-udf")


class HttpFunctionUDF:
    return_type = "string"

    def __init__(self, endpoint: Optional[str], api: Optional[str], code: Optional[str], method: str,
                 params: List[str], retries: int = 5, timeout: float = 10.0, budget_s: float = 30.0):
        self.url = (endpoint or "").rstrip("/") + "/api/" + (api or "")
        self.code = code
        self.method = (method or "get").lower()
        self.params = params
        self.retries = retries
        self.timeout = timeout
        self.budget_s = budget_s

    def call_one(self, args, deadline: Optional[float] = None) -> Optional[str]:
        q = dict(zip(self.params, ["" if a is None else str(a) for a in args]))
        if self.code:
            q["code"] = self.code
        deadline = time.monotonic() + self.budget_s if deadline is None else deadline
        for attempt in range(self.retries):
            left = deadline - time.monotonic()
            if left <= 0:
                break
            if attempt:
                pause = min(0.1 * (1 << (attempt - 1)), left)
                time.sleep(pause)
                left -= pause
                if left <= 0:
                    break
            try:
                if self.method == "get":
                    req = urllib.request.Request(self.url + "?" + urllib.parse.urlencode(q))
                else:
                    req = urllib.request.Request(self.url + (f"?code={self.code}" if self.code else ""),
                                                 data=json.dumps(q).encode(), method="POST",
                                                 headers={"Content-Type": "application/json"})
                with urllib.request.urlopen(req, timeout=min(self.timeout, left)) as r:
                    return r.read().decode()
            except Exception:  # noqa: BLE001 — any failure is retried, as AzureFunctionCaller does
                continue
        return None

    def __call__(self, cols, ctx, n, device):
        from ..engine.column import ConstColumn, column_from_pylist
        from ..ops.groupby import group_rows
        if n == 0:
            return column_from_pylist([], "string", device)
        groups = group_rows(list(cols))
        rep = groups.rep
        uniq_cols = [[c.value] * groups.ngroups if isinstance(c, ConstColumn) else c.take(rep).to_pylist()
                     for c in cols]
        uniq = list(zip(*uniq_cols)) if uniq_cols else [()] * groups.ngroups
        deadline = time.monotonic() + self.budget_s
        results = list(_pool.map(lambda a: self.call_one(a, deadline), uniq))
        return column_from_pylist(results, "string", device).take(groups.gid.long())
