"""HTTP function UDF (the reference's Azure Function UDF: AzureFunctionHandler.scala:14-65 and
datax-utility/.../AzureFunctionCaller.scala:21-103 — GET/POST, ≤3 string params, 5 retries, pooled clients).

Distinct argument tuples of a batch are called once each, concurrently (20 workers), so a batch of a million rows
with a handful of distinct keys costs a handful of requests."""
from __future__ import annotations

import json
import urllib.parse
import urllib.request
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

_pool = ThreadPoolExecutor(max_workers=20, thread_name_prefix="dxa-http-udf")


class HttpFunctionUDF:
    return_type = "string"

    def __init__(self, endpoint: Optional[str], api: Optional[str], code: Optional[str], method: str,
                 params: List[str], retries: int = 5, timeout: float = 10.0):
        self.url = (endpoint or "").rstrip("/") + "/api/" + (api or "")
        self.code = code
        self.method = (method or "get").lower()
        self.params = params
        self.retries = retries
        self.timeout = timeout

    def call_one(self, args) -> Optional[str]:
        q = dict(zip(self.params, ["" if a is None else str(a) for a in args]))
        if self.code:
            q["code"] = self.code
        last = None
        for _ in range(self.retries):
            try:
                if self.method == "get":
                    req = urllib.request.Request(self.url + "?" + urllib.parse.urlencode(q))
                else:
                    req = urllib.request.Request(self.url + (f"?code={self.code}" if self.code else ""),
                                                 data=json.dumps(q).encode(), method="POST",
                                                 headers={"Content-Type": "application/json"})
                with urllib.request.urlopen(req, timeout=self.timeout) as r:
                    return r.read().decode()
            except Exception as e:  # noqa: BLE001
                last = e
        return None

    def __call__(self, cols, ctx, n, device):
        from ..engine.column import ConstColumn, column_from_pylist
        lists = [c.to_pylist() if not isinstance(c, ConstColumn) else [c.value] * n for c in cols]
        rows = [tuple(l[i] for l in lists) for i in range(n)]
        uniq = list(dict.fromkeys(rows))
        results = dict(zip(uniq, _pool.map(self.call_one, uniq)))
        return column_from_pylist([results[r] for r in rows], "string", device)
