"""Small shared helpers — the counterparts of the reference's datax-utility module
(DataProcessing/datax-utility/src/main/scala/datax/utility/*.scala):

=====================  ======================================================================
reference              here
=====================  ======================================================================
ArgumentsParser        ``named_args``                     (k=v program arguments)
DataNormalization      ``sanitize_column_name``           (backtick names with . - space ')
GZipHelper             ``deflate_lines`` / ``deflate`` / ``inflate`` / ``inflate_bytes``
GuidUtil               ``generate_guid``
MapManipulation        ``lowercase_keys`` / ``merge_maps`` / ``add_property``
DataMerger             ``merge_map_of_counts`` / ``flatten_map_of_counts``
DateTimeUtil           ``format_simple``
Validation             ``ensure_not_null`` / ``ensure_not_empty``
FutureUtil             ``fail_fast``
StreamingUtility       ``ip_octet``
ConcurrentDateFormat   ``dxa.ops.strings.py_string_to_timestamp_us`` (device: ``to_timestamp``)
CSVUtil                ``dxa.io.refdata.load_csv``
DataGenerator          ``dxa.simulate.datagen`` (GPU + bit-identical CPU)
AzureFunctionCaller    ``dxa.udf.http.HttpFunctionUDF``
SinkerUtil             ``dxa.io.sinks``
=====================  ======================================================================
"""
from __future__ import annotations

import base64
import datetime as _dt
import gc
import gzip
import io
import os
import uuid
from concurrent.futures import FIRST_EXCEPTION, Future, wait
from typing import Dict, Iterable, List, Mapping, Optional, Sequence, TypeVar

T = TypeVar("T")


def named_args(args: Iterable[str]) -> Dict[str, str]:
    """``["conf=a.conf", "x=1"]`` → ``{"conf": "a.conf", "x": "1"}`` (first ``=`` splits; others ignored)."""
    out = {}
    for a in args:
        pos = a.find("=")
        if pos > 0:
            out[a[:pos]] = a[pos + 1:]
    return out


def sanitize_column_name(name: str) -> str:
    return f"`{name}`" if any(c in name for c in ".- '") else name


def deflate_lines(lines: Sequence[str]) -> bytes:
    """Newline-joined lines, gzip-compressed (what blob / event hub sinks write)."""
    buf = io.BytesIO()
    with gzip.GzipFile(fileobj=buf, mode="wb") as z:
        for i, l in enumerate(lines):
            if i:
                z.write(b"\n")
            z.write(l.encode())
    return buf.getvalue()


def deflate_bytes(txt: str) -> bytes:
    return gzip.compress(txt.encode())


def deflate(txt: str) -> str:
    return base64.b64encode(deflate_bytes(txt)).decode()


def inflate(deflated_b64: str) -> str:
    return gzip.decompress(base64.b64decode(deflated_b64)).decode()


def inflate_bytes(data: bytes) -> str:
    return gzip.decompress(data).decode()


def generate_guid() -> str:
    return str(uuid.uuid4())


def lowercase_keys(m: Optional[Mapping[str, T]]) -> Optional[Dict[str, T]]:
    return None if m is None else {k.lower(): v for k, v in m.items()}


def merge_maps(a: Optional[Mapping], b: Optional[Mapping]) -> Optional[Dict]:
    if a is None:
        return None if b is None else dict(b)
    if b is None:
        return dict(a)
    return {**a, **b}


def add_property(props: Optional[Mapping[str, str]], key: str, value: Optional[str]) -> Optional[Dict[str, str]]:
    if value is None:
        return None if props is None else dict(props)
    return {**(props or {}), key: value}


def merge_map_of_counts(a: Mapping[str, int], b: Mapping[str, int]) -> Dict[str, int]:
    out = dict(a)
    for k, v in b.items():
        out[k] = out.get(k, 0) + v
    return out


def flatten_map_of_counts(m: Mapping[str, Mapping[str, int]]) -> Dict[str, int]:
    return {f"{k}_{k2}": v for k, sub in m.items() for k2, v in sub.items()}


def format_simple(t: _dt.datetime) -> str:
    return t.strftime("%Y%m%d-%H%M%S")


def ensure_not_null(param, name: str):
    if param is None:
        raise ValueError(f"{name} cannot be null")


def ensure_not_empty(param, name: str):
    if param is None:
        raise ValueError(f"{name} cannot be null")
    if len(param) == 0:
        raise ValueError(f"{name} cannot be empty")


def fail_fast(futures: List[Future]) -> List:
    """Results of all futures, raising the first failure as soon as it happens."""
    done, pending = wait(futures, return_when=FIRST_EXCEPTION)
    for f in done:
        if f.exception() is not None:
            for p in pending:
                p.cancel()
            raise f.exception()
    return [f.result() for f in futures]


def ip_octet(ip: Optional[str], index: int) -> int:
    if not ip:
        return 0
    parts = ip.split(".")
    return int(parts[index]) if len(parts) > index else 0


def settle_gc(gen0_threshold: int = 20_000) -> bool:
    """Before a streaming loop: collect once, move every surviving object (modules, compiled plans, kernel
    wrappers, reference tables' Python shells) to the permanent generation and raise the young-generation
    threshold.  A micro-batch allocates thousands of short-lived Python objects; with the default threshold
    (700) the collector runs many times per batch, and a full collection re-scans the whole start-up heap, which
    shows as a multi-millisecond outlier in ``Latency-Process`` (profiles/gc/)."""
    gc.collect()
    gc.freeze()
    t0, t1, t2 = gc.get_threshold()
    gc.set_threshold(max(t0, gen0_threshold), t1, t2)
    return True
