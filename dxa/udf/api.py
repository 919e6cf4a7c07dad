"""Plugin contracts (the reference's extension API, DataProcessing/datax-core/src/main/scala/datax/extension/
DynamicUDF.scala:12-46, PreProjectionProcessor.scala:10-12, StringNormalizer.scala:10-12, and Spark's
UDF1..UDF22 / UserDefinedAggregateFunction used by jar UDFs).

There is no JVM: a flow names Python classes (``module:Class`` or the reference's ``datax.sample…`` class names, which
map onto the ports in ``dxa.udf.samples``).  Three granularities, fastest first:

* ``VectorUDF``  — ``evaluate(columns, ctx) → Column`` on whole device columns (torch ops / HIP kernels);
* ``RowUDF``     — ``call(*values)`` per row, evaluated host-side (the Spark UDF1 contract; convenient, slow path);
* ``DynamicUDF`` — a ``Generator`` returning a RowUDF/VectorUDF plus ``on_interval(batch_time)`` refreshed once per
  batch before processing (``DynamicUDF.onInterval``);
* ``UDAF``       — ``initialize() / update(buf, *values) / merge(buf, other) / evaluate(buf)`` per group (host-side),
  or override ``aggregate(columns, groups, ctx)`` for a device implementation.
"""
from __future__ import annotations

from typing import Any, Callable, List, Optional

import torch


class VectorUDF:
    return_type = "string"

    def evaluate(self, cols, ctx):
        raise NotImplementedError

    def __call__(self, cols, ctx, n, device):
        return self.evaluate(cols, ctx)


class RowUDF:
    """Spark ``UDF1..N``-style scalar function evaluated row by row."""
    return_type = "string"
    null_safe = False

    def call(self, *args):
        raise NotImplementedError

    def __call__(self, cols, ctx, n, device):
        from ..engine.column import ConstColumn, column_from_pylist
        lists = [c.to_pylist() if not isinstance(c, ConstColumn) else [c.value] * n for c in cols]
        out = []
        for i in range(n):
            vals = [l[i] for l in lists]
            if not self.null_safe and any(v is None for v in vals) and vals:
                out.append(None)
                continue
            out.append(self.call(*vals))
        return column_from_pylist(out, self.return_type, device)


class FunctionUDF(RowUDF):
    def __init__(self, fn: Callable, return_type: str = "string", null_safe: bool = False):
        self.fn = fn
        self.return_type = return_type
        self.null_safe = null_safe

    def call(self, *args):
        return self.fn(*args)


class Generator:
    """DynamicUDF generator: ``initialize(settings) → (udf, on_interval or None)``."""

    def initialize(self, settings):
        raise NotImplementedError


class UDAF:
    return_type = "string"

    def initialize(self) -> Any:
        return None

    def update(self, buf, *values):
        raise NotImplementedError

    def merge(self, buf, other):
        raise NotImplementedError

    def evaluate(self, buf):
        return buf

    def aggregate(self, cols, groups, ctx):
        from ..engine.column import column_from_pylist
        lists = [c.to_pylist() for c in cols]
        gid = groups.gid.cpu().tolist()
        bufs = [self.initialize() for _ in range(groups.ngroups)]
        for i, g in enumerate(gid):
            bufs[g] = self.update(bufs[g], *[l[i] for l in lists])
        return column_from_pylist([self.evaluate(b) for b in bufs], self.return_type, groups.rep.device)


class StringNormalizer:
    """Raw-event normaliser applied before JSON parsing (``datax.job.process.inputnormalizer``,
    InputNormalizerHandler.scala).  A ``byte_map()`` (256 entries) runs as the device byte-map kernel over the whole
    raw batch in one pass; otherwise ``normalize(str)`` is applied per event on the host (re-framed afterwards)."""

    def byte_map(self) -> Optional[List[int]]:
        return None

    def normalize(self, s: str) -> str:
        return s

    def __call__(self, buf: torch.Tensor, offs: torch.Tensor):
        """Normalise a framed raw batch → (buf, offs)."""
        m = self.byte_map()
        if m is not None:
            return apply_byte_map(buf, m), offs
        data = bytes(buf.cpu().numpy())
        o = offs.cpu().tolist()
        recs = [self.normalize(data[o[i]:o[i + 1]].decode("utf-8", "replace")).encode() for i in range(len(o) - 1)]
        from ..ops.jsonparse import frame_records
        return frame_records(recs, device=buf.device)


def apply_byte_map(buf: torch.Tensor, table: List[int]) -> torch.Tensor:
    lut = torch.tensor(table, dtype=torch.uint8)
    if buf.is_cuda:
        from ..ops import native as N
        out = torch.empty_like(buf)
        lut = lut.to(buf.device)
        try:
            N.call("dxa_byte_map", N.ptr(buf), N.ptr(out), buf.numel(), N.ptr(lut), N.stream_handle(buf.device))
            return out
        except N.NativeError:          # unaligned view: fall through to the tensor-op path
            pass
    return lut.to(buf.device)[buf.long()]


class PreProjectionProcessor:
    def process(self, table, ctx):
        return table
