"""Row → JSON text with Spark ``to_json(struct(*))`` semantics (reference: DataProcessing/datax-host/src/main/scala/
datax/sink/OutputManager.scala:116-118): field order = column order, null struct fields omitted, doubles in Java
``Double.toString`` form, timestamps as ``yyyy-MM-dd'T'HH:mm:ss.SSSZ`` (UTC), ``filterNull`` arrays skip nulls.

``table_to_json_lines`` is the host formatter used for low-volume outputs (metrics, alerts, aggregates); large
outputs go through the device serializer in ``dxa.ops.serialize`` when available.
"""
from __future__ import annotations

import datetime as _dt
import json
from typing import Any, List, Optional

from . import functions as F
from .decimal import is_decimal, render, to_text_values
from .column import (ArrayColumn, Column, ConstColumn, JsonColumn, PrimColumn, StrColumn, StructColumn, Table,
                     datetime_to_us)
from .types import ArrayType, MapType, StructType


def _jstr(s: str) -> str:
    return json.dumps(s, ensure_ascii=False)


def json_value(v: Any, dtype) -> Any:
    """Python value → JSON-compatible value (for json.dumps)."""
    if v is None:
        return None
    if dtype == "timestamp" and isinstance(v, _dt.datetime):
        return F.format_timestamp_us(datetime_to_us(v))
    if dtype == "date" and isinstance(v, _dt.date):
        return v.isoformat()
    return v


def _frag_values(col: Column) -> List[Optional[str]]:
    """Per-row JSON text of a column's value (None = null)."""
    n = col.length
    if isinstance(col, ConstColumn):
        if col.value is None:
            return [None] * n
        return [_scalar_text(col.value, col.dtype, raw=True)] * n
    if isinstance(col, JsonColumn):
        arena = col.arena.cpu().numpy().tobytes()
        valid = col.valid.cpu().tolist() if col.valid is not None else [True] * n
        return [arena[s:s + l].decode("utf-8", "replace") if ok else None
                for s, l, ok in zip(col.starts.cpu().tolist(), col.lens.cpu().tolist(), valid)]
    if isinstance(col, StrColumn):
        return [None if v is None else _jstr(v) for v in col.to_pylist()]
    if isinstance(col, PrimColumn) and is_decimal(col.dtype):
        return to_text_values(col)
    if isinstance(col, PrimColumn):
        valid = col.valid.cpu().tolist() if col.valid is not None else [True] * n
        data = col.data.cpu().tolist()
        dt = col.dtype
        if dt == "boolean":
            fmt = lambda v: "true" if v else "false"
        elif dt in ("byte", "short", "int", "long"):
            fmt = str
        elif dt == "timestamp":
            fmt = lambda v: '"' + F.format_timestamp_us(v) + '"'
        elif dt == "date":
            fmt = lambda v: '"' + (_dt.date(1970, 1, 1) + _dt.timedelta(days=int(v))).isoformat() + '"'
        else:
            fmt = _double_text
        return [fmt(v) if ok else None for v, ok in zip(data, valid)]
    if isinstance(col, StructColumn):
        kids = [(_jstr(nm), _frag_values(c)) for nm, c in zip(col.names, col.children)]
        valid = col.valid.cpu().tolist() if col.valid is not None else [True] * n
        out = []
        for i in range(n):
            if not valid[i]:
                out.append(None)
                continue
            parts = []
            for nm, vals in kids:
                v = vals[i]
                if v is None:
                    if col.is_map:
                        parts.append(f"{nm}:null")
                    continue
                parts.append(f"{nm}:{v}")
            out.append("{" + ",".join(parts) + "}")
        return out
    if isinstance(col, ArrayColumn):
        els = [_frag_values(e) for e in col.elements]
        valid = col.valid.cpu().tolist() if col.valid is not None else [True] * n
        pres = col.present.cpu().tolist() if col.present is not None else None
        out = []
        for i in range(n):
            if not valid[i]:
                out.append(None)
                continue
            parts = [e[i] for j, e in enumerate(els) if pres is None or pres[i][j]]
            if col.drop_nulls:
                parts = [p for p in parts if p is not None]
            else:
                parts = ["null" if p is None else p for p in parts]
            out.append("[" + ",".join(parts) + "]")
        return out
    raise TypeError(f"cannot serialise {col!r}")


def _double_text(v: float) -> str:
    if v != v or v in (float("inf"), float("-inf")):
        return '"' + F.java_double_str(v) + '"'
    return F.java_double_str(v)


def _scalar_text(v, dtype, raw=True) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if dtype == "timestamp":
        return '"' + F.format_timestamp_us(v) + '"'
    if dtype == "date":
        return '"' + (_dt.date(1970, 1, 1) + _dt.timedelta(days=int(v))).isoformat() + '"'
    if is_decimal(dtype):
        return render(v, dtype.scale)
    if isinstance(v, float) or dtype in ("double", "float", "decimal"):
        return _double_text(float(v))
    if isinstance(v, int):
        return str(v)
    if isinstance(v, (dict, list)):
        return json.dumps(v, separators=(",", ":"))
    return _jstr(str(v))


def column_json_values(col: Column) -> List[Optional[str]]:
    """JSON text of each value (used by to_json(), CAST(struct AS STRING), nested-key hashing)."""
    return _frag_values(col)


def table_to_json_lines(t: Table) -> List[str]:
    from ..ops import serialize as native_ser
    if native_ser.available():
        return native_ser.table_lines(t)
    return table_to_json_lines_py(t)


def table_to_json_lines_py(t: Table) -> List[str]:
    cols = [(_jstr(nm), _frag_values(c)) for nm, c in zip(t.names, t.columns)]
    out = []
    for i in range(t.length):
        parts = []
        for nm, vals in cols:
            v = vals[i]
            if v is not None:
                parts.append(f"{nm}:{v}")
        out.append("{" + ",".join(parts) + "}")
    return out
