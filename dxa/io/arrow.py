"""Columnar Table ⇄ Arrow conversion without per-row Python objects (state-table Parquet files, Parquet sinks).

Primitive columns move as one D2H copy + a validity bitmap; strings as (offsets, bytes) buffers after a device-side
compaction; nested columns fall back to Python values (rare for accumulators)."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from ..engine.column import ConstColumn, PrimColumn, StrColumn, Table, materialize
from ..engine.types import StructType


def _pa():
    import pyarrow as pa
    return pa


_PA_TYPES = {"long": "int64", "int": "int64", "double": "float64", "float": "float64", "boolean": "bool_",
             "timestamp": None, "date": None, "string": "string"}


def _pa_type(dtype):
    pa = _pa()
    if dtype == "timestamp":
        return pa.timestamp("us")
    if dtype == "date":
        return pa.date32()
    name = _PA_TYPES.get(dtype)
    return getattr(pa, name)() if name else None


def column_to_arrow(col, dtype):
    pa = _pa()
    col = materialize(col)
    n = col.length
    valid = None
    if col.valid is not None:
        valid = col.valid.detach().cpu().numpy().astype(bool)
    mask = None if valid is None else ~valid
    if isinstance(col, StrColumn):
        c = col.compact()
        offs = np.zeros(n + 1, dtype=np.int64)
        if n:
            offs[1:] = np.cumsum(c.lens.detach().cpu().numpy().astype(np.int64))
        data = c.arena.detach().cpu().numpy()[: int(offs[-1])].tobytes()
        bitmap = None
        if valid is not None:
            bitmap = pa.py_buffer(np.packbits(valid, bitorder="little").tobytes())
        return pa.Array.from_buffers(pa.large_string(), n, [bitmap, pa.py_buffer(offs.tobytes()),
                                                             pa.py_buffer(data)],
                                     null_count=-1 if valid is not None else 0).cast(pa.string())
    if isinstance(col, PrimColumn):
        t = _pa_type(dtype if isinstance(dtype, str) else col.dtype)
        if t is None:
            raise TypeError(dtype)
        arr = col.data.detach().cpu().numpy()
        if dtype == "boolean":
            arr = arr.astype(bool)
        elif dtype == "date":
            arr = arr.astype(np.int32)
        return pa.array(arr, type=t, mask=mask)
    # nested: python values
    return pa.array(col.to_pylist())


def table_to_arrow(t: Table, schema: Optional[StructType] = None):
    pa = _pa()
    fields = schema.fields if schema is not None else None
    names, arrays = [], []
    if fields is None:
        for n, c in zip(t.names, t.columns):
            names.append(n)
            arrays.append(column_to_arrow(c, c.dtype))
    else:
        for f in fields:
            c = t.column(f.name)
            names.append(f.name)
            if c is None:
                arrays.append(pa.nulls(t.length, type=_pa_type(f.dtype) or pa.null()))
            elif isinstance(f.dtype, str):
                arrays.append(column_to_arrow(c, f.dtype))
            else:
                arrays.append(pa.array(materialize(c).to_pylist()))
    return pa.Table.from_arrays(arrays, names=names)


def table_from_arrow(at, schema: StructType, device) -> Table:
    """Arrow table → device Table (primitive + string columns columnar; others via Python values)."""
    from ..engine.column import column_from_pylist
    device = torch.device(device)
    cols = []
    for f in schema.fields:
        if f.name not in at.column_names:
            cols.append(ConstColumn(None, f.dtype, at.num_rows, device))
            continue
        a = at.column(f.name).combine_chunks()
        dt = f.dtype
        valid = None
        if a.null_count:
            valid = torch.from_numpy(np.asarray(a.is_valid().to_numpy(zero_copy_only=False), dtype=bool)).to(device)
        if dt in ("long", "int", "double", "float", "boolean", "timestamp", "date"):
            if dt == "timestamp":
                np_arr = a.cast(_pa().int64()).fill_null(0).to_numpy()
            elif dt == "date":
                np_arr = a.cast(_pa().int32()).fill_null(0).to_numpy().astype(np.int64)
            elif dt == "boolean":
                np_arr = a.fill_null(False).to_numpy(zero_copy_only=False).astype(bool)
            else:
                np_arr = a.fill_null(0).to_numpy()
                np_arr = np_arr.astype(np.float64 if dt in ("double", "float") else np.int64)
            cols.append(PrimColumn(dt, torch.from_numpy(np.array(np_arr, copy=True)).to(device), valid))
        else:
            cols.append(column_from_pylist(a.to_pylist(), dt, device))
    return Table([f.name for f in schema.fields], cols, at.num_rows, device)


def to_host_async(t: Table):
    """Start copying a device table to pinned host memory on the current stream → (host Table, event or None).
    The host table may only be read after ``event.synchronize()``.

    Every leaf buffer (data, validity, string arena / starts / lengths) is packed into one device staging buffer by
    one concatenation launch (widest elements first, so every host view stays aligned) and crosses PCIe as ONE
    copy, instead of a copy per buffer."""
    from ..engine.column import column_from_pylist
    if t.device.type != "cuda":
        return t, None
    leaves: list = []                       # device tensors to ship

    def leaf(x):
        leaves.append(x.detach().contiguous())
        return len(leaves) - 1

    plan = []
    for c in t.columns:
        c = materialize(c)
        if isinstance(c, StrColumn):
            # a small arena crosses as it is (the host side packs the strings when it builds Arrow): no device
            # compaction, whose size read would stall the batch thread; a view into a large buffer (a batch's raw
            # input) is compacted first so only its rows' bytes cross PCIe
            small = c.arena.numel() <= max(1 << 20, 512 * c.length)
            cc = c if small else c.compact()
            plan.append(("str", type(cc), cc.dtype, leaf(cc.arena), leaf(cc.starts), leaf(cc.lens),
                         None if cc.valid is None else leaf(cc.valid)))
        elif isinstance(c, PrimColumn):
            plan.append(("prim", c.dtype, leaf(c.data), None if c.valid is None else leaf(c.valid)))
        else:                                   # nested: synchronous Python round trip (rare)
            plan.append(("host", column_from_pylist(c.to_pylist(), c.dtype, "cpu")))
    order = sorted(range(len(leaves)), key=lambda i: -leaves[i].element_size())
    offs, pos = {}, 0
    for i in order:
        offs[i] = pos
        pos += leaves[i].numel() * leaves[i].element_size()
    host_buf = torch.empty(max(pos, 1), dtype=torch.uint8, pin_memory=True)
    keep: list = []
    if pos:
        staged = torch.cat([leaves[i].view(torch.uint8).reshape(-1) for i in order])
        host_buf[:pos].copy_(staged, non_blocking=True)
        keep.append(staged)

    def view(i):
        x = leaves[i]
        nb = x.numel() * x.element_size()
        return host_buf[offs[i]:offs[i] + nb].view(x.dtype).view(x.shape)

    cols = []
    for p in plan:
        if p[0] == "str":
            _, typ, dt, a, st, ln, v = p
            cols.append(typ(view(a), view(st), view(ln), None if v is None else view(v), dt))
        elif p[0] == "prim":
            _, dt, d, v = p
            cols.append(PrimColumn(dt, view(d), None if v is None else view(v)))
        else:
            cols.append(p[1])
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))
    host = Table(list(t.names), cols, t.length, "cpu")
    host._keep = keep + [host_buf]
    return host, ev
