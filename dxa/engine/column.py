"""Device-resident columnar batch model.

The reference processes Spark ``DataFrame`` rows with a nested ``Raw`` struct
(DataProcessing/datax-host/src/main/scala/datax/processor/CommonProcessorFactory.scala:90-103).  Here a batch is a
``Table`` of columns held in HBM as torch tensors (CPU tensors in host-only tests):

* ``PrimColumn``   fixed-width values (bool / int64 / float64 / timestamp-µs) + optional validity mask;
* ``StrColumn``    string *views*: ``starts``/``lens`` into a byte ``arena`` (for parsed input the arena IS the raw
                   JSON buffer already on the device — the parser never copies string bytes);
* ``ConstColumn``  a broadcast literal (``'maxTemperature' AS MetricName``) — never materialised unless needed;
* ``StructColumn`` struct or constant-keyed map (``MAP('ruleId', …)``) with child columns;
* ``ArrayColumn``  fixed-arity array of element columns (``Array(IF(c, MAP(…), NULL), …)``), ``drop_nulls`` gives
                   the reference's ``filterNull`` UDF (DataProcessing/datax-host/src/main/scala/datax/host/
                   UdfInitializer.scala:16-18);
* ``JsonColumn``   raw JSON text of an input map/array value, emitted verbatim on output.

A validity mask of ``None`` means "no nulls".  Every operation is written once against torch so it runs on the
MI355X (HBM tensors, HIP kernels underneath) and on the CPU for reference tests; the hot paths dispatch into the
hand-written kernels in ``dxa.ops``.
"""
from __future__ import annotations

import datetime as _dt
import json
import math
from typing import Any, Dict, Iterable, List, Optional, Sequence

import torch

from .types import (ArrayType, MapType, StructField, StructType, is_integral, is_nested)

EPOCH = _dt.datetime(1970, 1, 1)

TORCH_DTYPE = {
    "boolean": torch.bool, "byte": torch.int64, "short": torch.int64, "int": torch.int64, "long": torch.int64,
    "float": torch.float64,
    "double": torch.float64, "decimal": torch.float64, "timestamp": torch.int64, "date": torch.int64,
    "null": torch.bool,
}


def and_valid(a: Optional[torch.Tensor], b: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if a is None:
        return b
    if b is None:
        return a
    return a & b


def ts_to_datetime(us: int) -> _dt.datetime:
    return EPOCH + _dt.timedelta(microseconds=int(us))


def datetime_to_us(d: _dt.datetime) -> int:
    if d.tzinfo is not None:
        d = d.astimezone(_dt.timezone.utc).replace(tzinfo=None)
    delta = d - EPOCH
    return (delta.days * 86400 + delta.seconds) * 1_000_000 + delta.microseconds


class Column:
    dtype: Any
    length: int
    valid: Optional[torch.Tensor]

    @property
    def device(self) -> torch.device:
        raise NotImplementedError

    def __len__(self):
        return self.length

    def take(self, idx: torch.Tensor) -> "Column":
        raise NotImplementedError

    def filter(self, mask: torch.Tensor) -> "Column":
        return self.take(torch.nonzero(mask, as_tuple=False).flatten())

    def with_valid(self, extra: Optional[torch.Tensor]) -> "Column":
        raise NotImplementedError

    def valid_mask(self) -> torch.Tensor:
        if self.valid is None:
            return torch.ones(self.length, dtype=torch.bool, device=self.device)
        return self.valid

    def null_count(self) -> int:
        return 0 if self.valid is None else int((~self.valid).sum().item())

    def to_pylist(self) -> list:
        raise NotImplementedError

    def to(self, device) -> "Column":
        raise NotImplementedError


def _take_valid(valid, idx):
    return None if valid is None else valid[idx]


def _plan_take(c: "Column", idx: torch.Tensor, leaves: List[torch.Tensor]):
    """Register c's leaf tensors in ``leaves``; return a builder taking the gathered leaves (in registration order).
    Module-level recursion on purpose: a self-referencing nested function is a reference cycle, and this one would
    keep every leaf (the batch's raw input arena included) alive until the cyclic collector ran."""
    if isinstance(c, PrimColumn):
        i = len(leaves)
        leaves.append(c.data)
        if c.valid is not None:
            leaves.append(c.valid)
        has_v = c.valid is not None
        return lambda g: PrimColumn(c.dtype, g[i], g[i + 1] if has_v else None)
    if isinstance(c, StrColumn):
        i = len(leaves)
        leaves.extend([c.starts, c.lens])
        if c.valid is not None:
            leaves.append(c.valid)
        has_v = c.valid is not None
        return lambda g: _with_max_len(type(c)(c.arena, g[i], g[i + 1], g[i + 2] if has_v else None, c.dtype),
                                       c.max_len)
    if isinstance(c, StructColumn):
        i = len(leaves)
        if c.valid is not None:
            leaves.append(c.valid)
        has_v = c.valid is not None
        kids = [_plan_take(k, idx, leaves) for k in c.children]
        n = int(idx.shape[0])
        return lambda g: StructColumn(c.names, [b(g) for b in kids], n, g[i] if has_v else None, c.is_map,
                                      c.dtype, c.device)
    if isinstance(c, ArrayColumn) and c.present is not None:
        taken = c.take(idx)                   # a [rows x slots] presence mask: not a 1-D leaf of the batched gather
        return lambda g: taken
    if isinstance(c, ArrayColumn):
        i = len(leaves)
        if c.valid is not None:
            leaves.append(c.valid)
        has_v = c.valid is not None
        els = [_plan_take(e, idx, leaves) for e in c.elements]
        n = int(idx.shape[0])
        return lambda g: ArrayColumn([b(g) for b in els], n, g[i] if has_v else None, c.drop_nulls, c.device)
    taken = c.take(idx)                       # constants and other kinds: their own take
    return lambda g: taken


def take_columns(cols: Sequence["Column"], idx: torch.Tensor) -> List["Column"]:
    """Row gather of several columns with the same index vector.  On the GPU every leaf tensor (data, validity,
    string starts / lengths, nested validity) moves in one multi-column gather launch (dxa.ops.gather) instead of
    one indexing kernel per leaf; the CPU path is each column's own ``take``."""
    cols = list(cols)
    if idx.device.type != "cuda" or not cols:
        return [c.take(idx) for c in cols]
    leaves: List[torch.Tensor] = []
    builders = [_plan_take(c, idx, leaves) for c in cols]
    if len(leaves) < 2:
        return [c.take(idx) for c in cols]
    if any(t.dim() != 1 or t.shape[0] != leaves[0].shape[0] for t in leaves):
        return [c.take(idx) for c in cols]
    from ..ops.gather import gather_many
    g = gather_many(leaves, idx)
    return [b(g) for b in builders]


class PrimColumn(Column):
    def __init__(self, dtype: str, data: torch.Tensor, valid: Optional[torch.Tensor] = None):
        self.dtype = dtype
        self.data = data
        self.valid = valid
        self.length = int(data.shape[0])

    @property
    def device(self):
        return self.data.device

    def take(self, idx):
        return PrimColumn(self.dtype, self.data[idx], _take_valid(self.valid, idx))

    def with_valid(self, extra):
        return PrimColumn(self.dtype, self.data, and_valid(self.valid, extra))

    def to(self, device):
        return PrimColumn(self.dtype, self.data.to(device), None if self.valid is None else self.valid.to(device))

    def to_pylist(self):
        from .decimal import is_decimal, to_python
        if is_decimal(self.dtype):
            return to_python(self)
        vals = self.data.cpu().tolist()
        valid = self.valid.cpu().tolist() if self.valid is not None else None
        if valid is not None:
            vals = [v if ok else None for v, ok in zip(vals, valid)]      # values under a null are undefined bytes
        if self.dtype == "timestamp":
            vals = [None if v is None else ts_to_datetime(v) for v in vals]
        elif self.dtype == "date":
            vals = [None if v is None else (EPOCH + _dt.timedelta(days=int(v))).date() for v in vals]
        return vals

    def __repr__(self):
        return f"PrimColumn({self.dtype}, n={self.length})"


def _with_max_len(c, m):
    if m is not None:
        c.max_len = m
    return c


class StrColumn(Column):
    dtype = "string"
    # a known bound on every row's byte length (None: unknown).  Rows viewing a window dictionary's fixed-width key
    # slots have one; it survives gathers and concatenations, so their string bytes can be sized on the host
    # without reading the exact total back (strings.concat_multi)
    max_len: Optional[int] = None

    def __init__(self, arena: torch.Tensor, starts: torch.Tensor, lens: torch.Tensor,
                 valid: Optional[torch.Tensor] = None, dtype: Any = "string"):
        self.arena = arena          # uint8
        self.starts = starts        # int64
        self.lens = lens            # int32
        self.valid = valid
        self.length = int(starts.shape[0])
        self.dtype = dtype
        self._hash = None

    @property
    def device(self):
        return self.starts.device

    def take(self, idx):
        c = type(self)(self.arena, self.starts[idx], self.lens[idx], _take_valid(self.valid, idx), self.dtype)
        return _with_max_len(c, self.max_len)

    def with_valid(self, extra):
        c = type(self)(self.arena, self.starts, self.lens, and_valid(self.valid, extra), self.dtype)
        c._hash = self._hash
        return _with_max_len(c, self.max_len)

    def to(self, device):
        c = self.compact()
        return type(self)(c.arena.to(device), c.starts.to(device), c.lens.to(device),
                          None if c.valid is None else c.valid.to(device), self.dtype)

    def byte_size(self) -> int:
        return int(self.lens.sum().item()) if self.length else 0

    def compact(self) -> "StrColumn":
        """Copy the referenced bytes into a fresh, densely packed arena (used before retaining / concatenating)."""
        from ..ops import strings as sops
        return sops.compact(self)

    def to_pylist(self):
        if self.arena.numel() > 4 * self.length * 64 + 4096 and not getattr(self, "_compact", False):
            return self.compact().to_pylist()     # never copy a whole raw-input arena to the host
        arena = self.arena.cpu().numpy().tobytes()
        starts = self.starts.cpu().tolist()
        lens = self.lens.cpu().tolist()
        valid = self.valid.cpu().tolist() if self.valid is not None else [True] * self.length
        if self.dtype == "binary":
            return [arena[s:s + l] if ok else None for s, l, ok in zip(starts, lens, valid)]
        out = []
        for s, l, ok in zip(starts, lens, valid):
            out.append(arena[s:s + l].decode("utf-8", errors="replace") if ok else None)
        return out

    def __repr__(self):
        return f"StrColumn(n={self.length})"


class JsonColumn(StrColumn):
    """Raw JSON text of a nested input value (map / array / struct-as-string); serialised verbatim."""

    def to_pylist(self):
        return [None if s is None else json.loads(s) for s in super().to_pylist()]


class ConstColumn(Column):
    def __init__(self, value: Any, dtype: Any, length: int, device):
        self.value = value
        self.dtype = dtype
        self.length = int(length)
        self._device = torch.device(device)
        self.valid = None if value is not None else torch.zeros(self.length, dtype=torch.bool, device=self._device)

    @property
    def device(self):
        return self._device

    def take(self, idx):
        return ConstColumn(self.value, self.dtype, int(idx.shape[0]), self._device)

    def with_valid(self, extra):
        if extra is None:
            return self
        return self.materialize().with_valid(extra)

    def to(self, device):
        return ConstColumn(self.value, self.dtype, self.length, device)

    def materialize(self) -> Column:
        return column_from_pylist([self.value] * self.length, self.dtype, self._device) if self.dtype in (
            "string",) or is_nested(self.dtype) else _const_prim(self.value, self.dtype, self.length, self._device)

    def to_pylist(self):
        v = self.value
        if self.dtype == "timestamp" and v is not None:
            v = ts_to_datetime(v)
        elif self.dtype == "date" and isinstance(v, int) and not isinstance(v, bool):
            v = (EPOCH + _dt.timedelta(days=v)).date()
        return [v] * self.length

    def __repr__(self):
        return f"ConstColumn({self.value!r}, {self.dtype}, n={self.length})"


def _const_prim(value, dtype, n, device):
    from .decimal import const_column, is_decimal
    if is_decimal(dtype):
        return const_column(value, dtype, n, device)
    tdt = TORCH_DTYPE.get(dtype, torch.float64)
    if value is None:
        return PrimColumn(dtype, torch.zeros(n, dtype=tdt, device=device), torch.zeros(n, dtype=torch.bool,
                                                                                         device=device))
    return PrimColumn(dtype, torch.full((n,), value, dtype=tdt, device=device))


class StructColumn(Column):
    """Struct, or (``is_map``) a map whose keys are the constant child names."""

    def __init__(self, names: List[str], children: List[Column], length: int, valid=None, is_map=False,
                 dtype=None, device=None):
        self.names = list(names)
        self.children = list(children)
        self.length = int(length)
        self.valid = valid
        self.is_map = is_map
        self._device = torch.device(device) if device is not None else (
            children[0].device if children else torch.device("cpu"))
        if dtype is None:
            if is_map:
                vt = children[0].dtype if children else "string"
                dtype = MapType("string", vt)
            else:
                dtype = StructType(tuple(StructField(n, c.dtype) for n, c in zip(names, children)))
        self.dtype = dtype

    @property
    def device(self):
        return self._device

    def child(self, name: str) -> Optional[Column]:
        for n, c in zip(self.names, self.children):
            if n == name:
                return c
        low = name.lower()
        if not self.is_map:
            for n, c in zip(self.names, self.children):
                if n.lower() == low:
                    return c
        return None

    def take(self, idx):
        # children through one batched gather on the GPU (take_columns); never take_columns([self]) here: its
        # fallback for a layout it cannot batch is this method
        return StructColumn(self.names, take_columns(self.children, idx), int(idx.shape[0]),
                            _take_valid(self.valid, idx), self.is_map, self.dtype, self._device)

    def with_valid(self, extra):
        return StructColumn(self.names, self.children, self.length, and_valid(self.valid, extra), self.is_map,
                            self.dtype, self._device)

    def to(self, device):
        return StructColumn(self.names, [c.to(device) for c in self.children], self.length,
                            None if self.valid is None else self.valid.to(device), self.is_map, self.dtype, device)

    def to_pylist(self):
        cols = [c.to_pylist() for c in self.children]
        valid = self.valid.cpu().tolist() if self.valid is not None else [True] * self.length
        out = []
        for i in range(self.length):
            if not valid[i]:
                out.append(None)
                continue
            d = {}
            for n, col in zip(self.names, cols):
                if self.is_map or col[i] is not None or True:
                    d[n] = col[i]
            out.append(d)
        return out

    def __repr__(self):
        return f"StructColumn({'map' if self.is_map else 'struct'} {self.names}, n={self.length})"


class ArrayColumn(Column):
    """K element slots per row.  A row's array is its PRESENT slots, left to right: every slot, unless
    ``drop_nulls`` (null slots are absent) or a ``present`` mask [rows × K] says otherwise — arrays of different
    lengths in one column (``IF(c, array(1), array(2, 3))``, unions) keep their own lengths that way."""

    def __init__(self, elements: List[Column], length: int, valid=None, drop_nulls=False, device=None,
                 present: Optional[torch.Tensor] = None):
        self.elements = list(elements)
        self.length = int(length)
        self.valid = valid
        self.drop_nulls = drop_nulls
        self.present = present
        self._device = torch.device(device) if device is not None else (
            elements[0].device if elements else torch.device("cpu"))
        et = elements[0].dtype if elements else "null"
        self.dtype = ArrayType(et)

    @property
    def device(self):
        return self._device

    def canonical(self) -> Optional["ArrayColumn"]:
        """The same arrays without a ``present`` mask: absent slots become null slots of a ``drop_nulls`` array —
        exact unless a present slot holds a real null element (then None: the caller renders on the host)."""
        if self.present is None:
            return self
        els = []
        for j, e in enumerate(self.elements):
            e = materialize(e)
            p = self.present[:, j]
            if not self.drop_nulls and bool((p & ~e.valid_mask()).any()):
                return None
            els.append(e.with_valid(p))
        return ArrayColumn(els, self.length, self.valid, True, self._device)

    def slot_present(self, j: int) -> Optional[torch.Tensor]:
        """Presence of slot j per row from the ``present`` mask (None: every row has it)."""
        return None if self.present is None else self.present[:, j]

    def take(self, idx):
        return ArrayColumn(take_columns(self.elements, idx), int(idx.shape[0]), _take_valid(self.valid, idx),
                           self.drop_nulls, self._device,
                           present=None if self.present is None else self.present[idx])

    def with_valid(self, extra):
        return ArrayColumn(self.elements, self.length, and_valid(self.valid, extra), self.drop_nulls, self._device,
                           present=self.present)

    def to(self, device):
        return ArrayColumn([e.to(device) for e in self.elements], self.length,
                           None if self.valid is None else self.valid.to(device), self.drop_nulls, device,
                           present=None if self.present is None else self.present.to(device))

    def to_pylist(self):
        els = [e.to_pylist() for e in self.elements]
        valid = self.valid.cpu().tolist() if self.valid is not None else [True] * self.length
        pres = self.present.cpu().tolist() if self.present is not None else None
        out = []
        for i in range(self.length):
            if not valid[i]:
                out.append(None)
                continue
            if pres is not None:
                row = [col[i] for j, col in enumerate(els) if pres[i][j]]
                if self.drop_nulls:
                    row = [v for v in row if v is not None]
                out.append(row)
                continue
            row = [col[i] for col in els]
            if self.drop_nulls:
                row = [v for v in row if v is not None]
            out.append(row)
        return out


# ----------------------------------------------------------------------------------------------------------------
# Construction helpers
# ----------------------------------------------------------------------------------------------------------------

def strings_from_pylist(values: Sequence[Optional[str]], device, dtype="string") -> StrColumn:
    enc = [b"" if v is None else (v if isinstance(v, bytes) else str(v).encode("utf-8")) for v in values]
    lens = [len(b) for b in enc]
    starts = [0] * len(enc)
    acc = 0
    for i, l in enumerate(lens):
        starts[i] = acc
        acc += l
    blob = b"".join(enc)
    arena = _h2d(blob + b"\0" * 16, torch.uint8, device)
    valid = None
    if any(v is None for v in values):
        valid = _h2d([v is not None for v in values], torch.bool, device)
    cls = JsonColumn if dtype != "string" else StrColumn
    return cls(arena, _h2d(starts, torch.int64, device),
               _h2d(lens, torch.int32, device), valid, dtype)


def _py_to_storage(v, dtype):
    if v is None:
        return 0
    if dtype == "timestamp":
        if isinstance(v, _dt.datetime):
            return datetime_to_us(v)
        return int(v)
    if dtype == "date":
        if isinstance(v, _dt.date):
            return (v - EPOCH.date()).days
        return int(v)
    if dtype == "boolean":
        return bool(v)
    if dtype in ("byte", "short", "int", "long"):
        return int(v)
    return float(v)


def column_from_pylist(values: Sequence[Any], dtype: Any, device="cpu") -> Column:
    n = len(values)
    if dtype == "string":
        return strings_from_pylist(values, device)
    if isinstance(dtype, StructType):
        names = [f.name for f in dtype.fields]
        children = [column_from_pylist([None if v is None else v.get(f.name) for v in values], f.dtype, device)
                    for f in dtype.fields]
        valid = None
        if any(v is None for v in values):
            valid = _h2d([v is not None for v in values], torch.bool, device)
        return StructColumn(names, children, n, valid, False, dtype, device)
    if isinstance(dtype, (MapType, ArrayType)):
        return strings_from_pylist([None if v is None else json.dumps(v, separators=(",", ":")) for v in values],
                                   device, dtype)
    if dtype == "null":
        return ConstColumn(None, "null", n, device)
    from .decimal import from_python, is_decimal
    if is_decimal(dtype):
        return from_python(values, dtype, device)
    tdt = TORCH_DTYPE[dtype]
    data = _h2d([_py_to_storage(v, dtype) for v in values], tdt, device)
    valid = None
    if any(v is None or (isinstance(v, float) and dtype == "null") for v in values):
        valid = _h2d([v is not None for v in values], torch.bool, device)
    return PrimColumn(dtype, data, valid)


def empty_column(dtype, device) -> Column:
    return column_from_pylist([], dtype, device)


def materialize(col: Column) -> Column:
    return col.materialize() if isinstance(col, ConstColumn) else col


def _null_like(col, n: int):
    """An all-null column shaped like array / struct column ``col`` (same element / field layout)."""
    dev = col.device
    none = torch.zeros(n, dtype=torch.bool, device=dev)
    if isinstance(col, ArrayColumn):
        return ArrayColumn([], n, none, col.drop_nulls, dev, present=torch.zeros((n, 0), dtype=torch.bool,
                                                                                     device=dev))
    return StructColumn(col.names, [ConstColumn(None, c.dtype, n, dev) for c in col.children], n, none, col.is_map,
                        col.dtype, dev)


def concat_columns(cols: List[Column]) -> Column:
    """Row-wise concatenation (UNION ALL, window unions).  Types must already agree."""
    cols = [c for c in cols]
    if len(cols) == 1:
        return cols[0]
    n = sum(c.length for c in cols)
    device = cols[0].device
    if all(isinstance(c, ConstColumn) for c in cols) and len({(repr(c.value), str(c.dtype)) for c in cols}) == 1:
        return ConstColumn(cols[0].value, cols[0].dtype, n, device)
    shaped = next((c for c in cols if isinstance(c, (ArrayColumn, StructColumn))), None)
    if shaped is not None:
        # a NULL literal next to arrays / structs (IF(c, array(1), NULL), a CASE's missing ELSE): an all-null
        # column of the same shape, not a JSON text column
        cols = [_null_like(shaped, c.length) if (isinstance(c, ConstColumn) and c.value is None) else c
                for c in cols]
    cols = [materialize(c) for c in cols]
    any_null = any(c.valid is not None for c in cols)
    valid = torch.cat([c.valid_mask() for c in cols]) if any_null else None
    first = cols[0]
    if isinstance(first, StrColumn):
        from ..ops import strings as sops
        return sops.concat([c if isinstance(c, StrColumn) else c for c in cols], valid)
    if isinstance(first, PrimColumn):
        dt = first.dtype
        datas = []
        for c in cols:
            d = c.data
            if d.dtype != first.data.dtype:
                d = d.to(first.data.dtype)
            datas.append(d)
        return PrimColumn(dt, torch.cat(datas), valid)
    if isinstance(first, StructColumn):
        names = first.names
        children = []
        for i, nm in enumerate(names):
            children.append(concat_columns([c.child(nm) if c.child(nm) is not None else
                                            ConstColumn(None, first.children[i].dtype, c.length, device)
                                            for c in cols]))
        return StructColumn(names, children, n, valid, first.is_map, first.dtype, device)
    if isinstance(first, ArrayColumn):
        k = max(len(c.elements) for c in cols)
        et = next((c.elements[0].dtype for c in cols if c.elements), "null")
        elements = []
        for j in range(k):
            parts = []
            for c in cols:
                if j < len(c.elements):
                    parts.append(c.elements[j])
                else:
                    parts.append(ConstColumn(None, et, c.length, device))
            elements.append(concat_columns(parts))
        present = None
        if any(len(c.elements) != k or c.present is not None for c in cols):
            # a shorter array's missing slots are absent, not null elements
            pm = []
            for c in cols:
                p = torch.zeros((c.length, k), dtype=torch.bool, device=device)
                if c.present is not None:
                    p[:, :len(c.elements)] = c.present
                else:
                    p[:, :len(c.elements)] = True
                pm.append(p)
            present = torch.cat(pm)
        return ArrayColumn(elements, n, valid, first.drop_nulls, device, present=present)
    raise TypeError(f"cannot concat {type(first)}")


class LazyColumns(list):
    """A column list whose entries are produced on first access (``_make(i)``).  Tables and scopes keep such a list
    as is, so a view whose columns a consumer never reads never pays for them (e.g. ``SELECT * … WHERE`` feeding
    an alert that only needs the row count).  Iteration and indexing resolve entries; the list's own slots hold
    ``None`` until then, so list-internal operations (``+``, ``.copy()``) must not be used on it."""

    def _make(self, i):
        raise NotImplementedError

    def prefetch(self, idxs) -> None:
        """Resolve several entries together (subclasses batch their gathers into one launch); the default resolves
        them one by one."""
        for i in idxs:
            self[i]

    def _unresolved(self, idxs):
        return [i for i in dict.fromkeys(idxs) if 0 <= i < len(self) and list.__getitem__(self, i) is None]

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        v = list.__getitem__(self, i)
        if v is None:
            v = self._make(i)
            list.__setitem__(self, i, v)
        return v

    def __iter__(self):
        self.prefetch(range(len(self)))            # every entry will be read: resolve them together
        return (self[i] for i in range(len(self)))

    def __reversed__(self):
        return (self[i] for i in range(len(self) - 1, -1, -1))


class Table:
    """An ordered set of named columns with a common length (a Spark DataFrame's role in the reference)."""

    def __init__(self, names: List[str], columns: List[Column], length: Optional[int] = None, device=None):
        self.names = list(names)
        self.columns = columns if isinstance(columns, LazyColumns) else list(columns)
        if length is None:
            length = columns[0].length if columns else 0
        self.length = int(length)
        self._device = torch.device(device) if device is not None else (
            columns[0].device if columns else torch.device("cpu"))
        self.dist = "replicated"     # distribution across ranks (see dxa.parallel)

    def _like(self, names, cols, length) -> "Table":
        t = Table(names, cols, length, self._device)
        t.dist = self.dist
        return t

    @property
    def device(self):
        return self._device

    def __len__(self):
        return self.length

    def column(self, name: str) -> Optional[Column]:
        for i, n in enumerate(self.names):          # by index: a lazy column list resolves only the match
            if n == name:
                return self.columns[i]
        i = self.index_of(name)
        return self.columns[i] if i >= 0 else None

    def index_of(self, name: str) -> int:
        low = name.lower()
        for i, n in enumerate(self.names):
            if n.lower() == low:
                return i
        return -1

    def schema(self) -> StructType:
        return StructType(tuple(StructField(n, c.dtype) for n, c in zip(self.names, self.columns)))

    def take(self, idx: torch.Tensor) -> "Table":
        return self._like(self.names, take_columns(self.columns, idx), int(idx.shape[0]))

    def filter(self, mask: torch.Tensor) -> "Table":
        idx = torch.nonzero(mask, as_tuple=False).flatten()
        return self.take(idx)

    def slice(self, start: int, stop: int) -> "Table":
        idx = torch.arange(start, min(stop, self.length), device=self._device)
        return self.take(idx)

    def select(self, names: List[str]) -> "Table":
        return self._like(names, [self.column(n) for n in names], self.length)

    def with_column(self, name: str, col: Column) -> "Table":
        i = self.index_of(name)
        names, cols = list(self.names), list(self.columns)
        if i >= 0:
            cols[i] = col
        else:
            names.append(name)
            cols.append(col)
        return self._like(names, cols, self.length)

    def to(self, device) -> "Table":
        return Table(self.names, [c.to(device) for c in self.columns], self.length, device)

    def to_pylist(self) -> List[Dict[str, Any]]:
        cols = [c.to_pylist() for c in self.columns]
        return [{n: col[i] for n, col in zip(self.names, cols)} for i in range(self.length)]

    def to_pydict(self) -> Dict[str, list]:
        return {n: c.to_pylist() for n, c in zip(self.names, self.columns)}

    @staticmethod
    def from_pylist(rows: List[Dict[str, Any]], schema: StructType, device="cpu") -> "Table":
        cols = [column_from_pylist([r.get(f.name) for r in rows], f.dtype, device) for f in schema.fields]
        return Table([f.name for f in schema.fields], cols, len(rows), device)

    @staticmethod
    def empty(schema: StructType, device="cpu") -> "Table":
        return Table.from_pylist([], schema, device)

    def __repr__(self):
        return f"Table(n={self.length}, cols={self.names})"


class DeferredTable(Table):
    """A statement's result whose host-side completion — a status read behind its own kernels — runs on first use
    of any attribute (``length``, ``columns``, ``names``, ``dist`` …); it then becomes the completed table (its class
    and attributes).  The batch thread plans the statements that do not read it in the meantime, so the read finds
    the kernels done instead of draining the stream (query._exec_select, processor.route)."""

    def __init__(self, finish):                 # noqa: no Table.__init__: every attribute comes from ``finish``
        self.__dict__["_finish"] = finish

    def resolve(self) -> Table:
        f = self.__dict__.pop("_finish", None)
        if f is None:
            return self
        t = f()
        if isinstance(t, DeferredTable):
            t = t.resolve()
        extra = dict(self.__dict__)            # attributes set while pending win over the completed table's
        self.__class__ = type(t)
        self.__dict__.update(t.__dict__)
        self.__dict__.update(extra)
        return self

    def __getattr__(self, name):
        if name != "_finish" and "_finish" in self.__dict__:
            self.resolve()
            return getattr(self, name)
        raise AttributeError(name)


def concat_tables(tables: List[Table]) -> Table:
    tables = [t for t in tables]
    if not tables:
        raise ValueError("no tables")
    if len(tables) == 1:
        return tables[0]
    names = tables[0].names
    device = tables[0].device
    batched = torch.device(device).type == "cuda"
    segs = None
    if batched:
        from ..ops.copybatch import Segments, concat_prims, valid_segments
        segs = Segments()
    same = all(t.names == names for t in tables)      # the usual case: one schema, no per-column name lookups
    cols = []
    str_groups = []                                 # (output position, parts) of the string columns
    for i, n in enumerate(names):
        if same:
            parts = [t.columns[i] for t in tables]
        else:
            parts = [t.column(n) if t.names[i].lower() != n.lower() else t.columns[i] for t in tables]
        kinds = {type(c) for c in parts}
        if batched and len(kinds) == 1:
            kind = next(iter(kinds))
            if kind is PrimColumn:
                got = concat_prims(parts, device, segs)
                if got is not None:
                    cols.append(PrimColumn(parts[0].dtype, got[0], got[1]))
                    continue
            elif kind is StrColumn:
                str_groups.append((len(cols), parts))
                cols.append(None)
                continue
        cols.append(concat_columns(parts))
    if str_groups:
        from ..ops.strings import concat_multi
        got = concat_multi([p for _, p in str_groups])
        for (at, parts), (arena, starts, lens) in zip(str_groups, got):
            valid, _ = valid_segments(parts, device, segs)
            cols[at] = type(parts[0])(arena, starts, lens, valid, parts[0].dtype)
            cols[at]._compact = True        # disjoint, in order in a fresh arena: its size bounds the bytes
            bounded = [p.max_len for p in parts if p.length]
            if all(m is not None for m in bounded):
                cols[at].max_len = max(bounded, default=0)
    if segs:
        segs.launch(device)                         # every fixed-width leaf of every table: one launch
    return Table(names, cols, sum(t.length for t in tables), device)


def _h2d(data, dtype, device):
    from ..ops.native import h2d
    return h2d(data, dtype, device)
