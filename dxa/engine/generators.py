"""Table-generating functions: ``explode`` / ``posexplode`` / ``inline`` / ``stack`` (and their ``_outer`` forms),
in a SELECT list or behind ``LATERAL VIEW [OUTER]``.

Arrays here are fixed-slot columns (``ArrayColumn``: K element columns; with ``drop_nulls`` an invalid slot is not
part of the array), so a generator is a set of per-slot row selections: slot j contributes the rows where it is
present, the selections are concatenated and put back in (input row, slot) order with one stable sort.  Every step
is a device op; the only host read is the output row count.
"""
from __future__ import annotations

from typing import List, Tuple

import torch

from ..sql import ast as A
from .column import (ArrayColumn, Column, ConstColumn, StructColumn, concat_columns, materialize)
from .expr import EvalError, _slot_present, cast_column, evaluate
from .types import common_type

GENERATORS = {"explode", "explode_outer", "posexplode", "posexplode_outer", "inline", "inline_outer", "stack",
              "json_tuple"}


def is_generator(e) -> bool:
    return isinstance(e, A.Call) and e.name in GENERATORS


def _typed_nulls(like: Column, n: int) -> Column:
    """``n`` null rows shaped like ``like``."""
    if n == 0 or like.length == 0:
        return ConstColumn(None, like.dtype, n, like.device)
    idx = torch.zeros(n, dtype=torch.int64, device=like.device)
    return materialize(like).take(idx).with_valid(torch.zeros(n, dtype=torch.bool, device=like.device))


def _unify(cols: List[Column]) -> List[Column]:
    types = {str(c.dtype) for c in cols if not (isinstance(c, ConstColumn) and c.value is None)}
    if len(types) <= 1:
        t = next(iter(types), None)
        return [ConstColumn(None, t, c.length, c.device) if t and isinstance(c, ConstColumn) and c.value is None
                else c for c in cols]
    t = cols[0].dtype
    for c in cols[1:]:
        t = common_type(t, c.dtype)
    return [cast_column(c, t) if c.dtype != t else c for c in cols]


def generate(call: A.Call, scope, ctx, outer: bool = False) -> Tuple[torch.Tensor, List[str], List[Column]]:
    """(input row of every output row, output column names, output columns)."""
    name = call.name
    outer = outer or name.endswith("_outer")
    base = name[:-6] if name.endswith("_outer") else name
    n, dev = scope.length, scope.device
    if base == "stack":
        return _stack(call, scope, ctx)
    if base == "json_tuple":
        return _json_tuple(call, scope, ctx)
    if not call.args:
        raise EvalError(f"{name}() expects an argument")
    src = evaluate(call.args[0], scope, ctx)
    if isinstance(src, ConstColumn) and src.value is None:
        slots, keys, present = [], [], []
    elif isinstance(src, ArrayColumn):
        slots = list(src.elements)
        keys = None
        present = [_slot_present(src, el) for el in slots]
    elif isinstance(src, StructColumn) and src.is_map:
        slots = list(src.children)
        keys = list(src.names)
        base_ok = src.valid_mask()
        present = [base_ok for _ in slots]
    else:
        raise EvalError(f"{name}() expects an array or a map, got {src.dtype}")
    K = len(slots)
    rows_l, slot_l, pos_l, vals_l, key_l = [], [], [], [], []
    seen = torch.zeros(n, dtype=torch.int64, device=dev)
    for j in range(K):
        idx = torch.nonzero(present[j]).flatten()
        rows_l.append(idx)
        slot_l.append(torch.full_like(idx, j))
        pos_l.append(seen[idx])                      # position among the row's present slots
        seen = seen + present[j].to(torch.int64)
        vals_l.append(materialize(slots[j]).take(idx))
        if keys is not None:
            key_l.append(ConstColumn(keys[j], "string", int(idx.shape[0]), dev))
    elem_like = slots[0] if slots else ConstColumn(None, "null", n, dev)
    if outer:
        miss = torch.nonzero(seen == 0).flatten()
        rows_l.append(miss)
        slot_l.append(torch.full_like(miss, K))
        pos_l.append(torch.zeros_like(miss))
        m = int(miss.shape[0])
        vals_l.append(_typed_nulls(elem_like, m))
        if keys is not None:
            key_l.append(ConstColumn(None, "string", m, dev))
    rows = torch.cat(rows_l) if rows_l else torch.zeros(0, dtype=torch.int64, device=dev)
    slot = torch.cat(slot_l) if slot_l else rows
    order = torch.argsort(rows * (K + 1) + slot, stable=True) if rows.numel() else rows
    rows = rows[order]
    vals = concat_columns(_unify(vals_l)).take(order) if vals_l else ConstColumn(None, "null", 0, dev)
    pos = torch.cat(pos_l)[order] if pos_l else rows
    from .column import PrimColumn
    pos_col = PrimColumn("int", pos, None if not outer else (slot[order] < K))
    names: List[str]
    cols: List[Column]
    if keys is not None:
        kc = concat_columns([materialize(k) for k in key_l]).take(order) if key_l else \
            ConstColumn(None, "string", 0, dev)
        names, cols = ["key", "value"], [kc, vals]
    elif base == "inline":
        if not isinstance(elem_like, StructColumn):
            raise EvalError("inline() expects an array of structs")
        names = list(elem_like.names)
        cols = [vals.child(nm) if isinstance(vals, StructColumn) else ConstColumn(None, "null", len(rows), dev)
                for nm in names]
    else:
        names, cols = ["col"], [vals]
    if base == "posexplode":
        names, cols = ["pos"] + names, [pos_col] + cols
    return rows, names, cols


def _stack(call: A.Call, scope, ctx):
    """stack(n, v1, …, vk): n output rows per input row, k/n columns (row r takes v[r*m .. r*m+m-1])."""
    n, dev = scope.length, scope.device
    k0 = evaluate(call.args[0], scope, ctx)
    if not isinstance(k0, ConstColumn) or not isinstance(k0.value, int) or k0.value <= 0:
        raise EvalError("stack() expects a positive integer row count first")
    nr = int(k0.value)
    vals = [evaluate(a, scope, ctx) for a in call.args[1:]]
    m = (len(vals) + nr - 1) // nr
    vals += [ConstColumn(None, "null", n, dev)] * (nr * m - len(vals))
    rows = torch.arange(n, dtype=torch.int64, device=dev).repeat(nr)        # [r0 rows…, r1 rows…, …]
    r_of = torch.arange(nr, dtype=torch.int64, device=dev).repeat_interleave(n)
    order = torch.argsort(rows * nr + r_of, stable=True)
    cols = []
    for c in range(m):
        parts = _unify([vals[r * m + c] for r in range(nr)])
        cols.append(concat_columns([materialize(p) for p in parts]).take(order))
    return rows[order], [f"col{c}" for c in range(m)], cols


def _json_tuple(call: A.Call, scope, ctx):
    """json_tuple(json, 'k1', …): one row per input row, one string column per top-level key (c0, c1, …)."""
    from .sqlfuncs import _get_json_object
    from .column import strings_from_pylist
    n, dev = scope.length, scope.device
    src = evaluate(call.args[0], scope, ctx)
    keys = []
    for a in call.args[1:]:
        k = evaluate(a, scope, ctx)
        if not isinstance(k, ConstColumn):
            raise EvalError("json_tuple() keys must be constants")
        keys.append(str(k.value))
    docs = src.to_pylist() if not isinstance(src, ConstColumn) else [src.value] * n
    import json as _json
    cols = []
    parsed = []
    for d in docs:
        try:
            parsed.append(_json.loads(d) if d is not None else None)
        except ValueError:
            parsed.append(None)
    for k in keys:
        vals = []
        for doc in parsed:
            v = doc.get(k) if isinstance(doc, dict) else None
            vals.append(None if v is None else v if isinstance(v, str) else
                        ("true" if v is True else "false" if v is False else _json.dumps(v, separators=(",", ":"))))
        cols.append(strings_from_pylist(vals, dev))
    return torch.arange(n, dtype=torch.int64, device=dev), [f"c{i}" for i in range(len(keys))], cols
