"""Array built-ins without per-row host work: sort_array / array_sort / array_distinct / array_max / array_min /
array_position / slice / array_union / array_intersect / array_except / array_join.

Arrays are ``ArrayColumn``s of K element slots (a row's elements are its present slots, left to right).  For
fixed-width elements every function here is a handful of tensor operations over the [rows × K] slot matrix —
comparisons across slots as one [rows × K × K] broadcast, compaction as a stable sort of slot indices — so the work
is O(1) launches per call on the device (and the same code is the CPU evaluator).  String elements use the device
string comparisons slot pair by slot pair (K² launches, K is small); sorting string arrays and nested elements stay
on the row-wise path.  Reference semantics: Spark 2.4 collectionOperations (sort_array: nulls first ascending,
last descending; array_sort: nulls last; array_distinct / union / intersect / except keep first occurrences, a null
equal to a null; slice: 1-based start, negative from the end, start 0 is an error)."""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from .column import ArrayColumn, ConstColumn, PrimColumn, StrColumn, materialize
from .expr import EvalError, _args, _slot_present, cast_column

_NUM = ("long", "int", "double", "float", "timestamp", "date", "boolean", "short", "byte")


class Unsupported(Exception):
    pass


_ROWWISE = False          # tests: force the row-wise functions (the oracle) — set through ``rowwise()``


class rowwise:
    """``with rowwise():`` evaluates the array built-ins row by row on the host (the differential tests' oracle)."""

    def __enter__(self):
        global _ROWWISE
        self.prev, _ROWWISE = _ROWWISE, True

    def __exit__(self, *exc):
        global _ROWWISE
        _ROWWISE = self.prev


def _elem_kind(arr: ArrayColumn) -> str:
    if not arr.elements:
        raise Unsupported("empty slot list")
    dt = arr.elements[0].dtype
    if any(e.dtype != dt for e in arr.elements):
        raise Unsupported("mixed slot types")
    if isinstance(dt, str) and dt in _NUM:
        return "num"
    if dt == "string":
        return "str"
    raise Unsupported(f"element type {dt}")


def _slots(arr: ArrayColumn):
    """(values [n, K] or None for strings, present [n, K], nonnull [n, K], element columns)."""
    els = [materialize(e) for e in arr.elements]
    n = arr.length
    present = torch.stack([_slot_present(arr, e) for e in els], 1) if els else \
        torch.zeros((n, 0), dtype=torch.bool, device=arr.device)
    nonnull = torch.stack([e.valid_mask() for e in els], 1) & present
    vals = None
    if els and isinstance(els[0], PrimColumn):
        vals = torch.stack([e.data for e in els], 1)
    return vals, present, nonnull, els


def _eq_slots(a_els, a_vals, b_els, b_vals) -> torch.Tensor:
    """[n, Ka, Kb]: element i of a equals element j of b (values only; nulls are the caller's)."""
    if a_vals is not None and b_vals is not None:
        x, y = a_vals, b_vals
        if x.dtype != y.dtype:
            x, y = x.to(torch.float64), y.to(torch.float64)
        return x.unsqueeze(2) == y.unsqueeze(1)
    from ..ops import strings as S
    rows = []
    for ea in a_els:
        rows.append(torch.stack([_str_eq(ea, eb, S) for eb in b_els], 1))
    return torch.stack(rows, 1)


def _str_eq(a, b, S):
    if a.starts.is_cuda:
        return S.eq_columns(a, b)
    return torch.tensor([x == y for x, y in zip(a.to_pylist(), b.to_pylist())], dtype=torch.bool)


def _build(els: List, order: torch.Tensor, keep: torch.Tensor, row_valid, drop_nulls=True) -> ArrayColumn:
    """Output slots: slot j of row r is input slot ``order[r, j]`` when ``keep[r, j]`` (kept slots first).  The
    element stacks are built once and gathered for every output slot together ([n, K] → [K, n] rows)."""
    n = order.shape[0]
    dev = order.device
    K = order.shape[1]
    if not K or not els:
        return ArrayColumn([], n, row_valid, True, dev)
    e0 = els[0]
    val = torch.stack([e.valid_mask() for e in els], 1).gather(1, order) & keep
    val_t = val.t().contiguous()
    if isinstance(e0, PrimColumn):
        data_t = torch.stack([e.data for e in els], 1).gather(1, order).t().contiguous()
        out = [PrimColumn(e0.dtype, data_t[j], val_t[j]) for j in range(K)]
        return ArrayColumn(out, n, row_valid, drop_nulls, dev)
    arena = e0.arena
    if len({id(e.arena) for e in els}) != 1:
        # slots over different arenas: one compact arena holding every slot's bytes (slot k, row r at k*n + r)
        from ..ops import strings as S
        cat = S.concat(els, None)
        starts = cat.starts.view(len(els), e0.length).t()
        arena = cat.arena
    else:
        starts = torch.stack([e.starts.to(torch.int64) for e in els], 1)
    lens = torch.stack([e.lens.to(torch.int32) for e in els], 1)
    st_t = starts.gather(1, order).t().contiguous()
    ln_t = lens.gather(1, order).t().contiguous()
    out = [type(e0)(arena, st_t[j], ln_t[j], val_t[j], e0.dtype) for j in range(K)]
    return ArrayColumn(out, n, row_valid, drop_nulls, dev)


def _compact(keep: torch.Tensor) -> torch.Tensor:
    """Slot order that moves kept slots to the front, stably."""
    K = keep.shape[1]
    key = (~keep).to(torch.int8)
    return torch.sort(key, dim=1, stable=True).indices if K else key.to(torch.int64)


def _first_occurrence(eq: torch.Tensor, present: torch.Tensor, nonnull: torch.Tensor) -> torch.Tensor:
    """keep[r, i]: present slot i has no equal present slot before it (null equals null).  Slots are classed
    0 absent / 1 null / 2 value: two slots are the same when their classes agree and they are null or equal."""
    n, K = present.shape
    cls = present.to(torch.int8) + nonnull.to(torch.int8)
    c = cls.unsqueeze(2)
    earlier = torch.ones((K, K), dtype=torch.bool, device=present.device).tril(-1)      # j < i
    same = (c == cls.unsqueeze(1)) & (eq | (c == 1)) & earlier
    return present & ~same.any(2)


def _row_valid(arr):
    return arr.valid


def _check_nulls_representable(arr, nonnull, present):
    """Variable-length results drop null slots (drop_nulls arrays): a real null element of a fixed-length input
    array would be lost — those inputs take the row-wise path."""
    if not arr.drop_nulls and bool((present & ~nonnull).any()):
        raise Unsupported("null elements in a variable-length result")


# ---- functions ------------------------------------------------------------------------------------------------

def array_max_min(arr: ArrayColumn, is_max: bool):
    if _elem_kind(arr) != "num":
        raise Unsupported("string max/min")
    vals, present, nonnull, els = _slots(arr)
    dt = els[0].dtype
    if vals.dtype == torch.bool:
        vals = vals.to(torch.int8)
    if vals.is_floating_point():
        fill = float("-inf") if is_max else float("inf")
        v = torch.where(nonnull, vals, torch.full_like(vals, fill))
        # NaN is larger than every value (Spark's ordering)
        if is_max:
            out = torch.where(torch.isnan(v).any(1), torch.full((v.shape[0],), float("nan"), dtype=v.dtype,
                                                                 device=v.device), v.max(1).values)
        else:
            out = torch.where(nonnull & ~torch.isnan(vals), vals, torch.full_like(vals, float("inf"))).min(1).values
            all_nan = (nonnull & torch.isnan(vals)).any(1) & ~(nonnull & ~torch.isnan(vals)).any(1)
            out = torch.where(all_nan, torch.full_like(out, float("nan")), out)
    else:
        info = torch.iinfo(vals.dtype)
        fill = info.min if is_max else info.max
        v = torch.where(nonnull, vals, torch.full_like(vals, fill))
        out = v.max(1).values if is_max else v.min(1).values
    if els[0].data.dtype == torch.bool:
        out = out.to(torch.bool)
    valid = nonnull.any(1)
    if arr.valid is not None:
        valid = valid & arr.valid
    return PrimColumn(dt, out, valid)


def array_position(arr: ArrayColumn, v):
    kind = _elem_kind(arr)
    vals, present, nonnull, els = _slots(arr)
    n = arr.length
    if isinstance(v, ConstColumn):
        if v.value is None:
            return PrimColumn("long", torch.zeros(n, dtype=torch.int64, device=arr.device),
                              torch.zeros(n, dtype=torch.bool, device=arr.device))
        v = materialize(v)
    if kind == "num":
        if not isinstance(v, PrimColumn):
            raise Unsupported("value type")
        x, y = vals, v.data.unsqueeze(1)
        if x.dtype != y.dtype:
            x, y = x.to(torch.float64), y.to(torch.float64)
        eq = x == y
    else:
        if not isinstance(v, StrColumn):
            v = cast_column(v, "string")
        from ..ops import strings as S
        eq = torch.stack([_str_eq(e, v, S) for e in els], 1)
    hit = eq & nonnull
    pos = torch.cumsum(present.to(torch.int64), 1)              # 1-based index among the row's elements
    big = torch.iinfo(torch.int64).max
    first = torch.where(hit, pos, torch.full_like(pos, big)).min(1).values if pos.shape[1] else \
        torch.full((n,), big, dtype=torch.int64, device=arr.device)
    out = torch.where(first == big, torch.zeros_like(first), first)
    valid = v.valid_mask()
    if arr.valid is not None:
        valid = valid & arr.valid
    return PrimColumn("long", out, valid)


def sort_array(arr: ArrayColumn, ascending: bool = True, nulls_first: Optional[bool] = None):
    """sort_array(arr, asc): nulls first ascending / last descending; array_sort: ascending, nulls last."""
    if _elem_kind(arr) != "num":
        raise Unsupported("string sort")
    vals, present, nonnull, els = _slots(arr)
    if nulls_first is None:
        nulls_first = ascending
    K = vals.shape[1]
    v = vals.to(torch.int8) if vals.dtype == torch.bool else vals
    o1 = torch.sort(v, dim=1, descending=not ascending, stable=True).indices
    # categories: absent slots last; nulls before or after the values
    cat = torch.where(present, torch.where(nonnull, torch.ones_like(o1, dtype=torch.int8),
                                           torch.full_like(o1, 0 if nulls_first else 2, dtype=torch.int8)),
                      torch.full_like(o1, 3, dtype=torch.int8))
    cat1 = cat.gather(1, o1)
    o2 = torch.sort(cat1, dim=1, stable=True).indices
    order = o1.gather(1, o2)
    keep = present.gather(1, order)
    if arr.drop_nulls:
        return _build(els, order, keep & nonnull.gather(1, order), arr.valid, True)
    return _build(els, order, keep & nonnull.gather(1, order), arr.valid, False) if bool(present.all()) else \
        _raise(Unsupported("partially present fixed-length array"))


def _raise(e):
    raise e


def array_distinct(arr: ArrayColumn):
    vals, present, nonnull, els = _slots(arr)
    _check_nulls_representable(arr, nonnull, present)
    eq = _eq_slots(els, vals, els, vals)
    keep = _first_occurrence(eq, present, nonnull)
    order = _compact(keep)
    return _build(els, order, keep.gather(1, order), arr.valid)


def slice_array(arr: ArrayColumn, start: int, length: int):
    if start == 0:
        raise EvalError("Unexpected value for start in function slice: SQL array indices start at 1.")
    if length < 0:
        raise EvalError(f"Unexpected value for length in function slice: length must be greater than or equal to 0.")
    vals, present, nonnull, els = _slots(arr)
    _check_nulls_representable(arr, nonnull, present)
    idx = torch.cumsum(present.to(torch.int64), 1) - 1
    count = present.sum(1, keepdim=True)
    s0 = torch.full_like(count, start - 1) if start > 0 else count + start
    keep = present & (idx >= s0) & (idx < s0 + length) & (s0 >= 0)
    order = _compact(keep)
    return _build(els, order, keep.gather(1, order), arr.valid)


def _two(a: ArrayColumn, b: ArrayColumn):
    ka, kb = _elem_kind(a), _elem_kind(b)
    if ka != kb:
        raise Unsupported("element types differ")
    return _slots(a), _slots(b)


def array_set_op(a: ArrayColumn, b: ArrayColumn, op: str):
    """array_union / array_intersect / array_except (first occurrences; null equals null; null array → null)."""
    (va, pa, na, ea), (vb, pb, nb, eb) = _two(a, b)
    _check_nulls_representable(a, na, pa)
    _check_nulls_representable(b, nb, pb)
    row_valid = a.valid_mask() & b.valid_mask() if (a.valid is not None or b.valid is not None) else None
    if op == "union":
        if va is not None and va.dtype != vb.dtype:
            raise Unsupported("numeric types differ")
        els = ea + eb
        vals = torch.cat([va, vb], 1) if va is not None else None
        present = torch.cat([pa, pb], 1)
        nonnull = torch.cat([na, nb], 1)
        eq = _eq_slots(els, vals, els, vals)
        keep = _first_occurrence(eq, present, nonnull)
        order = _compact(keep)
        return _build(els, order, keep.gather(1, order), row_valid)
    eq_ab = _eq_slots(ea, va, eb, vb)
    null_a = pa & ~na
    null_b = pb & ~nb
    in_b = ((eq_ab & na.unsqueeze(2) & nb.unsqueeze(1)) | (null_a.unsqueeze(2) & null_b.unsqueeze(1)))
    in_b = (in_b & pb.unsqueeze(1)).any(2)
    first = _first_occurrence(_eq_slots(ea, va, ea, va), pa, na)
    keep = first & (in_b if op == "intersect" else ~in_b)
    order = _compact(keep)
    return _build(ea, order, keep.gather(1, order), row_valid)


def array_join(arr: ArrayColumn, sep: str, null_rep: Optional[str] = None):
    """array_join(arr, sep[, nullReplacement]) → concat_ws over the slots (null elements skipped, or replaced)."""
    from ..ops import strings as S
    from .column import strings_from_pylist
    els = [materialize(e) for e in arr.elements]
    parts = []
    for e in els:
        c = e if isinstance(e, StrColumn) else cast_column(e, "string")
        present = _slot_present(arr, e)
        if null_rep is not None:
            # present null elements become the replacement; absent slots stay skipped
            nul = present & ~e.valid_mask()
            if bool(nul.any()):
                rep = materialize(ConstColumn(null_rep, "string", arr.length, arr.device))
                from .expr import _select_by_conditions
                c = _select_by_conditions([PrimColumn("boolean", nul)], [rep], c, arr.length, arr.device)
                c = materialize(c)
        parts.append(type(c)(c.arena, c.starts, c.lens, (c.valid_mask() & present), c.dtype))
    if not (parts and parts[0].starts.is_cuda):
        raise Unsupported("host")               # concat_ws runs on the device only; the CPU takes the row path
    out = S.concat_ws(sep, parts, arr.length, arr.device)
    if arr.valid is not None:
        out = type(out)(out.arena, out.starts, out.lens, arr.valid if out.valid is None else out.valid & arr.valid,
                        out.dtype)
    return out


def array_remove(arr: ArrayColumn, v):
    """array_remove(arr, v): every element equal to v dropped (null elements stay; a null v → null)."""
    vals, present, nonnull, els = _slots(arr)
    _check_nulls_representable(arr, nonnull, present)
    n = arr.length
    if isinstance(v, ConstColumn) and v.value is None:
        return ArrayColumn(arr.elements, n, torch.zeros(n, dtype=torch.bool, device=arr.device), arr.drop_nulls,
                           arr.device)
    v = materialize(v)
    if vals is not None:
        if not isinstance(v, PrimColumn):
            raise Unsupported("value type")
        x, y = vals, v.data.unsqueeze(1)
        if x.dtype != y.dtype:
            x, y = x.to(torch.float64), y.to(torch.float64)
        eq = x == y
    else:
        from ..ops import strings as S
        v = v if isinstance(v, StrColumn) else cast_column(v, "string")
        eq = torch.stack([_str_eq(e, v, S) for e in els], 1)
    keep = present & ~(eq & nonnull)
    order = _compact(keep)
    valid = v.valid_mask() if arr.valid is None else arr.valid & v.valid_mask()
    return _build(els, order, keep.gather(1, order), valid)


def arrays_overlap(a: ArrayColumn, b: ArrayColumn):
    """true if a non-null element is in both; otherwise null when both are non-empty and either holds a null, else
    false (Spark's ArraysOverlap)."""
    (va, pa, na, ea), (vb, pb, nb, eb) = _two(a, b)
    eq = _eq_slots(ea, va, eb, vb) & na.unsqueeze(2) & nb.unsqueeze(1)
    hit = eq.any(2).any(1)
    has_null = (pa & ~na).any(1) | (pb & ~nb).any(1)
    nonempty = pa.any(1) & pb.any(1)
    valid = hit | ~(nonempty & has_null)
    if a.valid is not None:
        valid = valid & a.valid
    if b.valid is not None:
        valid = valid & b.valid
    return PrimColumn("boolean", hit, valid)


# ---- registration ---------------------------------------------------------------------------------------------

def _wrap(name, device_fn, host_fn):
    """``device_fn(args)``; ``Unsupported`` → the row-wise host function (the previous implementation)."""
    def f(e, scope, ctx, subst):
        if _ROWWISE:
            return host_fn(e, scope, ctx, subst)
        args = _args(e, scope, ctx, subst)
        if args and isinstance(args[0], ArrayColumn):
            try:
                return device_fn(args)
            except Unsupported:
                pass
        return host_fn(e, scope, ctx, subst)
    f.__name__ = f"_f_{name}"
    return f


def _const(a, default=None):
    if a is None:
        return default
    if not isinstance(a, ConstColumn):
        raise Unsupported("non-constant argument")
    return a.value


def register(host: dict):
    """Override the row-wise registrations in ``host`` (name → function)."""
    from .expr import register_function as reg
    reg("array_max", _wrap("array_max", lambda a: array_max_min(a[0], True), host["array_max"]))
    reg("array_min", _wrap("array_min", lambda a: array_max_min(a[0], False), host["array_min"]))
    reg("array_position", _wrap("array_position", lambda a: array_position(a[0], a[1]), host["array_position"]))
    reg("sort_array", _wrap("sort_array", lambda a: sort_array(a[0], bool(_const(a[1] if len(a) > 1 else None,
                                                                                     True))), host["sort_array"]))
    reg("array_sort", _wrap("array_sort", lambda a: sort_array(a[0], True, False), host["array_sort"]))
    reg("array_distinct", _wrap("array_distinct", lambda a: array_distinct(a[0]), host["array_distinct"]))
    reg("slice", _wrap("slice", lambda a: slice_array(a[0], int(_const(a[1])), int(_const(a[2]))), host["slice"]))
    for op in ("union", "intersect", "except"):
        reg(f"array_{op}", _wrap(f"array_{op}", lambda a, op=op: _set_args(a, op), host[f"array_{op}"]))
    reg("array_remove", _wrap("array_remove", lambda a: array_remove(a[0], a[1]), host["array_remove"]))
    reg("arrays_overlap", _wrap("arrays_overlap", lambda a: _ovl(a), host["arrays_overlap"]))
    reg("array_join", _wrap("array_join", lambda a: array_join(a[0], str(_const(a[1])),
                                                                None if len(a) < 3 else _const(a[2])),
                            host["array_join"]))


def _ovl(a):
    if len(a) != 2 or not isinstance(a[1], ArrayColumn):
        raise Unsupported("second argument")
    return arrays_overlap(a[0], a[1])


def _set_args(a, op):
    if len(a) != 2 or not isinstance(a[1], ArrayColumn):
        raise Unsupported("second argument")
    return array_set_op(a[0], a[1], op)


def _register_once():
    from .expr import _FUNCS
    if getattr(_FUNCS.get("array_max"), "__name__", "") != "_f_array_max":
        register(dict(_FUNCS))


_register_once()
