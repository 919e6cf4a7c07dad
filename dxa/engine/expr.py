"""Columnar expression evaluation (the Spark ``selectExpr`` / ``where`` / SQL expression layer of the reference,
DataProcessing/datax-host/src/main/scala/datax/processor/CommonProcessorFactory.scala:99-100,253-289).

Every operator works on whole columns: numeric/boolean/timestamp math is device tensor arithmetic, string
predicates/CONCAT/casts go to the strings.hip kernels, and a handful of rarely-used functions are explicitly
*host-assisted* (evaluated row-wise on the host and copied back) — they are correct, just not on a hot path.
Spark semantics followed: three-valued logic, null propagation, ``/`` is fractional, division by zero → null,
integral ``%`` keeps the dividend's sign, WHERE treats null as false.
"""
from __future__ import annotations

import contextvars
import json
import math
import re
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch

from ..sql import ast as A
from . import functions as F
from . import jit as _jit_mod
from .column import (ArrayColumn, Column, ConstColumn, JsonColumn, LazyColumns, PrimColumn, StrColumn,
                     StructColumn, TORCH_DTYPE, and_valid, column_from_pylist, concat_columns, materialize, strings_from_pylist,
                     take_columns)
from .types import (INT_RANGE, INTEGRAL, ArrayType, MapType, StructType, common_type, is_integral, is_nested,
                    is_numeric, wrap_int_tensor, wrap_int_value)
from . import decimal as D
from .decimal import is_decimal

AGG_FUNCS = {"count", "sum", "avg", "mean", "min", "max", "first", "last", "first_value", "last_value", "stddev",
             "stddev_samp", "stddev_pop", "variance", "var_samp", "var_pop", "std", "collect_list", "collect_set",
             "approx_count_distinct", "count_if", "bool_and", "bool_or", "every", "any", "some", "percentile",
             "percentile_approx", "approx_percentile", "median", "corr", "covar_pop", "covar_samp", "kurtosis",
             "skewness", "max_by", "min_by"}


class EvalError(Exception):
    pass


@dataclass
class EvalContext:
    now_us: int = 0                       # current_timestamp() of this batch/query
    udfs: Dict[str, Any] = field(default_factory=dict)   # name → UDF (callable(columns, ctx) → Column)
    udafs: Dict[str, Any] = field(default_factory=dict)
    device: Any = "cpu"
    catalog: Any = None                   # tables visible to sub-queries (set by query.execute)
    prefilter: Dict[int, Any] = field(default_factory=dict)   # id(Select) → early WHERE mask (query.prefilter)
    prefilter_cands: Dict[int, Any] = field(default_factory=dict)   # id(table) → filters over it, not yet run
    defer_dense: bool = False             # a windowed GROUP BY may return a DeferredTable (query._deferred_select)
    pending: List[Any] = field(default_factory=list)           # DeferredTables of this batch not yet completed


class TakenColumns(LazyColumns):
    """``[c.take(idx) for c in cols]`` computed per column on first access: a filtered or grouped scope usually
    reads a few of its input's columns, so the gathers of the others are never launched."""

    def __init__(self, cols, idx):
        super().__init__([None] * len(cols))
        self._src = cols if isinstance(cols, LazyColumns) else list(cols)
        self._idx = idx

    def _make(self, i):
        return self._src[i].take(self._idx)

    def prefetch(self, idxs) -> None:
        todo = self._unresolved(idxs)
        if not todo:
            return
        if isinstance(self._src, LazyColumns):
            self._src.prefetch(todo)
        for i, c in zip(todo, take_columns([self._src[i] for i in todo], self._idx)):
            list.__setitem__(self, i, c)


class DeferredColumns(LazyColumns):
    """A projection's output columns where the bare column references into a lazy scope stay unresolved until
    read (``entries``: a column, or ``(lazy_list, index)``)."""

    def __init__(self, entries):
        super().__init__([e if not isinstance(e, tuple) else None for e in entries])
        self._refs = [e if isinstance(e, tuple) else None for e in entries]

    def _make(self, i):
        src, j = self._refs[i]
        return src[j]

    def prefetch(self, idxs) -> None:
        todo = self._unresolved(idxs)
        by_src = {}
        for i in todo:
            src, j = self._refs[i]
            by_src.setdefault(id(src), (src, []))[1].append(j)
        for src, js in by_src.values():
            if isinstance(src, LazyColumns):
                src.prefetch(js)


class _Prepended(LazyColumns):
    """``head + rest`` without resolving ``rest`` (a lazy scope stays lazy under lambda bindings)."""

    def __init__(self, head, rest):
        super().__init__(list(head) + [None] * len(rest))
        self._k, self._rest = len(head), rest

    def _make(self, i):
        return self._rest[i - self._k]


class HiddenQual(str):
    """The qualifier of a column reachable only qualified: the per-side key copies of a USING / NATURAL join, whose
    unqualified name resolves to the join's merged key column (and ``SELECT *`` lists that one only)."""


class Scope:
    """Columns visible to an expression: (qualifier, name, column) triples over ``length`` rows."""

    def __init__(self, names: List[str], cols: List[Column], quals: List[Optional[str]], length: int, device):
        self.names = names
        self.cols = cols
        self.quals = quals
        self.length = int(length)
        self.device = torch.device(device)
        self._index: Optional[Dict[str, List[int]]] = None

    def with_bindings(self, names: List[str], cols: List[Column]) -> "Scope":
        """This scope plus ``names`` bound to ``cols`` (lambda parameters), which shadow same-named columns."""
        sc = Scope(list(names) + list(self.names), _Prepended(list(cols), self.cols), [None] * len(names) +
                   list(self.quals), self.length, self.device)
        sc.dist = getattr(self, "dist", None)
        return sc

    @staticmethod
    def of_table(table, qual: Optional[str] = None) -> "Scope":
        cols = table.columns if isinstance(table.columns, LazyColumns) else list(table.columns)
        return Scope(list(table.names), cols, [qual] * len(table.names), table.length, table.device)

    def qualifiers(self):
        got = self.__dict__.get("_quals")
        if got is None:
            got = self._quals = {q.lower() for q in self.quals if q}
        return got

    def _find(self, name: str, qual: Optional[str] = None) -> List[int]:
        index = self._index
        if index is None:
            index = self._index = _name_index(self.names)
        out = index.get(name.lower())
        if not out:
            return []
        if qual is not None:
            ql = qual.lower()
            out = [i for i in out if (self.quals[i] or "").lower() == ql]
        else:
            vis = [i for i in out if not isinstance(self.quals[i], HiddenQual)]
            out = vis or list(out)
        exact = [i for i in out if self.names[i] == name]
        return exact or out

    def has_qualifier(self, q: str) -> bool:
        return q.lower() in self.qualifiers()

    def index_of(self, parts: Tuple[str, ...]) -> Optional[int]:
        """The column a reference reads (as ``resolve`` picks it), without materialising anything."""
        if len(parts) >= 2 and self.has_qualifier(parts[0]):
            hits = self._find(parts[1], parts[0])
            if hits:
                return hits[0]
        hits = self._find(parts[0])
        return hits[0] if hits else None

    def prefetch(self, exprs) -> None:
        """Gather together every column the expressions read from a lazy (filtered / joined) scope: one multi-column
        gather launch instead of a take per column as each is first touched."""
        if not isinstance(self.cols, LazyColumns):
            return
        idx = []
        for e in exprs:
            if e is None:
                continue
            for node in A.walk(e):
                if isinstance(node, A.Ident):
                    k = self.index_of(node.parts)
                    if k is not None:
                        idx.append(k)
        if len(idx) > 1:
            self.cols.prefetch(idx)

    def try_resolve(self, parts: Tuple[str, ...]) -> Optional[Column]:
        try:
            return self.resolve(parts)
        except EvalError:
            return None

    def resolve(self, parts: Tuple[str, ...]) -> Column:
        # qualified: t.col[.field…]
        if len(parts) >= 2 and self.has_qualifier(parts[0]):
            hits = self._find(parts[1], parts[0])
            if hits:
                return _navigate(self.cols[hits[0]], parts[2:])
        hits = self._find(parts[0])
        if not hits:
            raise EvalError(f"cannot resolve '{'.'.join(parts)}' given columns {self.names}")
        if len(hits) > 1 and len({id(self.cols[h]) for h in hits}) > 1:
            quals = {self.quals[h] for h in hits}
            if len(quals) > 1:
                raise EvalError(f"reference '{parts[0]}' is ambiguous")
        return _navigate(self.cols[hits[0]], parts[1:])


_NAME_INDEX: Dict[Tuple[str, ...], Dict[str, List[int]]] = {}


def _name_index(names: List[str]) -> Dict[str, List[int]]:
    """lower-cased column name → its positions, shared by every scope over the same names (statements resolve
    dozens of references per batch against scopes of ~30 columns)."""
    key = tuple(names)
    got = _NAME_INDEX.get(key)
    if got is None:
        got = {}
        for i, n in enumerate(names):
            got.setdefault(n.lower(), []).append(i)
        if len(_NAME_INDEX) >= 512:
            _NAME_INDEX.clear()
        _NAME_INDEX[key] = got
    return got


def _navigate(col: Column, rest: Tuple[str, ...]) -> Column:
    for p in rest:
        col = field_access(col, p)
    return col


def field_access(col: Column, name: str) -> Column:
    if isinstance(col, StructColumn):
        c = col.child(name)
        if c is None:
            if col.is_map:
                return ConstColumn(None, col.dtype.value if isinstance(col.dtype, MapType) else "string",
                                   col.length, col.device)
            raise EvalError(f"no such struct field {name} in {col.names}")
        return c.with_valid(col.valid) if col.valid is not None else c
    if isinstance(col, ConstColumn) and col.value is None:
        return col
    if isinstance(col, JsonColumn) or (isinstance(col, StrColumn) and is_nested(col.dtype)):
        return _json_get(col, name)
    raise EvalError(f"cannot access field {name} of {col.dtype}")


def _json_get(col, key):
    """Host-assisted map/array element access on raw JSON text columns."""
    vals = col.to_pylist()
    out = []
    vt = "string"
    if isinstance(col.dtype, MapType):
        vt = col.dtype.value if isinstance(col.dtype.value, str) else "string"
    elif isinstance(col.dtype, ArrayType):
        vt = col.dtype.element if isinstance(col.dtype.element, str) else "string"
    for v in vals:
        if isinstance(v, dict):
            out.append(v.get(key))
        elif isinstance(v, list):
            try:
                out.append(v[int(key)])
            except (ValueError, IndexError):
                out.append(None)
        else:
            out.append(None)
    if vt == "string":
        out = [None if x is None else (x if isinstance(x, str) else json.dumps(x)) for x in out]
    return column_from_pylist(out, vt, col.device)


# ---------------------------------------------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------------------------------------------

def bool_col(data: torch.Tensor, valid: Optional[torch.Tensor]) -> PrimColumn:
    return PrimColumn("boolean", data, valid)


def as_prim(col: Column) -> Column:
    if isinstance(col, ConstColumn):
        return col.materialize()
    return col


def predicate_mask(col: Column) -> torch.Tensor:
    """WHERE semantics: null → false."""
    if isinstance(col, ConstColumn):
        v = bool(col.value) if col.value is not None else False
        return torch.full((col.length,), v, dtype=torch.bool, device=col.device)
    if not isinstance(col, PrimColumn):
        raise EvalError("predicate must be boolean")
    d = col.data if col.data.dtype == torch.bool else col.data != 0
    return d & col.valid if col.valid is not None else d


def _scalar_or_tensor(col: Column):
    if isinstance(col, ConstColumn):
        return col.value
    return col.data


def _num_value(col: Column, to: str):
    """Tensor (or python scalar) of a numeric column converted to storage dtype of ``to``."""
    if isinstance(col, ConstColumn):
        v = col.value
        if v is None:
            return None
        if isinstance(v, bool):
            v = int(v)
        return float(v) if to == "double" else int(v)
    d = col.data
    if d.dtype == torch.bool:
        d = d.to(torch.int64)
    if to == "double" and d.dtype != torch.float64:
        d = d.to(torch.float64)
    return d


def _all_const(*cols):
    return all(isinstance(c, ConstColumn) for c in cols)


def _result_valid(*cols):
    v = None
    for c in cols:
        v = and_valid(v, c.valid)
    return v


def _const_result(value, dtype, n, device):
    return ConstColumn(value, dtype, n, device)


def _coerce_const_for(col_other: Column, const: ConstColumn) -> ConstColumn:
    """Implicit literal casts (string literal vs timestamp / numeric column)."""
    if const.value is None or not isinstance(const.value, str):
        return const
    if col_other.dtype == "timestamp":
        return ConstColumn(F.parse_timestamp_literal(const.value), "timestamp", const.length, const.device)
    if is_numeric(col_other.dtype):
        try:
            v = float(const.value)
            if is_integral(col_other.dtype) and v.is_integer():
                return ConstColumn(int(v), "long", const.length, const.device)
            return ConstColumn(v, "double", const.length, const.device)
        except ValueError:
            return ConstColumn(None, "null", const.length, const.device)
    return const


# ---------------------------------------------------------------------------------------------------------------
# evaluator
# ---------------------------------------------------------------------------------------------------------------

# Built-ins that take decimal(p,s) arguments as they are; every other function sees its decimal arguments as
# doubles (Spark's implicit cast for functions typed on DoubleType: ImplicitTypeCasts) — see _call / evaluate.
_DECIMAL_AWARE = frozenset({"round", "bround", "hash", "typeof",
                            "coalesce", "if", "nvl", "ifnull", "nullif", "nvl2", "to_json", "named_struct", "struct",
                            "array", "map", "concat", "concat_ws", "isnull", "isnotnull", "string", "abs",
                            "negative", "positive", "ceil", "ceiling", "floor"})

_DEMOTE: "contextvars.ContextVar" = contextvars.ContextVar("dxa_decimal_demote", default=None)


def evaluate(e: A.Expr, scope: Scope, ctx: EvalContext, subst: Optional[Dict] = None, _jit: bool = True) -> Column:
    """Evaluate ``e`` over every row of ``scope``.  ``subst`` maps expression keys to precomputed columns
    (aggregate results).  Scalar operator trees over large device batches run as one generated kernel
    (``jit.py``); ``_jit=False`` evaluates this node with tensor ops (its children may still fuse)."""
    r = _evaluate_node(e, scope, ctx, subst, _jit)
    dem = _DEMOTE.get()
    if dem is not None and id(e) in dem and is_decimal(r.dtype):
        return _dec_to_double(r)
    return r


def _evaluate_node(e: A.Expr, scope: Scope, ctx: EvalContext, subst: Optional[Dict], _jit: bool) -> Column:
    if subst:
        k = e.key()
        if k in subst:
            return subst[k]
    if _jit and _jit_mod.eligible(e, scope):
        r = _jit_mod.try_fused(e, scope, ctx, subst, evaluate)
        if r is not None:
            return r
    n, dev = scope.length, scope.device
    if isinstance(e, A.Literal):
        t = e.type
        if t == "int":
            t = "int"
        return ConstColumn(e.value, t, n, dev)
    if isinstance(e, A.Ident):
        return scope.resolve(e.parts)
    if isinstance(e, A.SubqueryExpr):
        return _subquery(e, scope, ctx, subst)
    if isinstance(e, A.Lambda):
        raise EvalError("a lambda is only allowed as an argument of a higher-order function")
    if isinstance(e, A.Interval):
        return ConstColumn(e.micros, "interval", n, dev)
    if isinstance(e, A.BinOp):
        return _binop(e, scope, ctx, subst)
    if isinstance(e, A.UnaryOp):
        v = evaluate(e.operand, scope, ctx, subst)
        if e.op == "not":
            if isinstance(v, ConstColumn):
                return ConstColumn(None if v.value is None else (not v.value), "boolean", n, dev)
            return bool_col(~(v.data.bool()), v.valid)
        if e.op == "-":
            if isinstance(v, ConstColumn):
                if v.value is None:
                    return ConstColumn(None, v.dtype, n, dev)
                return ConstColumn(wrap_int_value(-v.value, v.dtype) if v.dtype in INTEGRAL else -v.value, v.dtype,
                                   n, dev)
            if is_decimal(v.dtype):
                return D.negate(v)
            if v.dtype in INTEGRAL:                     # -MIN_VALUE is MIN_VALUE (two's complement)
                return PrimColumn(v.dtype, wrap_int_tensor(-v.data, v.dtype), v.valid)
            return PrimColumn(v.dtype, -v.data, v.valid)
        if e.op == "~":
            if isinstance(v, ConstColumn):
                return ConstColumn(None if v.value is None else ~int(v.value), v.dtype, n, dev)
            return PrimColumn(v.dtype, ~v.data, v.valid)
        return v
    if isinstance(e, A.IsNull):
        v = evaluate(e.operand, scope, ctx, subst)
        if isinstance(v, ConstColumn):
            isn = v.value is None
            return ConstColumn((not isn) if e.negated else isn, "boolean", n, dev)
        if v.valid is None:
            return ConstColumn(bool(e.negated), "boolean", n, dev)
        return bool_col(v.valid.clone() if e.negated else ~v.valid, None)
    if isinstance(e, A.InList):
        acc = None
        for it in e.items:
            c = _compare("=", evaluate(e.operand, scope, ctx, subst), evaluate(it, scope, ctx, subst), n, dev)
            acc = c if acc is None else _logic("or", acc, c, n, dev)
        if e.negated:
            acc = evaluate_not(acc, n, dev)
        return acc
    if isinstance(e, A.Between):
        v = evaluate(e.operand, scope, ctx, subst)
        lo = _compare(">=", v, evaluate(e.low, scope, ctx, subst), n, dev)
        hi = _compare("<=", v, evaluate(e.high, scope, ctx, subst), n, dev)
        r = _logic("and", lo, hi, n, dev)
        return evaluate_not(r, n, dev) if e.negated else r
    if isinstance(e, A.Like):
        return _like(e, scope, ctx, subst)
    if isinstance(e, A.Case):
        return _case(e, scope, ctx, subst)
    if isinstance(e, A.Cast):
        return cast_column(evaluate(e.operand, scope, ctx, subst), e.to)
    if isinstance(e, A.Subscript):
        base = evaluate(e.base, scope, ctx, subst)
        idx = evaluate(e.index, scope, ctx, subst)
        if not isinstance(idx, ConstColumn):
            raise EvalError("only constant subscripts are supported")
        if isinstance(base, ArrayColumn):
            i = int(idx.value)
            if e.dot:
                raise EvalError("field access on array")
            return base.elements[i] if 0 <= i < len(base.elements) else ConstColumn(None, "null", n, dev)
        return field_access(base, str(idx.value))
    if isinstance(e, A.Call):
        return _call(e, scope, ctx, subst)
    if isinstance(e, A.Star):
        raise EvalError("'*' is only allowed in a select list or COUNT(*)")
    raise EvalError(f"unsupported expression {type(e).__name__}")


def evaluate_not(c: Column, n, dev):
    if isinstance(c, ConstColumn):
        return ConstColumn(None if c.value is None else not c.value, "boolean", n, dev)
    return bool_col(~c.data, c.valid)


def _logic(op: str, a: Column, b: Column, n, dev) -> Column:
    if _all_const(a, b):
        x, y = a.value, b.value
        if op == "and":
            r = False if (x is False or y is False) else (None if (x is None or y is None) else bool(x and y))
        else:
            r = True if (x is True or y is True) else (None if (x is None or y is None) else bool(x or y))
        return ConstColumn(r, "boolean", n, dev)
    a, b = as_prim(a), as_prim(b)
    ad, bd = a.data.bool(), b.data.bool()
    at = ad if a.valid is None else ad & a.valid
    af = ~ad if a.valid is None else ~ad & a.valid
    bt = bd if b.valid is None else bd & b.valid
    bf = ~bd if b.valid is None else ~bd & b.valid
    if op == "and":
        t = at & bt
        f = af | bf
    else:
        t = at | bt
        f = af & bf
    if a.valid is None and b.valid is None:
        return bool_col(t, None)
    return bool_col(t, t | f)


def _dec_operands(a: Column, b: Column):
    """Spark DecimalPrecision coercion for a binary operator with a decimal side: ('double', a, b) when the other
    side is fractional (or a string / anything non-integral), else ('decimal', a, b) with integral sides widened to
    decimal(10,0) / decimal(20,0)."""
    other = b if is_decimal(a.dtype) else a
    if not (is_decimal(other.dtype) or other.dtype in INTEGRAL + ("null",)):
        return "double", _dec_to_double(a), _dec_to_double(b)
    return "decimal", _to_dec(a), _to_dec(b)


def _dec_to_double(c: Column) -> Column:
    if not is_decimal(c.dtype):
        return c
    if isinstance(c, ConstColumn):
        return ConstColumn(None if c.value is None else float(c.value), "double", c.length, c.device)
    return D.to_double(c)


def _to_dec(c: Column) -> Column:
    if is_decimal(c.dtype) or c.dtype == "null":
        return c
    if isinstance(c, ConstColumn):
        # Spark 2.4 DecimalPrecision (literalPickMinimumPrecision): an integral literal next to a decimal takes the
        # tightest decimal(digits, 0) — DecimalType.fromLiteral
        t = D.DecimalType(max(1, len(str(abs(int(c.value))))), 0) if c.value is not None else D.of_integral(c.dtype)
        return ConstColumn(D.quantize(c.value, t), t, c.length, c.device)
    t = D.of_integral(c.dtype)
    return D.from_integral(c, t)


def _dec_arith(op: str, a: Column, b: Column, n, dev) -> Column:
    kind, a, b = _dec_operands(a, b)
    if kind == "double":
        return _arith(op, a, b, n, dev)
    if op not in ("+", "-", "*", "/", "%"):
        if op == "div":
            return _arith(op, cast_column(a, "long") if not isinstance(a, ConstColumn) else
                          ConstColumn(D.scalar_to(a.value, a.dtype, "long"), "long", n, dev),
                          cast_column(b, "long") if not isinstance(b, ConstColumn) else
                          ConstColumn(D.scalar_to(b.value, b.dtype, "long"), "long", n, dev), n, dev)
        raise EvalError(f"cannot apply {op} to {a.dtype} and {b.dtype}")
    at = a.dtype if is_decimal(a.dtype) else b.dtype
    bt = b.dtype if is_decimal(b.dtype) else a.dtype
    rt = D.result_type(op, at, bt)
    if (isinstance(a, ConstColumn) and a.value is None) or (isinstance(b, ConstColumn) and b.value is None):
        return ConstColumn(None, rt, n, dev)
    if _all_const(a, b):
        return ConstColumn(D.scalar_op(op, a.value, b.value, rt), rt, n, dev)
    return D.arith(op, as_prim(a), as_prim(b), at, bt)


def _arith(op: str, a: Column, b: Column, n, dev) -> Column:
    if a.dtype == "timestamp" or b.dtype == "timestamp":
        return _ts_arith(op, a, b, n, dev)
    if is_decimal(a.dtype) or is_decimal(b.dtype):
        return _dec_arith(op, a, b, n, dev)
    rt = common_type(a.dtype if a.dtype != "interval" else "long", b.dtype if b.dtype != "interval" else "long")
    if op == "/":
        rt = "double"
    if rt == "null":
        rt = "int"                                      # NULL op NULL: Spark types the untyped NULLs as INT
    if rt not in INTEGRAL + ("double", "float", "decimal"):
        if a.dtype == "string" or b.dtype == "string":
            rt = "double"
            a = cast_column(a, "double")
            b = cast_column(b, "double")
        else:
            raise EvalError(f"cannot apply {op} to {a.dtype} and {b.dtype}")
    st = "double" if rt in ("double", "float", "decimal") else "long"
    x, y = _num_value(a, st), _num_value(b, st)
    if x is None or y is None:
        return ConstColumn(None, rt if op != "div" else "long", n, dev)
    valid = _result_valid(a, b)
    if _all_const(a, b):
        if op in ("/", "%", "div") and y == 0:
            return ConstColumn(None, rt, n, dev)
        r = {"+": lambda: x + y, "-": lambda: x - y, "*": lambda: x * y, "/": lambda: x / y,
             "%": lambda: math.fmod(x, y) if st == "double" else (0 if y == -1 else int(math.fmod(x, y))),
             "div": lambda: int(x // y) if (x >= 0) == (y >= 0) else -int(abs(x) // abs(y)),
             "&": lambda: int(x) & int(y), "|": lambda: int(x) | int(y), "^": lambda: int(x) ^ int(y)}[op]()
        if op == "div":
            return ConstColumn(wrap_int_value(r, "long"), "long", n, dev)
        # constant folding stays inside the result type: integer overflow wraps as the JVM's does
        return ConstColumn(wrap_int_value(r, rt) if st == "long" and op != "/" else r, rt, n, dev)
    if op == "+":
        r = x + y
    elif op == "-":
        r = x - y
    elif op == "*":
        r = x * y
    elif op == "/":
        xt = x.to(torch.float64) if torch.is_tensor(x) else torch.full((n,), float(x), dtype=torch.float64, device=dev)
        yt = y.to(torch.float64) if torch.is_tensor(y) else torch.full((n,), float(y), dtype=torch.float64, device=dev)
        zero = yt == 0
        r = xt / torch.where(zero, torch.ones_like(yt), yt)
        if bool(zero.any()):
            valid = and_valid(valid, ~zero)
    elif op in ("%", "div"):
        xt = x if torch.is_tensor(x) else torch.full((n,), x, device=dev,
                                                     dtype=torch.float64 if st == "double" else torch.int64)
        yt = y if torch.is_tensor(y) else torch.full((n,), y, device=dev,
                                                     dtype=torch.float64 if st == "double" else torch.int64)
        zero = yt == 0
        # integer x % -1 / x div -1 are computed without dividing (INT64_MIN / -1 traps on the host)
        neg1 = (yt == -1) if yt.dtype == torch.int64 else None
        bad = zero if neg1 is None else zero | neg1
        ys = torch.where(bad, torch.ones_like(yt), yt)
        if op == "%":
            r = torch.fmod(xt, ys)
            if neg1 is not None:
                r = torch.where(neg1, torch.zeros_like(r), r)
        else:
            r = torch.div(xt, ys, rounding_mode="trunc").to(torch.int64)
            if neg1 is not None:
                r = torch.where(neg1, -xt, r)
            rt = "long"
        if bool(zero.any()):
            valid = and_valid(valid, ~zero)
    elif op in ("&", "|", "^"):
        r = {"&": lambda: x & y, "|": lambda: x | y, "^": lambda: x ^ y}[op]()
    else:
        raise EvalError(op)
    if not torch.is_tensor(r):
        r = torch.full((n,), r, device=dev)
    if r.dim() == 0:
        r = r.expand(n).clone()
    if op in ("+", "-", "*") and st == "long":
        r = wrap_int_tensor(r, rt)                      # int / smallint / tinyint overflow wraps to the width
    return PrimColumn(rt, r, valid)


def _ts_arith(op, a, b, n, dev):
    # timestamp ± interval, timestamp - timestamp (→ interval µs as long)
    if a.dtype == "timestamp" and b.dtype in ("interval",) + INTEGRAL and op in ("+", "-"):
        x, y = _num_value(a, "long"), _num_value(b, "long")
        if x is None or y is None:
            return ConstColumn(None, "timestamp", n, dev)
        r = x + y if op == "+" else x - y
        if _all_const(a, b):
            return ConstColumn(r, "timestamp", n, dev)
        return PrimColumn("timestamp", r if torch.is_tensor(r) else torch.full((n,), r, device=dev),
                          _result_valid(a, b))
    if a.dtype == "timestamp" and b.dtype == "timestamp" and op == "-":
        x, y = _num_value(a, "long"), _num_value(b, "long")
        if _all_const(a, b):
            return ConstColumn(x - y, "long", n, dev)
        r = x - y
        return PrimColumn("long", r if torch.is_tensor(r) else torch.full((n,), r, device=dev), _result_valid(a, b))
    raise EvalError(f"unsupported timestamp arithmetic {a.dtype} {op} {b.dtype}")


def _compare(op: str, a: Column, b: Column, n, dev) -> Column:
    if op == "<=>":
        eq = _compare("=", a, b, n, dev)
        av, bv = as_prim(a).valid_mask(), as_prim(b).valid_mask()
        eqd = predicate_mask(eq)
        return bool_col((av & bv & eqd) | (~av & ~bv), None)
    # literal coercion
    if isinstance(b, ConstColumn) and not isinstance(a, ConstColumn):
        b = _coerce_const_for(a, b)
    if isinstance(a, ConstColumn) and not isinstance(b, ConstColumn):
        a = _coerce_const_for(b, a)
    if (isinstance(a, ConstColumn) and a.value is None) or (isinstance(b, ConstColumn) and b.value is None):
        return ConstColumn(None, "boolean", n, dev)
    if is_decimal(a.dtype) or is_decimal(b.dtype):
        kind, a, b = _dec_operands(a, b)
        if kind == "decimal" and not _all_const(a, b):
            return bool_col(D.compare_lanes(op, as_prim(a), as_prim(b), a.dtype, b.dtype), _result_valid(a, b))
    if _all_const(a, b):
        x, y = a.value, b.value
        try:
            r = {"=": x == y, "!=": x != y, "<": x < y, "<=": x <= y, ">": x > y, ">=": x >= y}[op]
        except TypeError:
            r = {"=": str(x) == str(y), "!=": str(x) != str(y), "<": str(x) < str(y), "<=": str(x) <= str(y),
                 ">": str(x) > str(y), ">=": str(x) >= str(y)}[op]
        return ConstColumn(r, "boolean", n, dev)
    valid = _result_valid(a, b)
    a_str = a.dtype == "string"
    b_str = b.dtype == "string"
    if a_str or b_str:
        from ..ops import strings as S
        if a_str and b_str:
            if isinstance(b, ConstColumn):
                r = S.cmp_literal(a, str(b.value), op)
            elif isinstance(a, ConstColumn):
                flip = {"<": ">", "<=": ">=", ">": "<", ">=": "<="}.get(op, op)
                r = S.cmp_literal(b, str(a.value), flip)
            else:
                r = S.compare_columns(a, b, op)
            return bool_col(r, valid)
        # string vs numeric/bool column: cast string side to the other type
        if a_str:
            a = cast_column(a, "double" if is_numeric(b.dtype) else b.dtype)
        else:
            b = cast_column(b, "double" if is_numeric(a.dtype) else a.dtype)
        valid = _result_valid(a, b)
    if a.dtype == "boolean" or b.dtype == "boolean":
        x = _scalar_or_tensor(a)
        y = _scalar_or_tensor(b)
        x = x.to(torch.int64) if torch.is_tensor(x) else int(bool(x))
        y = y.to(torch.int64) if torch.is_tensor(y) else int(bool(y))
    else:
        st = "double" if (a.dtype in ("double", "float", "decimal") or b.dtype in ("double", "float", "decimal")) \
            else "long"
        x, y = _num_value(a, st), _num_value(b, st)
    if op == "=":
        r = x == y
    elif op == "!=":
        r = x != y
    elif op == "<":
        r = x < y
    elif op == "<=":
        r = x <= y
    elif op == ">":
        r = x > y
    elif op == ">=":
        r = x >= y
    else:
        raise EvalError(op)
    if not torch.is_tensor(r):
        r = torch.full((n,), bool(r), device=dev)
    return bool_col(r, valid)


def _binop(e: A.BinOp, scope, ctx, subst):
    n, dev = scope.length, scope.device
    op = e.op
    if op in ("and", "or"):
        a = evaluate(e.left, scope, ctx, subst)
        # short-circuit constant folding keeps rules' IF(...) trees cheap
        if isinstance(a, ConstColumn):
            if op == "and" and a.value is False:
                return ConstColumn(False, "boolean", n, dev)
            if op == "or" and a.value is True:
                return ConstColumn(True, "boolean", n, dev)
        b = evaluate(e.right, scope, ctx, subst)
        return _logic(op, a, b, n, dev)
    a = evaluate(e.left, scope, ctx, subst)
    b = evaluate(e.right, scope, ctx, subst)
    if op in ("=", "!=", "<", "<=", ">", ">=", "<=>"):
        return _compare(op, a, b, n, dev)
    if op == "||":
        return _concat([a, b], n, dev)
    return _arith(op, a, b, n, dev)


def _like(e: A.Like, scope, ctx, subst):
    n, dev = scope.length, scope.device
    v = evaluate(e.operand, scope, ctx, subst)
    p = evaluate(e.pattern, scope, ctx, subst)
    if not isinstance(p, ConstColumn):
        raise EvalError("LIKE pattern must be a literal")
    if isinstance(v, ConstColumn):
        v = v.materialize()
    if v.dtype != "string":
        v = cast_column(v, "string")
    pat = str(p.value)
    from ..ops import strings as S
    if not e.regex:
        # fast paths on the device: 'abc', 'abc%', '%abc', '%abc%'
        body = pat.strip("%")
        plain = "%" not in body and "_" not in body and "\\" not in body
        if plain:
            if pat == body:
                r = S.cmp_literal(v, body, "=")
            elif pat == body + "%":
                r = S.cmp_literal(v, body, "startswith")
            elif pat == "%" + body:
                r = S.cmp_literal(v, body, "endswith")
            else:
                r = S.cmp_literal(v, body, "contains")
        elif isinstance(v, StrColumn) and v.starts.is_cuda:
            r = S.like(v, _like_tokens(pat))
        else:
            rx = re.compile(_like_to_regex(pat), re.S)
            r = torch.tensor([s is not None and rx.fullmatch(s) is not None for s in v.to_pylist()],
                             dtype=torch.bool, device=dev)
    else:
        from ..ops import regex_dfa
        dfa = None
        if isinstance(v, StrColumn) and v.starts.is_cuda:
            try:
                dfa = regex_dfa.compile_rlike(pat)
            except regex_dfa.Unsupported:
                dfa = None                              # outside the regular subset: host regex
        if dfa is not None:
            r = S.rlike(v, dfa)
        else:
            rx = re.compile(regex_dfa.java_to_python(pat), re.ASCII)
            r = torch.tensor([s is not None and rx.search(s) is not None for s in v.to_pylist()], dtype=torch.bool,
                             device=dev)
    out = bool_col(r, v.valid)
    return evaluate_not(out, n, dev) if e.negated else out


def _like_tokens(p: str) -> List[int]:
    """LIKE pattern → device tokens: literal bytes, 256 for '_', 257 for '%' (escapes resolved)."""
    out: List[int] = []
    i = 0
    while i < len(p):
        c = p[i]
        if c == "\\" and i + 1 < len(p):
            out.extend(p[i + 1].encode("utf-8"))
            i += 2
            continue
        if c == "%":
            if not out or out[-1] != 257:
                out.append(257)
        elif c == "_":
            out.append(256)
        else:
            out.extend(c.encode("utf-8"))
        i += 1
    return out


def _like_to_regex(p: str) -> str:
    out = []
    i = 0
    while i < len(p):
        c = p[i]
        if c == "\\" and i + 1 < len(p):
            out.append(re.escape(p[i + 1]))
            i += 2
            continue
        out.append(".*" if c == "%" else "." if c == "_" else re.escape(c))
        i += 1
    return "".join(out)


def choose(branch: torch.Tensor, options: List[Column], n, dev) -> Column:
    """Row-wise selection: result[i] = options[branch[i]][i] (branch == len(options) → null)."""
    if any(is_decimal(o.dtype) for o in options):
        target = _unify_type(options)
        if is_decimal(target):
            return _choose_decimal(branch, options, target, n, dev)
    if all(isinstance(o, ConstColumn) for o in options):
        vals = [o.value for o in options] + [None]
        dtype = next((o.dtype for o in options if o.value is not None), options[0].dtype)
        if dtype == "string":
            lits = strings_from_pylist(vals, dev)
            return lits.take(branch.to(torch.int64))
        if dtype == "null":
            return ConstColumn(None, "null", n, dev)
        tdt = TORCH_DTYPE.get(dtype, torch.float64)
        table = _h2d([0 if v is None else v for v in vals], tdt, dev)
        ok = _h2d([v is not None for v in vals], torch.bool, dev)
        b = branch.to(torch.int64)
        okb = ok[b]
        return PrimColumn(dtype, table[b], None if bool(okb.all()) else okb)
    k = len(options)
    ref = next(o for o in options if not (isinstance(o, ConstColumn) and o.value is None))
    opts = []
    target = _unify_type([o for o in options])
    for o in options:
        if isinstance(o, ConstColumn) and o.value is None:
            o = ConstColumn(None, target, n, dev)
        elif o.dtype != target and not is_nested(target):
            o = cast_column(o, target)
        opts.append(o)
    opts.append(ConstColumn(None, target, n, dev))
    if all(isinstance(o, (PrimColumn, ConstColumn)) and not is_nested(o.dtype) and o.dtype != "string"
           for o in opts):
        tdt = TORCH_DTYPE.get(target, torch.float64)
        datas = []
        valids = []
        for o in opts:
            if isinstance(o, ConstColumn):
                datas.append(torch.full((n,), 0 if o.value is None else o.value, dtype=tdt, device=dev))
                valids.append(torch.full((n,), o.value is not None, dtype=torch.bool, device=dev))
            else:
                datas.append(o.data.to(tdt))
                valids.append(o.valid_mask())
        b = branch.to(torch.int64).unsqueeze(0)
        data = torch.stack(datas).gather(0, b).squeeze(0)
        valid = torch.stack(valids).gather(0, b).squeeze(0)
        return PrimColumn(target, data, None if bool(valid.all()) else valid)
    big = concat_columns([materialize(o) if not isinstance(o, ConstColumn) or o.dtype == "string" else o
                          for o in opts])
    idx = branch.to(torch.int64) * n + torch.arange(n, device=dev)
    return big.take(idx)


def _choose_decimal(branch, options, target, n, dev):
    opts = []
    for o in options + [ConstColumn(None, target, n, dev)]:
        if isinstance(o, ConstColumn):
            o = ConstColumn(None if o.value is None else _cast_value(o.value, o.dtype, target), target, n, dev)
            o = o.materialize()
        elif o.dtype != target:
            o = cast_column(o, target)
        opts.append(o)
    b = branch.to(torch.int64)
    data = torch.stack([o.data for o in opts])
    idx = b.view(1, n, 1).expand(1, n, 2) if data.dim() == 3 else b.view(1, n)
    valid = torch.stack([o.valid_mask() for o in opts]).gather(0, b.view(1, n)).squeeze(0)
    return PrimColumn(target, data.gather(0, idx).squeeze(0), None if bool(valid.all()) else valid)


def _unify_type(cols):
    t = "null"
    for c in cols:
        if isinstance(c, ConstColumn) and c.value is None:
            continue
        t = c.dtype if t == "null" else (c.dtype if is_nested(c.dtype) else common_type(t, c.dtype))
    return t if t != "null" else "string"


def _case(e: A.Case, scope, ctx, subst):
    n, dev = scope.length, scope.device
    conds = []
    vals = []
    for w, t in e.whens:
        if e.operand is not None:
            c = _compare("=", evaluate(e.operand, scope, ctx, subst), evaluate(w, scope, ctx, subst), n, dev)
        else:
            c = evaluate(w, scope, ctx, subst)
        conds.append(c)
        vals.append(evaluate(t, scope, ctx, subst))
    default = evaluate(e.default, scope, ctx, subst) if e.default is not None else ConstColumn(None, "null", n, dev)
    return _select_by_conditions(conds, vals, default, n, dev)


def _select_by_conditions(conds, vals, default, n, dev):
    # IF(cond, X, NULL) fast path: just attach validity to X
    if len(conds) == 1 and isinstance(default, ConstColumn) and default.value is None:
        m = predicate_mask(conds[0])
        v = vals[0]
        if isinstance(v, ConstColumn) and not is_nested(v.dtype):
            v = v.materialize()
        return v.with_valid(m)
    if all(isinstance(c, ConstColumn) for c in conds):
        for c, v in zip(conds, vals):
            if c.value:
                return v
        return default
    branch = torch.full((n,), len(vals), dtype=torch.int64, device=dev)
    for i in range(len(conds) - 1, -1, -1):
        m = predicate_mask(conds[i])
        branch = torch.where(m, torch.full_like(branch, i), branch)
    return choose(branch, vals + [default], n, dev) if not (isinstance(default, ConstColumn) and
                                                             default.value is None) else choose(branch, vals, n, dev)


def _concat(parts: List[Column], n, dev):
    from ..ops import strings as S
    if all(isinstance(p, ConstColumn) for p in parts):
        if any(p.value is None for p in parts):
            return ConstColumn(None, "string", n, dev)
        return ConstColumn("".join(_const_str(p) for p in parts), "string", n, dev)
    args = []
    for p in parts:
        if isinstance(p, ConstColumn):
            if p.value is None:
                return ConstColumn(None, "string", n, dev)
            args.append(_const_str(p))
        else:
            args.append(p if p.dtype == "string" and isinstance(p, StrColumn) else cast_column(p, "string"))
    return S.concat_strings(args, n, dev)


def _const_str(c: ConstColumn) -> str:
    v = c.value
    if is_decimal(c.dtype):
        return D.render(v, c.dtype.scale)
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return F.java_double_str(v)
    if c.dtype == "timestamp":
        return F.format_timestamp_us(v, iso=False)
    return str(v)


# ---------------------------------------------------------------------------------------------------------------
# casts
# ---------------------------------------------------------------------------------------------------------------

def _complex_str(v, t) -> str:
    """Spark 2.4 ``Cast.castToString`` of an array / map / struct value (no spark.sql.legacy flag existed yet, this
    is the behaviour Spark 3.0 kept behind spark.sql.legacy.castComplexTypesToString.enabled): arrays ``[a, b]``,
    maps ``[k1 -> v1, k2 -> v2]``, structs ``[f1, f2]`` (maps and structs in brackets, not braces); a NULL element,
    map value or struct field is omitted, its separator kept (``array(1, NULL)`` → ``[1,]``); elements render as
    their own cast to string (no quotes).  JSON-text columns carry their parsed value with the schema type."""
    if v is None:
        return ""
    if isinstance(t, ArrayType) or (isinstance(v, list) and not isinstance(t, (MapType, StructType))):
        et = t.element if isinstance(t, ArrayType) else None
        out = "["
        for i, x in enumerate(v):
            if i:
                out += ","
            if x is not None:
                out += (" " if i else "") + _complex_str(x, et)
        return out + "]"
    if isinstance(t, MapType) or (isinstance(v, dict) and not isinstance(t, StructType)):
        kt, vt = (t.key, t.value) if isinstance(t, MapType) else (None, None)
        parts = []
        for k, x in v.items():
            parts.append(_complex_str(k, kt) + " ->" + ("" if x is None else " " + _complex_str(x, vt)))
        return "[" + ", ".join(parts) + "]"
    if isinstance(t, StructType) or isinstance(v, dict):
        fts = {f.name: f.dtype for f in t.fields} if isinstance(t, StructType) else {}
        out = "["
        for i, (k, x) in enumerate(v.items()):
            if i:
                out += ","
            if x is not None:
                out += (" " if i else "") + _complex_str(x, fts.get(k))
        return out + "]"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return F.java_double_str(v)
    import datetime as _dtm
    if isinstance(v, _dtm.datetime):
        return F.format_timestamp_us(int(round((v.replace(tzinfo=None) - _dtm.datetime(1970, 1, 1))
                                               .total_seconds() * 1e6)), iso=False)
    if isinstance(v, _dtm.date):
        return v.isoformat()
    if is_decimal(t):
        import decimal as _pd
        return D.render(_pd.Decimal(v), t.scale)
    return str(v)


def _d2i_value(v: float, to: str) -> int:
    """JVM double → integral conversion (Scala's ``toInt`` / ``toLong``, i.e. d2i / d2l): NaN → 0, saturating at the
    int (long) range, truncating toward zero; ``toShort`` / ``toByte`` are ``toInt`` then the low 16 / 8 bits."""
    if v != v:
        return 0
    lo, hi = INT_RANGE["long" if to == "long" else "int"]
    if v >= hi:
        r = hi
    elif v <= lo:
        r = lo
    else:
        r = int(v)
    return wrap_int_value(r, to)


def _d2i(d: torch.Tensor, to: str) -> torch.Tensor:
    """``_d2i_value`` over a float64 tensor."""
    lo, hi = INT_RANGE["long" if to == "long" else "int"]
    z = torch.where(torch.isnan(d), torch.zeros_like(d), d)
    # float(hi) rounds up to 2^63 for long: anything at or above it saturates to hi exactly
    r = torch.clamp(z, min=float(lo)).trunc()
    over = r >= float(hi)
    r = torch.where(over, torch.zeros_like(r), r).to(torch.int64)
    r = torch.where(over, torch.full_like(r, hi), r)
    return wrap_int_tensor(r, to)


def cast_column(col: Column, to: str) -> Column:
    to = {"integer": "int", "bigint": "long", "bool": "boolean", "smallint": "short", "tinyint": "byte"}.get(to, to)
    n, dev = col.length, col.device
    if col.dtype == to or (to == "string" and isinstance(col, StrColumn) and col.dtype == "string"):
        return col
    if isinstance(col, ConstColumn):
        return ConstColumn(_cast_value(col.value, col.dtype, to), to, n, dev)
    if is_decimal(to) or is_decimal(col.dtype):
        r = _cast_decimal(col, to)
        if r is not None:
            return r
    if to == "string":
        if isinstance(col, PrimColumn):
            if col.dtype in INTEGRAL:
                from ..ops import strings as S
                return S.from_int64(col.data, col.valid)
            if col.dtype in ("double", "float", "decimal") and col.data.is_cuda:
                from ..ops import native as N
                from ..ops.strings import _alloc_arena, _offsets
                d = col.data.to(torch.float64).contiguous()
                v = N.u8(col.valid)
                st = N.stream_handle(dev)
                lens = torch.empty(n, dtype=torch.int64, device=dev)
                N.call("dxa_f64_str_len", N.ptr(d), N.ptr(v), n, N.ptr(lens), st)
                off, total = _offsets(lens)
                arena = _alloc_arena(total, dev)
                N.call("dxa_f64_str_write", N.ptr(d), N.ptr(v), n, N.ptr(off), N.ptr(arena), st)
                return StrColumn(arena, off, lens.to(torch.int32), col.valid)
            if col.dtype == "boolean":
                return choose(torch.where(col.data, 0, 1).to(torch.int64),
                              [ConstColumn("true", "string", n, dev), ConstColumn("false", "string", n, dev)],
                              n, dev).with_valid(col.valid)
            vals = col.to_pylist()
            return strings_from_pylist([None if v is None else _cast_value(_storage_of(v, col.dtype), col.dtype,
                                                                          "string") for v in vals], dev)
        if isinstance(col, (StructColumn, ArrayColumn, JsonColumn)):
            t = col.dtype
            return strings_from_pylist([None if v is None else _complex_str(v, t) for v in col.to_pylist()], dev)
        raise EvalError(f"cannot cast {col.dtype} to string")
    if isinstance(col, StrColumn):
        if to == "timestamp":
            from ..ops import strings as S
            return S.to_timestamp(col)
        if to in INTEGRAL + ("double", "float", "decimal") and col.starts.is_cuda:
            from ..ops import native as N
            mode = 0 if to == "long" else (1 if to in INTEGRAL else 2)
            out = torch.empty(n, dtype=torch.int64, device=dev)
            ok = torch.empty(n, dtype=torch.uint8, device=dev)
            N.call("dxa_str_to_num", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), N.ptr(N.u8(col.valid)),
                   n, mode, N.ptr(out), N.ptr(ok), N.stream_handle(dev))
            okb = ok.view(torch.bool)
            if to in ("byte", "short"):                 # UTF8String.toByte / toShort: NULL outside the range
                lo, hi = INT_RANGE[to]
                okb = okb & (out >= lo) & (out <= hi)
            return PrimColumn(to, out.view(torch.float64) if mode == 2 else out, okb)
        vals = col.to_pylist()
        conv = [_cast_value(v, "string", to) for v in vals]
        return column_from_pylist(conv, to, dev)
    if isinstance(col, PrimColumn):
        d = col.data
        if to in INTEGRAL:
            if col.dtype == "timestamp":              # seconds (floor), then the width's low bits
                return PrimColumn(to, wrap_int_tensor(torch.div(d, 1_000_000, rounding_mode="floor"), to),
                                  col.valid)
            if d.dtype == torch.float64:
                return PrimColumn(to, _d2i(d, to), col.valid)
            return PrimColumn(to, wrap_int_tensor(d.to(torch.int64), to), col.valid)
        if to in ("double", "float", "decimal"):
            if col.dtype == "timestamp":
                return PrimColumn(to, D.true_div(d.to(torch.float64), 1e6), col.valid)
            return PrimColumn(to, d.to(torch.float64), col.valid)
        if to == "boolean":
            return PrimColumn("boolean", d != 0, col.valid)
        if to == "timestamp":
            if col.dtype == "date":
                return PrimColumn("timestamp", d * F.US_PER_DAY, col.valid)
            if d.dtype == torch.float64:
                return PrimColumn("timestamp", (d * 1e6).to(torch.int64), col.valid)
            return PrimColumn("timestamp", d.to(torch.int64) * 1_000_000, col.valid)
        if to == "date":
            if col.dtype == "timestamp":
                return PrimColumn("date", torch.div(d, F.US_PER_DAY, rounding_mode="floor"), col.valid)
    raise EvalError(f"cannot cast {col.dtype} to {to}")


def _cast_decimal(col: Column, to) -> Optional[Column]:
    """Casts into and out of decimal(p,s) (Spark Cast: HALF_UP to the scale, NULL on overflow; decimal → integral
    truncates toward zero)."""
    n, dev = col.length, col.device
    if is_decimal(to):
        if is_decimal(col.dtype):
            return D.change_type(col, to)
        if col.dtype in INTEGRAL + ("boolean",) and isinstance(col, PrimColumn):
            return D.from_integral(col, to)
        if col.dtype in ("double", "float") and isinstance(col, PrimColumn):
            return D.from_double(col, to)
        if col.dtype == "timestamp" and isinstance(col, PrimColumn):
            return D.from_double(PrimColumn("double", D.true_div(col.data.to(torch.float64), 1e6), col.valid), to)
        if col.dtype == "string" and isinstance(col, StrColumn):
            return D.from_text(col, to)
        raise EvalError(f"cannot cast {col.dtype} to {to}")
    if to in INTEGRAL:
        return D.to_integral(col, to)
    if to in ("double", "float"):
        return D.to_double(col)
    if to == "boolean":
        return D.to_boolean(col)
    if to == "string":
        return D.to_text_column(col)
    if to == "timestamp":
        d = D.to_double(col)
        return PrimColumn("timestamp", (d.data * 1e6).to(torch.int64), d.valid)
    return None


def _storage_of(v, dtype):
    from .column import datetime_to_us
    import datetime as dt
    if dtype == "timestamp" and isinstance(v, dt.datetime):
        return datetime_to_us(v)
    if dtype == "date" and isinstance(v, dt.date):
        return (v - dt.date(1970, 1, 1)).days
    return v


_CAST_WS = "".join(chr(c) for c in range(33))           # Spark trims bytes <= ' ' before numeric casts
_INT_STR = re.compile(r"^([+-]?)(\d*)(?:\.(\d*))?$")
_DBL_STR = re.compile(r"^[+-]?(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?$")


def _cast_value(v, frm, to):
    if v is None:
        return None
    if is_decimal(to):
        if frm == "timestamp":
            v = v / 1e6
        return D.cast_scalar(v, frm, to)
    if is_decimal(frm):
        if to == "timestamp":
            return int(float(v) * 1_000_000)
        return D.scalar_to(v, frm, to)
    try:
        if to == "string":
            if isinstance(v, bool):
                return "true" if v else "false"
            if frm == "timestamp":
                return F.format_timestamp_us(v, iso=False)
            if frm == "date":
                import datetime as dt
                return (dt.date(1970, 1, 1) + dt.timedelta(days=int(v))).isoformat()
            if isinstance(v, float):
                return F.java_double_str(v)
            return str(v)
        if to in INTEGRAL:
            if isinstance(v, str):
                # Spark (non-ANSI): [+-]digits[.digits] after trimming; the fraction truncates; no exponent; NULL
                # outside the type's range (UTF8String.toLong / toInt / toShort / toByte)
                m = _INT_STR.match(v.strip(_CAST_WS))
                if not m or not (m.group(2) or m.group(3)):
                    return None
                r = int((m.group(1) or "") + (m.group(2) or "0"))
                lo, hi = INT_RANGE[to]
                return r if lo <= r <= hi else None
            if frm == "timestamp":
                return wrap_int_value(int(v) // 1_000_000, to)
            if isinstance(v, float):
                return _d2i_value(v, to)
            return wrap_int_value(int(v), to)
        if to in ("double", "float", "decimal"):
            if isinstance(v, str):
                t = v.strip(_CAST_WS)
                low = t.lower()
                if low in ("inf", "+inf", "infinity", "+infinity"):
                    return float("inf")
                if low in ("-inf", "-infinity"):
                    return float("-inf")
                if low == "nan":
                    return float("nan")
                return float(t) if _DBL_STR.match(t) else None
            return float(v)
        if to == "boolean":
            if isinstance(v, str):
                s = v.strip().lower()
                if s in ("true", "t", "yes", "y", "1"):
                    return True
                if s in ("false", "f", "no", "n", "0"):
                    return False
                return None
            return bool(v)
        if to == "timestamp":
            if isinstance(v, str):
                return F.parse_timestamp_literal(v)
            if frm == "date":
                return int(v) * F.US_PER_DAY
            return int(float(v) * 1_000_000)
        if to == "date":
            if isinstance(v, str):
                us = F.parse_timestamp_literal(v)
                return None if us is None else us // F.US_PER_DAY
            if frm == "timestamp":
                return int(v) // F.US_PER_DAY
    except (ValueError, TypeError, OverflowError):
        return None
    raise EvalError(f"cannot cast {frm} to {to}")


# ---------------------------------------------------------------------------------------------------------------
# function calls
# ---------------------------------------------------------------------------------------------------------------

def _call(e: A.Call, scope: Scope, ctx: EvalContext, subst):
    n, dev = scope.length, scope.device
    name = e.name
    if name in AGG_FUNCS or name in ctx.udafs:
        raise EvalError(f"aggregate function {name}() is not allowed here")
    udf = ctx.udfs.get(name) or ctx.udfs.get(name.lower())
    if udf is not None:
        args = [evaluate(a, scope, ctx, subst) for a in e.args]
        return udf(args, ctx, n, dev)
    fn = _FUNCS.get(name)
    if fn is None:
        raise EvalError(f"undefined function {name}()")
    tok = _DEMOTE.set(None if name in _DECIMAL_AWARE else frozenset(id(a) for a in e.args))
    try:
        return fn(e, scope, ctx, subst)
    finally:
        _DEMOTE.reset(tok)


def _subquery(e: A.SubqueryExpr, scope: Scope, ctx: EvalContext, subst) -> Column:
    """Uncorrelated sub-queries: planned on their own against the statement's catalog."""
    from . import query as Q
    from .. import parallel as P
    n, dev = scope.length, scope.device
    if ctx.catalog is None:
        raise EvalError("sub-query outside a query")
    if e.kind in ("exists", "in"):
        hit = _correlated_semi(e, scope, ctx, subst)
        if hit is not None:
            return bool_col(~hit if e.negated else hit, None)
    try:
        t = Q.execute(e.query, ctx.catalog, ctx)
    except EvalError as err:
        raise EvalError(f"sub-query failed (only equality-correlated EXISTS / IN sub-queries are supported): "
                        f"{err}") from err
    if P.active() and P.dist_of(t) != P.REPLICATED:
        t = Q._gathered(t)
    if e.kind == "exists":
        return ConstColumn(t.length > 0, "boolean", n, dev)
    if len(t.columns) != 1:
        raise EvalError(f"sub-query must return one column, got {len(t.columns)}")
    rc = t.columns[0]
    if e.kind == "scalar":
        if t.length > 1:
            raise EvalError("scalar sub-query returned more than one row")
        v = rc.to_pylist()[0] if t.length else None
        return ConstColumn(v, rc.dtype, n, dev)
    # x [NOT] IN (SELECT c …): a semi-join membership test; SQL three-valued logic for nulls
    x = evaluate(e.operand, scope, ctx, subst)
    if isinstance(x, ConstColumn):
        x = x.materialize()
    rc = rc.materialize() if isinstance(rc, ConstColumn) else rc
    from ..ops import join as J
    from .query import _coerce_keys
    xs, rs = _coerce_keys([x], [rc])
    hit = torch.zeros(n, dtype=torch.bool, device=dev)
    if n and t.length:
        li, _ = J.hash_join(xs, rs, "semi")
        hit[li] = True
    rhs_null = bool((~rc.valid).any()) if (t.length and rc.valid is not None) else False
    valid = x.valid_mask() & (hit | (not rhs_null)) if (x.valid is not None or rhs_null) else None
    return bool_col(~hit if e.negated else hit, valid)


def _correlated_semi(e: A.SubqueryExpr, scope: Scope, ctx: EvalContext, subst) -> Optional[torch.Tensor]:
    """Decorrelate ``EXISTS (SELECT … FROM s WHERE s.k = outer.k AND …)`` and the IN form into a semi-join on the
    equality keys (plus the IN operand / select item).  None when the sub-query is not correlated that way."""
    from . import query as Q
    from .. import parallel as P
    from ..ops import join as J
    q = e.query
    body = q.body
    if q.ctes or not isinstance(body, A.Select) or body.where is None or body.group_by or body.having is not None:
        return None
    inner_probe = None
    outer_keys, inner_keys, rest = [], [], []
    for c in Q._split_and(body.where):
        if isinstance(c, A.BinOp) and c.op == "=":
            if inner_probe is None:
                inner_probe = Q._relation(body.from_, ctx.catalog, ctx)
            l_in, r_in = Q._refs_resolvable(c.left, inner_probe), Q._refs_resolvable(c.right, inner_probe)
            if l_in and not r_in and Q._refs_resolvable(c.right, scope):
                inner_keys.append(c.left)
                outer_keys.append(c.right)
                continue
            if r_in and not l_in and Q._refs_resolvable(c.left, scope):
                inner_keys.append(c.right)
                outer_keys.append(c.left)
                continue
        rest.append(c)
    if not outer_keys:
        return None
    inner = inner_probe
    for c in rest:
        if not Q._refs_resolvable(c, inner):
            raise EvalError("correlated sub-query predicates other than equality are not supported")
    if rest:
        m = None
        for c in rest:
            mc = predicate_mask(evaluate(c, inner, ctx))
            m = mc if m is None else m & mc
        idx = torch.nonzero(m).flatten()
        inner = Scope(inner.names, TakenColumns(inner.cols, idx), inner.quals, int(idx.shape[0]), inner.device)
    if e.kind == "in":
        items = Q._expand_items(body, inner)
        if len(items) != 1:
            raise EvalError("IN sub-query must return one column")
        inner_keys.append(items[0][0])
        outer_keys.append(e.operand)
    if P.active() and getattr(inner_probe, "dist", P.REPLICATED) != P.REPLICATED:
        inner = Q._gather_scope(inner)
    n = scope.length
    hit = torch.zeros(n, dtype=torch.bool, device=scope.device)
    if n and inner.length:
        ok = [materialize(evaluate(k, scope, ctx, subst)) for k in outer_keys]
        ik = [materialize(evaluate(k, inner, ctx)) for k in inner_keys]
        ok, ik = Q._coerce_keys(ok, ik)
        li, _ = J.hash_join(ok, ik, "semi")
        hit[li] = True
    return hit


def _lambda_arg(e: A.Call, k: int) -> A.Lambda:
    if len(e.args) <= k or not isinstance(e.args[k], A.Lambda):
        raise EvalError(f"{e.name}() expects a lambda as argument {k + 1}")
    return e.args[k]


def _hof_elements(e: A.Call, scope, ctx, subst):
    arr = evaluate(e.args[0], scope, ctx, subst)
    if not isinstance(arr, ArrayColumn):
        raise EvalError(f"{e.name}() expects an array")
    return arr


def _slot_present(arr: "ArrayColumn", el) -> torch.Tensor:
    """Element slot is part of the array (a dropped-null slot is not)."""
    n = arr.length
    base = arr.valid_mask() if arr.valid is not None else torch.ones(n, dtype=torch.bool, device=arr.device)
    if arr.present is not None:
        j = next((j for j, x in enumerate(arr.elements) if x is el), None)
        if j is not None:
            base = base & arr.present[:, j]
    if arr.drop_nulls:
        if isinstance(el, ConstColumn):
            return base & (el.value is not None)
        return base & el.valid_mask()
    return base


def _f_transform(e, scope, ctx, subst):
    """transform(arr, x -> f(x)) / transform(arr, (x, i) -> f(x, i))."""
    arr = _hof_elements(e, scope, ctx, subst)
    lam = _lambda_arg(e, 1)
    out = []
    for j, el in enumerate(arr.elements):
        binds = [el] + ([ConstColumn(j, "int", arr.length, arr.device)] if len(lam.params) > 1 else [])
        v = evaluate(lam.body, scope.with_bindings(list(lam.params[:len(binds)]), binds), ctx, subst)
        if arr.drop_nulls:                            # keep the slot structure: absent slots stay absent
            v = v.materialize() if isinstance(v, ConstColumn) else v
            v = v.with_valid(_slot_present(arr, el))
        out.append(v)
    return ArrayColumn(out, arr.length, arr.valid, arr.drop_nulls, arr.device)


def _f_array_filter(e, scope, ctx, subst):
    """filter(arr, x -> pred): slots failing the predicate are dropped."""
    arr = _hof_elements(e, scope, ctx, subst)
    lam = _lambda_arg(e, 1)
    out = []
    for j, el in enumerate(arr.elements):
        binds = [el] + ([ConstColumn(j, "int", arr.length, arr.device)] if len(lam.params) > 1 else [])
        keep = predicate_mask(evaluate(lam.body, scope.with_bindings(list(lam.params[:len(binds)]), binds), ctx,
                                       subst)) & _slot_present(arr, el)
        m = el.materialize() if isinstance(el, ConstColumn) else el
        out.append(m.with_valid(keep))
    return ArrayColumn(out, arr.length, arr.valid, True, arr.device)


def _f_array_exists(kind):
    def f(e, scope, ctx, subst):
        arr = _hof_elements(e, scope, ctx, subst)
        lam = _lambda_arg(e, 1)
        acc = torch.zeros(arr.length, dtype=torch.bool, device=arr.device) if kind == "exists" else \
            torch.ones(arr.length, dtype=torch.bool, device=arr.device)
        for el in arr.elements:
            p = predicate_mask(evaluate(lam.body, scope.with_bindings([lam.params[0]], [el]), ctx, subst))
            pres = _slot_present(arr, el)
            acc = (acc | (p & pres)) if kind == "exists" else (acc & (p | ~pres))
        return bool_col(acc, arr.valid)
    return f


def _f_array_aggregate(e, scope, ctx, subst):
    """aggregate(arr, init, (acc, x) -> merge [, acc -> finish])."""
    arr = _hof_elements(e, scope, ctx, subst)
    acc = evaluate(e.args[1], scope, ctx, subst)
    merge = _lambda_arg(e, 2)
    for el in arr.elements:
        nxt = evaluate(merge.body, scope.with_bindings(list(merge.params[:2]), [acc, el]), ctx, subst)
        pres = _slot_present(arr, el)
        acc = _select_by_conditions([bool_col(pres, None)], [nxt], acc, arr.length, arr.device)
    if len(e.args) > 3:
        fin = _lambda_arg(e, 3)
        acc = evaluate(fin.body, scope.with_bindings([fin.params[0]], [acc]), ctx, subst)
    return acc.with_valid(arr.valid) if arr.valid is not None else acc


def _args(e, scope, ctx, subst):
    return [evaluate(a, scope, ctx, subst) for a in e.args]


def _f_if(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    c, a, b = _args(e, scope, ctx, subst)
    return _select_by_conditions([c], [a], b, n, dev)


def _f_coalesce(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    cols = _args(e, scope, ctx, subst)
    conds = []
    for c in cols[:-1]:
        if isinstance(c, ConstColumn):
            conds.append(ConstColumn(c.value is not None, "boolean", n, dev))
        else:
            conds.append(bool_col(c.valid_mask(), None))
    return _select_by_conditions(conds, cols[:-1], cols[-1], n, dev)


def _f_nullif(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    a, b = _args(e, scope, ctx, subst)
    eq = _compare("=", a, b, n, dev)
    return _select_by_conditions([eq], [ConstColumn(None, a.dtype, n, dev)], a, n, dev)


def _f_map(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    if len(e.args) % 2:
        raise EvalError("map() expects key/value pairs")
    names, cols = [], []
    for i in range(0, len(e.args), 2):
        k = evaluate(e.args[i], scope, ctx, subst)
        if not isinstance(k, ConstColumn):
            raise EvalError("map() keys must be constants")
        names.append(_const_str(k))
        cols.append(evaluate(e.args[i + 1], scope, ctx, subst))
    return StructColumn(names, cols, n, None, True, None, dev)


def _expr_name(a: A.Expr, i: int) -> str:
    if isinstance(a, A.Ident):
        return a.parts[-1]
    return f"col{i + 1}"


def _f_struct(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    cols = _args(e, scope, ctx, subst)
    return StructColumn([_expr_name(a, i) for i, a in enumerate(e.args)], cols, n, None, False, None, dev)


def _f_named_struct(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    names, cols = [], []
    for i in range(0, len(e.args), 2):
        k = evaluate(e.args[i], scope, ctx, subst)
        names.append(_const_str(k))
        cols.append(evaluate(e.args[i + 1], scope, ctx, subst))
    return StructColumn(names, cols, n, None, False, None, dev)


def _f_array(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    return ArrayColumn(_args(e, scope, ctx, subst), n, None, False, dev)


def _f_filternull(e, scope, ctx, subst):
    (a,) = _args(e, scope, ctx, subst)
    if isinstance(a, ArrayColumn):
        return ArrayColumn(a.elements, a.length, a.valid, True, a.device)
    raise EvalError("filterNull() expects an array")


def _f_size(e, scope, ctx, subst):
    """size / cardinality: the number of present slots; Spark 2.4 (spark.sql.legacy.sizeOfNull) gives -1 for a NULL
    array or map."""
    n, dev = scope.length, scope.device
    (a,) = _args(e, scope, ctx, subst)
    if isinstance(a, ArrayColumn):
        cnt = torch.zeros(n, dtype=torch.int64, device=dev)
        ones = torch.ones(n, dtype=torch.bool, device=dev)
        for el in a.elements:
            p = _slot_present(ArrayColumn(a.elements, n, None, a.drop_nulls, dev, present=a.present), el)
            cnt += (p if isinstance(p, torch.Tensor) else ones & bool(p)).to(torch.int64)
        if a.valid is not None:
            cnt = torch.where(a.valid, cnt, torch.full_like(cnt, -1))
        return PrimColumn("int", cnt)
    vals = a.to_pylist()
    return column_from_pylist([-1 if v is None else len(v) for v in vals], "int", dev)


def _f_abs(e, scope, ctx, subst):
    (a,) = _args(e, scope, ctx, subst)
    if is_decimal(a.dtype):
        if isinstance(a, ConstColumn):
            return ConstColumn(None if a.value is None else abs(a.value), a.dtype, a.length, a.device)
        return D.absolute(a)
    r = _ABS_NUM(e, scope, ctx, subst)
    if r.dtype in INTEGRAL:                             # abs(MIN_VALUE) is MIN_VALUE (Java Math.abs)
        if isinstance(r, ConstColumn):
            return ConstColumn(None if r.value is None else wrap_int_value(r.value, r.dtype), r.dtype, r.length,
                               r.device)
        return PrimColumn(r.dtype, wrap_int_tensor(r.data, r.dtype), r.valid)
    return r


def _f_ceil_floor(up: bool):
    """ceil / floor: a decimal stays a decimal, decimal(p - s + 1, 0) (Spark 2.4 Ceil / Floor); a double (and
    anything implicitly cast to one) becomes a BIGINT by ``Math.ceil(x).toLong`` (saturating, NaN → 0); a BIGINT is
    unchanged."""
    base = _unary_num(torch.ceil if up else torch.floor, "long")

    def f(e, scope, ctx, subst):
        (a,) = _args(e, scope, ctx, subst)
        if is_decimal(a.dtype):
            if isinstance(a, ConstColumn):
                import decimal as _pd
                rt = D.bounded(a.dtype.precision - a.dtype.scale + 1, 0)
                if a.value is None:
                    return ConstColumn(None, rt, a.length, a.device)
                v = _pd.Decimal(a.value).to_integral_value(_pd.ROUND_CEILING if up else _pd.ROUND_FLOOR)
                return ConstColumn(v, rt, a.length, a.device)
            return D.ceil_floor_column(a, up)
        if a.dtype in INTEGRAL:
            return cast_column(a, "long")
        if isinstance(a, ConstColumn):
            if a.value is None:
                return ConstColumn(None, "long", a.length, a.device)
            x = float(a.value)
            return ConstColumn(_d2i_value(math.ceil(x) if up and math.isfinite(x) else
                                          (math.floor(x) if math.isfinite(x) else x), "long"), "long", a.length,
                               a.device)
        x = a.data.to(torch.float64)
        return PrimColumn("long", _d2i(torch.ceil(x) if up else torch.floor(x), "long"), a.valid)
    return f


def _unary_num(fn, out_type=None):
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        (a,) = _args(e, scope, ctx, subst)
        if isinstance(a, ConstColumn):
            if a.value is None:
                return a
            t = torch.tensor([a.value], dtype=torch.float64 if out_type == "double" or isinstance(a.value, float)
                             else torch.int64)
            r = fn(t)
            v = r.item()
            return ConstColumn(v, out_type or a.dtype, n, dev)
        d = a.data
        if out_type == "double":
            d = d.to(torch.float64)
        r = fn(d)
        rt = out_type or a.dtype
        if rt in INTEGRAL and r.dtype == torch.float64:
            r = r.to(torch.int64)
        return PrimColumn(rt, r, a.valid)
    return f


_ABS_NUM = _unary_num(torch.abs)


def _f_round(e, scope, ctx, subst):
    """round (HALF_UP) / bround (HALF_EVEN) — Spark 2.4's RoundBase:

    * decimal(p, s) → decimal(p, min(s, d)), exact (``decimal.round_column``);
    * double / float → ``BigDecimal(x).setScale(d, mode).toDouble``, where Scala's ``BigDecimal(x)`` is the shortest
      decimal that reads back as x (``Double.toString``).  So ``round(1.005, 2)`` on a double is 1.01, not the 1.0 that
      scaling the binary value gives.  On the device: t = (2f+1) / (2·10^d) is the double nearest to the tie point
      f + ½ above f = ⌊|x|·10^d⌋ (one correctly rounded division of exact operands).  x above t rounds up, below
      rounds down, and x == t is the tie, decided by the mode.  A double equal to the tie's nearest double has the
      tie as its shortest form except at 16-17 significant digits;
    * int / long: unchanged for d ≥ 0, rounded to 10^-d otherwise."""
    n, dev = scope.length, scope.device
    a = evaluate(e.args[0], scope, ctx, subst)
    digits = int(evaluate(e.args[1], scope, ctx, subst).value) if len(e.args) > 1 else 0
    half_even = e.name == "bround"
    if isinstance(a, ConstColumn):
        a = a.materialize()
    if is_decimal(a.dtype):
        return D.round_column(a, digits, half_even)
    if a.dtype in ("int", "long", "short", "byte"):
        if digits >= 0:
            return a
        m = 10 ** (-digits)
        x = a.data.to(torch.int64)
        q, r = torch.div(x.abs(), m, rounding_mode="floor"), x.abs() % m
        up = (2 * r > m) | ((2 * r == m) & (~torch.tensor(half_even, device=x.device) | (q % 2 == 1)))
        res = torch.sign(x) * (q + up.to(torch.int64)) * m
        return PrimColumn(a.dtype, res.to(a.data.dtype), a.valid)
    x = a.data.to(torch.float64)
    ax = x.abs()
    # (divisions through D.true_div: the GPU's scalar division is a reciprocal multiply, an ulp off at the ties)
    if digits >= 0:
        sc = 10.0 ** digits if digits <= 308 else float("inf")
        scaled = ax * sc
        f = torch.floor(scaled)
        t = D.true_div(2 * f + 1, 2 * sc)
    else:
        sc = 10.0 ** (-digits) if digits >= -308 else float("inf")
        f = torch.floor(D.true_div(ax, sc))
        t = (2 * f + 1) * sc / 2
    tie_up = (torch.remainder(f, 2) == 1) if half_even else torch.ones_like(ax, dtype=torch.bool)
    r = f + ((ax > t) | ((ax == t) & tie_up)).to(torch.float64)
    res = torch.sign(x) * (D.true_div(r, sc) if digits >= 0 else r * sc)
    if digits >= 0:
        # |x|·10^d beyond 2^53 (or overflowing): x has no digits below 10^-d, so BigDecimal(x).setScale(d) is x
        keep = ~torch.isfinite(scaled) | (scaled >= 2.0 ** 53)
        res = torch.where(keep, x, res)
    elif sc == float("inf"):
        res = torch.zeros_like(x)                                 # rounded left of every digit a double has
    res = torch.where(torch.isfinite(x), res, x)                  # NaN / ±Infinity pass through
    rt = "float" if a.dtype == "float" else "double"
    if rt == "float":
        res = res.to(a.data.dtype)
    return PrimColumn(rt, res, a.valid)


def _f_ts_part(part):
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        (a,) = _args(e, scope, ctx, subst)
        if a.dtype == "string":
            a = cast_column(a, "timestamp")
        if a.dtype == "date":
            a = cast_column(a, "timestamp")
        if isinstance(a, ConstColumn):
            if a.value is None:
                return ConstColumn(None, "int", n, dev)
            return ConstColumn(int(F.ts_part(torch.tensor([a.value]), part)[0]), "int", n, dev)
        return PrimColumn("int", F.ts_part(a.data, part), a.valid)
    return f


def _f_date_trunc(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    unit, a = _args(e, scope, ctx, subst)
    if a.dtype == "string":
        a = cast_column(a, "timestamp")
    if isinstance(a, ConstColumn):
        if a.value is None:
            return a
        return ConstColumn(int(F.ts_trunc(torch.tensor([a.value]), str(unit.value))[0]), "timestamp", n, dev)
    return PrimColumn("timestamp", F.ts_trunc(a.data, str(unit.value)), a.valid)


def _f_trunc(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    a, unit = _args(e, scope, ctx, subst)
    a = cast_column(a, "timestamp") if a.dtype != "timestamp" else a
    if isinstance(a, ConstColumn):
        return ConstColumn(int(F.ts_trunc(torch.tensor([a.value]), str(unit.value))[0]) // F.US_PER_DAY, "date", n,
                           dev)
    return PrimColumn("date", F.ts_trunc(a.data, str(unit.value)) // F.US_PER_DAY, a.valid)


def _f_now(e, scope, ctx, subst):
    return ConstColumn(ctx.now_us, "timestamp", scope.length, scope.device)


def _f_current_date(e, scope, ctx, subst):
    return ConstColumn(ctx.now_us // F.US_PER_DAY, "date", scope.length, scope.device)


def _f_unix_timestamp(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    if not e.args:
        return ConstColumn(ctx.now_us // 1_000_000, "long", n, dev)
    a = evaluate(e.args[0], scope, ctx, subst)
    if a.dtype != "timestamp":
        a = cast_column(a, "timestamp")
    if isinstance(a, ConstColumn):
        return ConstColumn(None if a.value is None else a.value // 1_000_000, "long", n, dev)
    return PrimColumn("long", torch.div(a.data, 1_000_000, rounding_mode="floor"), a.valid)


def _f_from_unixtime(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    a = evaluate(e.args[0], scope, ctx, subst)
    ts = cast_column(a, "timestamp")
    return cast_column(ts, "string")


def _f_to_timestamp(e, scope, ctx, subst):
    a = evaluate(e.args[0], scope, ctx, subst)
    return cast_column(a, "timestamp")


def _f_to_date(e, scope, ctx, subst):
    a = evaluate(e.args[0], scope, ctx, subst)
    return cast_column(cast_column(a, "timestamp") if a.dtype != "timestamp" else a, "date")


def _f_string_to_ts(e, scope, ctx, subst):
    (a,) = _args(e, scope, ctx, subst)
    if a.dtype != "string":
        # the reference's UDF takes a String: Spark casts the argument first
        a = cast_column(a, "string")
    if isinstance(a, ConstColumn):
        from ..ops.strings import py_string_to_timestamp_us
        return ConstColumn(py_string_to_timestamp_us(a.value), "timestamp", scope.length, scope.device)
    pre = getattr(a, "_parsed_ts", None)          # converted by the JSON parser from the same bytes (ParsePlan)
    if pre is not None and pre.length == a.length:
        return pre
    from ..ops import strings as S
    r = S.to_timestamp(a)
    return r


def _f_concat(e, scope, ctx, subst):
    return _concat(_args(e, scope, ctx, subst), scope.length, scope.device)


def _f_concat_ws(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    args = _args(e, scope, ctx, subst)
    sep = args[0]
    if isinstance(sep, ConstColumn) and sep.value is None:
        return ConstColumn(None, "string", n, dev)
    parts = []
    for i, a in enumerate(args[1:]):
        if i:
            parts.append(sep)
        parts.append(a)
    # Spark concat_ws skips nulls: on the GPU one skip-aware kernel pair; host-assisted elsewhere
    if dev.type == "cuda" and isinstance(sep, ConstColumn) and sep.value is not None and \
            not any(isinstance(p, ArrayColumn) for p in args[1:]):
        from ..ops import strings as S
        ps = []
        for p in args[1:]:
            if isinstance(p, ConstColumn):
                if p.value is not None:
                    ps.append(_const_str(p))
                continue
            ps.append(p if isinstance(p, StrColumn) else cast_column(p, "string"))
        return S.concat_ws(_const_str(sep), ps, n, dev)
    nullable = any((p.value is None) if isinstance(p, ConstColumn) else p.valid is not None for p in args[1:])
    if nullable or any(isinstance(p, ArrayColumn) for p in args[1:]) or not isinstance(sep, ConstColumn):
        # host: NULL arguments (and NULL array elements) are skipped, array<string> arguments contribute their
        # elements; a NULL separator makes the result NULL (Spark ConcatWs)
        seps = sep.to_pylist() if not isinstance(sep, ConstColumn) else [sep.value] * n
        cols = []
        for p in args[1:]:
            if isinstance(p, ArrayColumn):
                cols.append(("arr", p.to_pylist()))
            elif isinstance(p, ConstColumn):
                cols.append(("val", [None if p.value is None else _const_str(p)] * n))
            else:
                cols.append(("val", cast_column(p, "string").to_pylist()))
        out = []
        for i in range(n):
            if seps[i] is None:
                out.append(None)
                continue
            items = []
            for kind, c in cols:
                v = c[i]
                if v is None:
                    continue
                if kind == "arr":
                    items.extend(x if isinstance(x, str) else _complex_str(x, None) for x in v if x is not None)
                else:
                    items.append(v)
            out.append(str(seps[i]).join(items))
        return strings_from_pylist(out, dev)
    return _concat(parts, n, dev)


def _f_case_map(upper):
    def f(e, scope, ctx, subst):
        (a,) = _args(e, scope, ctx, subst)
        if isinstance(a, ConstColumn):
            return ConstColumn(None if a.value is None else (str(a.value).upper() if upper else str(a.value).lower()),
                               "string", a.length, a.device)
        from ..ops import strings as S
        return S.case_map(a if a.dtype == "string" else cast_column(a, "string"), upper)
    return f


def _f_length(e, scope, ctx, subst):
    (a,) = _args(e, scope, ctx, subst)
    if isinstance(a, ConstColumn):
        return ConstColumn(None if a.value is None else len(str(a.value)), "int", a.length, a.device)
    if not isinstance(a, StrColumn):
        a = cast_column(a, "string")
    # byte length == char length for ASCII; count UTF-8 lead bytes otherwise (host-assisted)
    return PrimColumn("int", a.lens.to(torch.int64), a.valid) if _ascii_only(a) else column_from_pylist(
        [None if v is None else len(v) for v in a.to_pylist()], "int", a.device)


def _ascii_only(a: StrColumn) -> bool:
    return True


def _host_string_fn(fn, out_type="string"):
    """Host-assisted string function: fn(*python_values) per row."""
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        args = _args(e, scope, ctx, subst)
        lists = [a.to_pylist() if not isinstance(a, ConstColumn) else [a.value] * n for a in args]
        out = []
        for i in range(n):
            vals = [l[i] for l in lists]
            if vals and vals[0] is None:
                out.append(None)
                continue
            try:
                out.append(fn(*vals))
            except Exception:
                out.append(None)
        if all(isinstance(a, ConstColumn) for a in args):
            return ConstColumn(out[0] if out else None, out_type, n, dev)
        return column_from_pylist(out, out_type, dev)
    return f


def _substr(s, pos, ln=None):
    s = str(s)
    pos = int(pos)
    if pos > 0:
        start = pos - 1
    elif pos < 0:
        start = max(0, len(s) + pos)
    else:
        start = 0
    if ln is None:
        return s[start:]
    return s[start:start + max(0, int(ln))]


def _f_greatest_least(kind):
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        cols = _args(e, scope, ctx, subst)
        t = _unify_type(cols)
        st = "double" if t in ("double", "float", "decimal") else "long"
        acc = None
        accv = None
        for c in cols:
            c = as_prim(c)
            d = c.data.to(torch.float64 if st == "double" else torch.int64)
            v = c.valid_mask()
            if acc is None:
                acc, accv = d, v
                continue
            better = (d > acc) if kind == "greatest" else (d < acc)
            take = v & (~accv | better)
            acc = torch.where(take, d, acc)
            accv = accv | v
        return PrimColumn(t, acc, accv)
    return f


def _f_isnull(neg):
    def f(e, scope, ctx, subst):
        return evaluate(A.IsNull(e.args[0], neg), scope, ctx, subst)
    return f


def _f_nvl2(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    a, b, c = _args(e, scope, ctx, subst)
    cond = ConstColumn(a.value is not None, "boolean", n, dev) if isinstance(a, ConstColumn) else bool_col(
        a.valid_mask(), None)
    return _select_by_conditions([cond], [b], c, n, dev)


def _f_element_at(e, scope, ctx, subst):
    base = evaluate(e.args[0], scope, ctx, subst)
    k = evaluate(e.args[1], scope, ctx, subst)
    if isinstance(base, ArrayColumn):
        i = int(k.value) - 1
        return base.elements[i] if 0 <= i < len(base.elements) else ConstColumn(None, "null", base.length,
                                                                                base.device)
    return field_access(base, str(k.value))


def _f_to_json(e, scope, ctx, subst):
    (a,) = _args(e, scope, ctx, subst)
    from .serialize import column_json_values
    return strings_from_pylist(column_json_values(a), scope.device)


def _f_monotonic(e, scope, ctx, subst):
    return PrimColumn("long", torch.arange(scope.length, dtype=torch.int64, device=scope.device))


_FUNCS: Dict[str, Callable] = {
    "if": _f_if, "iff": _f_if, "coalesce": _f_coalesce, "ifnull": _f_coalesce, "nvl": _f_coalesce,
    "nullif": _f_nullif, "nvl2": _f_nvl2, "isnull": _f_isnull(False), "isnotnull": _f_isnull(True),
    "map": _f_map, "struct": _f_struct, "named_struct": _f_named_struct, "array": _f_array,
    "filternull": _f_filternull, "size": _f_size, "cardinality": _f_size, "element_at": _f_element_at,
    "abs": _f_abs, "floor": _f_ceil_floor(False), "ceil": _f_ceil_floor(True), "ceiling": _f_ceil_floor(True),
    "sqrt": _unary_num(torch.sqrt, "double"),
    "exp": _unary_num(torch.exp, "double"), "ln": _unary_num(torch.log, "double"),
    "log10": _unary_num(torch.log10, "double"), "log2": _unary_num(torch.log2, "double"),
    "sign": _unary_num(torch.sign, "double"), "signum": _unary_num(torch.sign, "double"),
    "round": _f_round, "bround": _f_round,
    "hour": _f_ts_part("hour"), "minute": _f_ts_part("minute"), "second": _f_ts_part("second"),
    "year": _f_ts_part("year"), "month": _f_ts_part("month"), "day": _f_ts_part("day"),
    "dayofmonth": _f_ts_part("dayofmonth"), "dayofweek": _f_ts_part("dayofweek"),
    "weekday": _f_ts_part("weekday"), "dayofyear": _f_ts_part("dayofyear"), "quarter": _f_ts_part("quarter"),
    "date_trunc": _f_date_trunc, "trunc": _f_trunc, "current_timestamp": _f_now, "now": _f_now,
    "current_date": _f_current_date, "unix_timestamp": _f_unix_timestamp, "from_unixtime": _f_from_unixtime,
    "to_timestamp": _f_to_timestamp, "to_date": _f_to_date, "stringtotimestamp": _f_string_to_ts,
    "concat": _f_concat, "concat_ws": _f_concat_ws, "lower": _f_case_map(False), "lcase": _f_case_map(False),
    "upper": _f_case_map(True), "ucase": _f_case_map(True), "length": _f_length, "char_length": _f_length,
    "character_length": _f_length,
    "substring": _host_string_fn(_substr), "substr": _host_string_fn(_substr),
    "trim": _host_string_fn(lambda s: str(s).strip(" ")), "ltrim": _host_string_fn(lambda s: str(s).lstrip(" ")),
    "rtrim": _host_string_fn(lambda s: str(s).rstrip(" ")),
    "replace": _host_string_fn(lambda s, a, b="": str(s).replace(str(a), str(b))),
    "instr": _host_string_fn(lambda s, sub: str(s).find(str(sub)) + 1, "int"),
    "locate": _host_string_fn(lambda sub, s, pos=1: str(s).find(str(sub), max(0, int(pos) - 1)) + 1, "int"),
    "regexp_replace": _host_string_fn(lambda s, p, r: re.sub(p, re.sub(r"\$(\d)", r"\\\1", r), str(s))),
    "regexp_extract": _host_string_fn(lambda s, p, g=1: (lambda m: m.group(int(g)) if m else "")(re.search(p, str(s)))),
    "split_part": _host_string_fn(lambda s, d, i: (str(s).split(str(d)) + [""] * int(i))[int(i) - 1]),
    "lpad": _host_string_fn(lambda s, l, p=" ": (str(p) * int(l) + str(s))[-int(l):] if len(str(s)) < int(l)
                            else str(s)[:int(l)]),
    "rpad": _host_string_fn(lambda s, l, p=" ": (str(s) + str(p) * int(l))[:int(l)]),
    "reverse": _host_string_fn(lambda s: str(s)[::-1]),
    "md5": _host_string_fn(lambda s: __import__("hashlib").md5(str(s).encode()).hexdigest()),
    "sha1": _host_string_fn(lambda s: __import__("hashlib").sha1(str(s).encode()).hexdigest()),
    "uuid": _host_string_fn(lambda *a: str(__import__("uuid").uuid4())),
    "greatest": _f_greatest_least("greatest"), "least": _f_greatest_least("least"),
    "to_json": _f_to_json, "monotonically_increasing_id": _f_monotonic,
    "transform": _f_transform, "filter": _f_array_filter, "exists": _f_array_exists("exists"),
    "forall": _f_array_exists("forall"), "aggregate": _f_array_aggregate, "reduce": _f_array_aggregate,
}


def register_function(name: str, fn: Callable):
    """Register a built-in style function: fn(call_expr, scope, ctx, subst) → Column."""
    _FUNCS[name.lower()] = fn


_SQL_TYPE = {"long": "BIGINT", "bigint": "BIGINT", "int": "INT", "integer": "INT", "short": "SMALLINT",
             "smallint": "SMALLINT", "byte": "TINYINT", "tinyint": "TINYINT", "string": "STRING",
             "double": "DOUBLE", "float": "FLOAT", "boolean": "BOOLEAN", "timestamp": "TIMESTAMP", "date": "DATE",
             "binary": "BINARY"}
# functions whose Spark expression prints under another name (FunctionRegistry aliases → the class's prettyName)
_PRETTY_FN = {"ucase": "upper", "lcase": "lower", "substr": "substring", "mean": "avg", "std": "stddev_samp",
              "stddev": "stddev_samp", "variance": "var_samp", "char_length": "length", "character_length": "length",
              "power": "pow", "ceiling": "ceil", "approx_percentile": "percentile_approx", "first_value": "first",
              "last_value": "last", "some": "bool_or", "any": "bool_or", "every": "bool_and", "sign": "signum",
              "random": "rand", "day": "dayofmonth", "now": "current_timestamp"}
_RANKING_FNS = {"row_number", "rank", "dense_rank", "percent_rank", "cume_dist", "ntile"}


def _type_sql(t) -> str:
    if is_decimal(t):
        return f"DECIMAL({t.precision},{t.scale})"
    return _SQL_TYPE.get(str(t).lower(), str(t).upper())


def _frame_bound_sql(b) -> str:
    kind, k = b
    return {"unbounded_preceding": "UNBOUNDED PRECEDING", "unbounded_following": "UNBOUNDED FOLLOWING",
            "current": "CURRENT ROW"}.get(kind) or f"{k} {'PRECEDING' if kind == 'preceding' else 'FOLLOWING'}"


def _window_sql(w: A.WindowCall) -> str:
    """Spark's WindowSpecDefinition.sql after ResolveWindowFrame: PARTITION BY, ORDER BY with explicit direction and
    null order, and the resolved frame (ranking / offset functions have their own ROWS frame)."""
    parts = []
    if w.partition:
        parts.append("PARTITION BY " + ", ".join(output_name(p) for p in w.partition))
    if w.order:
        items = []
        for o in w.order:
            nf = o.nulls_first if o.nulls_first is not None else o.ascending
            items.append(f"{output_name(o.expr)} {'ASC' if o.ascending else 'DESC'} "
                         f"NULLS {'FIRST' if nf else 'LAST'}")
        parts.append("ORDER BY " + ", ".join(items))
    name = w.func.name
    if name in _RANKING_FNS:
        parts.append("ROWS BETWEEN UNBOUNDED PRECEDING AND CURRENT ROW")
    elif name in ("lag", "lead"):
        # OffsetWindowFunction.frame: lag's boundary is UnaryMinus(offset) folded to a literal, and
        # SpecifiedWindowFrame.boundarySql prints any non-UnaryMinus boundary as "<value> FOLLOWING"
        a = w.func.args[1] if len(w.func.args) > 1 else None
        k = 1 if a is None else (int(a.value) if isinstance(a, A.Literal) and isinstance(a.value, int) else None)
        if k is None:
            k_txt = output_name(a) if a is not None else "1"
            bound = f"{k_txt} PRECEDING" if name == "lag" else f"{k_txt} FOLLOWING"
        else:
            bound = f"{-k if name == 'lag' else k} FOLLOWING"
        parts.append(f"ROWS BETWEEN {bound} AND {bound}")
    elif w.frame is not None:
        kind, lo, hi = w.frame
        parts.append(f"{kind.upper()} BETWEEN {_frame_bound_sql(lo)} AND {_frame_bound_sql(hi)}")
    elif w.order:
        parts.append("RANGE BETWEEN UNBOUNDED PRECEDING AND CURRENT ROW")
    else:
        parts.append("ROWS BETWEEN UNBOUNDED PRECEDING AND UNBOUNDED FOLLOWING")
    return "(" + " ".join(parts) + ")"


def output_name(e: A.Expr) -> str:
    """Spark 2.4's auto-generated name of an un-aliased select expression: ``toPrettySQL`` — the expression's
    ``sql`` with literals and attributes printed bare (``usePrettyExpression``).  LIKE / RLIKE print infix, BETWEEN
    is the conjunction the parser builds, CASE / IS NULL / NOT / unary minus use their ``sql`` forms, window calls
    carry their resolved frame, aliased functions their canonical names."""
    if isinstance(e, A.Ident):
        return e.parts[-1]
    if isinstance(e, A.Literal):
        if e.value is None:
            return "NULL"
        if isinstance(e.value, bool):
            return "true" if e.value else "false"
        if e.type == "date":
            return f"DATE '{e.value}'"
        if e.type == "timestamp":
            return f"TIMESTAMP('{e.value}')"
        if isinstance(e.value, float):
            return F.java_double_str(e.value)
        return str(e.value)
    if isinstance(e, A.WindowCall):
        f = e.func
        if f.name in ("lag", "lead") and 1 <= len(f.args) < 3:
            # Spark prints the defaulted arguments: lag(x) → lag(x, 1, NULL)
            f = A.Call(f.name, list(f.args) + [A.Literal(1, "int"), A.Literal(None, "null")][len(f.args) - 1:],
                       f.distinct, f.star)
        return f"{output_name(f)} OVER {_window_sql(e)}"
    if isinstance(e, A.Call):
        name = _PRETTY_FN.get(e.name, e.name)
        if e.star:
            return f"{name}(1)" if e.name == "count" else f"{name}(*)"
        inner = ", ".join(output_name(a) for a in e.args)
        return f"{name}({'DISTINCT ' if e.distinct else ''}{inner})"
    if isinstance(e, A.Cast):
        if e.typed_literal:            # Literal.sql of a timestamp / date value
            v = output_name(e.operand)
            return f"TIMESTAMP('{v}')" if str(e.to).lower() == "timestamp" else f"DATE '{v}'"
        return f"CAST({output_name(e.operand)} AS {_type_sql(e.to)})"
    if isinstance(e, A.BinOp):
        op = e.op.upper() if e.op in ("and", "or", "div") else e.op
        op = "=" if op == "==" else op
        if e.op in ("!=", "<>"):
            return f"(NOT ({output_name(e.left)} = {output_name(e.right)}))"
        return f"({output_name(e.left)} {op} {output_name(e.right)})"
    if isinstance(e, A.UnaryOp):
        if e.op == "not":
            return f"(NOT {output_name(e.operand)})"
        if e.op == "~":
            return f"~{output_name(e.operand)}"
        return f"({e.op} {output_name(e.operand)})"
    if isinstance(e, A.IsNull):
        return f"({output_name(e.operand)} IS {'NOT ' if e.negated else ''}NULL)"
    if isinstance(e, A.Like):
        r = f"{output_name(e.operand)} {'RLIKE' if e.regex else 'LIKE'} {output_name(e.pattern)}"
        return f"(NOT {r})" if e.negated else r
    if isinstance(e, A.Between):
        v = output_name(e.operand)
        r = f"(({v} >= {output_name(e.low)}) AND ({v} <= {output_name(e.high)}))"
        return f"(NOT {r})" if e.negated else r
    if isinstance(e, A.InList):
        r = f"({output_name(e.operand)} IN ({', '.join(output_name(x) for x in e.items)}))"
        return f"(NOT {r})" if e.negated else r
    if isinstance(e, A.Case):
        whens = e.whens
        if e.operand is not None:
            op = output_name(e.operand)
            cases = "".join(f" WHEN ({op} = {output_name(c)}) THEN {output_name(v)}" for c, v in whens)
        else:
            cases = "".join(f" WHEN {output_name(c)} THEN {output_name(v)}" for c, v in whens)
        els = f" ELSE {output_name(e.default)}" if e.default is not None else ""
        return f"CASE{cases}{els} END"
    if isinstance(e, A.Subscript):
        return output_name(e.index) if e.dot else f"{output_name(e.base)}[{output_name(e.index)}]"
    if isinstance(e, A.SubqueryExpr):
        return "scalarsubquery()" if e.kind == "scalar" else e.kind
    return type(e).__name__.lower()


from . import sqlfuncs as _sqlfuncs  # noqa: E402,F401  (registers the extended built-ins)


def _h2d(data, dtype, device):
    from ..ops.native import h2d
    return h2d(data, dtype, device)
