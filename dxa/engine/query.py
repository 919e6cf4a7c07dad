"""Columnar SELECT execution: FROM/JOIN → WHERE → GROUP BY/aggregates → HAVING → SELECT → DISTINCT →
set operations → ORDER BY → LIMIT.

This is what ``spark.sql(statement)`` did for each transform statement in the reference
(DataProcessing/datax-host/src/main/scala/datax/processor/CommonProcessorFactory.scala:249-294); every step runs
over device columns with the dxa kernels (hash group-by / hash join / string ops).
"""
from __future__ import annotations

import functools

from typing import Dict, List, Optional, Tuple

import torch

from ..ops import groupby as G
from ..ops import join as J
from .. import parallel as P
from ..ops.hashing import hash_columns
from ..sql import ast as A
from ..sql.parser import parse_query
from ..telemetry.tracing import host_section
from .column import (ArrayColumn, Column, ConstColumn, DeferredTable, LazyColumns, PrimColumn, StrColumn,
                     StructColumn, Table, concat_columns, concat_tables, materialize, take_columns)
from .expr import (AGG_FUNCS, DeferredColumns, EvalContext, EvalError, HiddenQual, Scope, TakenColumns, cast_column,
                   evaluate, output_name, predicate_mask)
from . import windowfn as W
from .types import common_type, is_nested


class QueryError(Exception):
    pass


class Catalog:
    """Case-insensitive registry of named tables/views visible to SQL."""

    def __init__(self):
        self._t: Dict[str, Table] = {}
        self._built: Dict[Tuple, J.BuiltSide] = {}

    def register(self, name: str, table: Table):
        self._t[name.lower()] = table

    def drop(self, name: str):
        self._t.pop(name.lower(), None)

    def get(self, name: str) -> Optional[Table]:
        return self._t.get(name.lower())

    def names(self):
        return list(self._t)

    def child(self) -> "Catalog":
        """A scope for WITH: sees every table here; its own registrations stay local."""
        c = Catalog()
        c._t = dict(self._t)
        c._built = self._built
        return c

    def __contains__(self, name):
        return name.lower() in self._t

    # stream–static join support: hash tables over resident reference tables are built once
    def cached_build(self, key, builder):
        """Memoise per-table derived structures (join build sides of static tables).  Values hold a reference to
        their table so the ``id()`` in the key cannot be reused while cached."""
        b = self._built.get(key)
        if b is None:
            b = self._built[key] = builder()
        return b


@functools.lru_cache(maxsize=256)
def _parse_cached(sql: str):
    return parse_query(sql)          # ASTs are not mutated by execution (Processor reuses its parsed transform too)


def run_sql(sql: str, catalog: Catalog, ctx: EvalContext) -> Table:
    """Parse (cached per SQL text: the projection step re-runs the same statement every batch) and execute."""
    return execute(_parse_cached(sql), catalog, ctx)


def _gathered(t: Table) -> Table:
    g = P.allgather_table(t)
    g.dist = P.REPLICATED
    return g


def execute(q: A.Query, catalog: Catalog, ctx: EvalContext) -> Table:
    if q.ctes:
        # WITH: each named query sees the catalog plus the CTEs before it
        catalog = catalog.child()
        for name, cq in q.ctes:
            catalog.register(name, execute(cq, catalog, ctx))
    prev, ctx.catalog = ctx.catalog, catalog
    try:
        return _execute(q, catalog, ctx)
    finally:
        ctx.catalog = prev


def _execute(q: A.Query, catalog: Catalog, ctx: EvalContext) -> Table:
    out, src_scope = _exec_body(q.body, catalog, ctx, want_scope=bool(q.order_by or q.sort_by))
    if q.distribute_by or q.sort_by:
        out = _distribute_sort(q, out, src_scope, ctx)
        src_scope = None
    if (q.order_by or q.limit is not None) and P.active() and P.dist_of(out) != P.REPLICATED:
        # a total order / global LIMIT needs every row: gather (outputs of this shape are small in DataX flows)
        out = _gathered(out)
        src_scope = None
    if q.order_by:
        aliases = {}
        if isinstance(q.body, A.Select):
            # ORDER BY may repeat a select expression (e.g. ``R.owner`` after GROUP BY R.owner): map it to its column
            for it in q.body.items:
                if not isinstance(it.expr, A.Star):
                    aliases.setdefault(it.expr.key(), it.alias or output_name(it.expr))
        out = _order_by(out, q.order_by, ctx, src_scope, aliases)
    if q.limit is not None:
        out = out.slice(0, q.limit)
    return out


def _distribute_sort(q: A.Query, out: Table, src_scope, ctx) -> Table:
    """``DISTRIBUTE BY`` / ``SORT BY`` / ``CLUSTER BY`` (Spark's RepartitionByExpression + a per-partition sort):
    at N ranks the rows move to the owner of their key hash (one all-to-all) and each rank sorts its own share; on
    one rank the only partition is the whole result, so SORT BY orders it all and DISTRIBUTE BY moves nothing."""
    aliases = {}
    if isinstance(q.body, A.Select):
        for it in q.body.items:
            if not isinstance(it.expr, A.Star):
                aliases.setdefault(it.expr.key(), it.alias or output_name(it.expr))
    if q.distribute_by and P.active() and P.dist_of(out) != P.REPLICATED and out.length >= 0:
        sc = Scope.of_table(out)
        keys = []
        for e in q.distribute_by:
            try:
                keys.append(materialize(evaluate(e, sc, ctx)))
            except EvalError:
                named = aliases.get(e.key())
                if named is None or out.column(named) is None:
                    raise
                keys.append(materialize(out.column(named)))
        keys = [k if not isinstance(k, (StructColumn, ArrayColumn)) else _nested_key(k) for k in keys]
        dest = P.owner_of(hash_columns(keys)) if out.length else torch.empty(0, dtype=torch.int64, device=out.device)
        out = P.shuffle_table(out, dest)
        out.dist = P.HASHED
        src_scope = None
    if q.sort_by:
        dist = P.dist_of(out)
        out = _order_by(out, q.sort_by, ctx, src_scope, aliases)
        out.dist = dist
    return out


# ---------------------------------------------------------------------------------------------------------------

def _exec_body(body, catalog, ctx, want_scope=False):
    if isinstance(body, A.Select):
        return _exec_select(body, catalog, ctx, want_scope)
    if isinstance(body, A.SetOp):
        if body.op == "wrap":
            return execute(body.left, catalog, ctx), None
        left, _ = _exec_body(body.left, catalog, ctx)
        right, _ = _exec_body(body.right, catalog, ctx)
        return _set_op(body, left, right), None
    if isinstance(body, A.Query):
        return execute(body, catalog, ctx), None
    raise QueryError(f"unsupported query body {type(body).__name__}")


def _align(left: Table, right: Table) -> Tuple[Table, Table]:
    if len(left.names) != len(right.names):
        raise QueryError(f"set operation with {len(left.names)} vs {len(right.names)} columns")
    lcols, rcols = [], []
    for a, b in zip(left.columns, right.columns):
        if a.dtype != b.dtype and not is_nested(a.dtype) and not is_nested(b.dtype):
            t = common_type(a.dtype, b.dtype)
            if t == "null":
                t = "string"
            a = cast_column(a, t) if a.dtype != t else a
            b = cast_column(b, t) if b.dtype != t else b
        if isinstance(a, ConstColumn) and a.value is None and not isinstance(b, ConstColumn):
            a = ConstColumn(None, b.dtype, a.length, a.device)
        if isinstance(b, ConstColumn) and b.value is None and not isinstance(a, ConstColumn):
            b = ConstColumn(None, a.dtype, b.length, b.device)
        lcols.append(a)
        rcols.append(b)
    return (Table(left.names, lcols, left.length, left.device), Table(left.names, rcols, right.length, right.device))


def _set_op(op: A.SetOp, left: Table, right: Table) -> Table:
    ld, rd = P.dist_of(left), P.dist_of(right)
    left, right = _align(left, right)
    if P.active() and (ld != P.REPLICATED) != (rd != P.REPLICATED):
        # mixing a partitioned and a replicated input: keep the replicated rows once (on rank 0)
        if ld == P.REPLICATED and P.rank() != 0:
            left = left.slice(0, 0)
        if rd == P.REPLICATED and P.rank() != 0:
            right = right.slice(0, 0)
    if P.active() and op.op != "union" and (ld != P.REPLICATED or rd != P.REPLICATED):
        left = _gathered(left) if ld != P.REPLICATED else left
        right = _gathered(right) if rd != P.REPLICATED else right
        ld = rd = P.REPLICATED
    if op.op == "union":
        with host_section("setop:concat"):
            out = concat_tables([left, right])
        out.dist = P.REPLICATED if (ld == P.REPLICATED and rd == P.REPLICATED) else P.PARTITIONED
        return out if op.all else distinct(out)
    # INTERSECT / EXCEPT (distinct semantics)
    l, r = distinct(left), distinct(right)
    if l.length == 0:
        return l
    if r.length == 0:
        return l if op.op == "except" else l.slice(0, 0)
    kind = "semi" if op.op == "intersect" else "anti"
    li, _ = J.hash_join(list(l.columns), list(r.columns), kind)
    return l.take(li)


def distinct(t: Table) -> Table:
    if P.active() and P.dist_of(t) != P.REPLICATED and t.columns:
        keys = [c if not isinstance(c, (StructColumn, ArrayColumn)) else _nested_key(c) for c in t.columns]
        dest = P.owner_of(hash_columns(keys)) if t.length else torch.empty(0, dtype=torch.int64, device=t.device)
        t = P.shuffle_table(t, dest)
        out = _local_distinct(t)
        out.dist = P.HASHED
        return out
    return _local_distinct(t)


def _local_distinct(t: Table) -> Table:
    if t.length == 0 or not t.columns:
        return t
    if all(isinstance(c, ConstColumn) for c in t.columns):
        return t.slice(0, 1)                  # every row is the same row (alert views: SELECT DISTINCT <constants>)
    keys = [c for c in t.columns]
    hashable = [c for c in keys if not isinstance(c, (StructColumn, ArrayColumn))]
    if len(hashable) != len(keys):
        # nested columns: compare their JSON text
        from .serialize import column_json_values
        from .column import strings_from_pylist
        hashable = [c if not isinstance(c, (StructColumn, ArrayColumn)) else
                    strings_from_pylist(column_json_values(c), t.device) for c in keys]
    g = G.group_rows(hashable)
    return t.take(g.rep)


# ---------------------------------------------------------------------------------------------------------------
# FROM
# ---------------------------------------------------------------------------------------------------------------

def _relation(src, catalog: Catalog, ctx: EvalContext) -> Scope:
    if src is None:
        sc = Scope([], [], [], 1, ctx.device)
        sc.dist = P.REPLICATED
        return sc
    if isinstance(src, A.TableRef):
        name = src.name
        if src.timewindow:
            from ..sql.parser import parse_duration_micros
            name = f"{src.name}_{src.timewindow.replace(' ', '')}"
        t = catalog.get(name)
        if t is None:
            raise QueryError(f"table or view not found: {name}")
        if src.sample:
            t = _sample(t, src.sample)
        sc = Scope.of_table(t, src.alias or src.name.split(".")[-1])
        sc.dist = P.dist_of(t)
        return sc
    if isinstance(src, A.SubqueryRef):
        t = execute(src.query, catalog, ctx)
        if src.sample:
            t = _sample(t, src.sample)
        if src.columns:
            if len(src.columns) != len(t.columns):
                raise QueryError(f"{src.alias}({', '.join(src.columns)}) names {len(src.columns)} columns; "
                                 f"the relation has {len(t.columns)}")
            t = Table(list(src.columns), t.columns, t.length, t.device)
        sc = Scope.of_table(t, src.alias)
        sc.dist = P.dist_of(t)
        return sc
    if isinstance(src, A.Pivot):
        return _pivot(src, catalog, ctx)
    if isinstance(src, A.Join):
        return _join(src, catalog, ctx)
    if isinstance(src, A.LateralView):
        from . import generators as GEN
        if not GEN.is_generator(src.generator):
            raise QueryError(f"LATERAL VIEW needs a generator function, got {src.generator.name}()")
        base = _relation(src.source, catalog, ctx)
        rows, names, cols = GEN.generate(src.generator, base, ctx, src.outer)
        if src.columns:
            if len(src.columns) != len(names):
                raise QueryError(f"LATERAL VIEW {src.generator.name}() produces {len(names)} column(s), "
                                 f"{len(src.columns)} alias(es) given")
            names = list(src.columns)
        out = Scope(base.names + names, _Appended(TakenColumns(base.cols, rows), cols),
                    base.quals + [src.alias] * len(names), int(rows.shape[0]), base.device)
        out.dist = getattr(base, "dist", P.REPLICATED)
        return out
    raise QueryError(f"unsupported FROM item {type(src).__name__}")


_SAMPLE_SEED = 0x5DEECE66D


def _sample(t: Table, spec) -> Table:
    """``TABLESAMPLE``: ``("rows", n)`` keeps the first n rows (Spark plans it as a LIMIT — global, so a partitioned
    input is gathered first); ``("fraction", f)`` keeps each row with probability f, decided by a hash of the row's
    position and a fixed seed, so the same input gives the same sample on every run (Spark's Bernoulli sampler
    draws a fresh seed per query; here repeatability wins — rank r hashes its own positions salted with r)."""
    kind, v = spec
    dist = P.dist_of(t)
    if kind == "rows":
        if P.active() and dist != P.REPLICATED:
            t = _gathered(t)
            dist = P.REPLICATED
        out = t.slice(0, min(int(v), t.length))
        out.dist = dist
        return out
    if v >= 1.0 or t.length == 0:
        return t
    pos = torch.arange(t.length, dtype=torch.int64, device=t.device)
    salt = (_SAMPLE_SEED + 0x9E3779B97F4A7C15 * (P.rank() + 1)) & 0x7FFFFFFFFFFFFFFF
    h = pos * -7046029254386353131 + salt
    h = h ^ ((h >> 31) & 0x1FFFFFFFF)
    h = h * -4658895280553007687
    h = h ^ ((h >> 29) & 0x7FFFFFFFF)
    u = (h & ((1 << 53) - 1)).to(torch.float64) / float(1 << 53)
    out = t.take(torch.nonzero(u < v).flatten())
    out.dist = dist
    return out


def _pivot(pv: A.Pivot, catalog, ctx) -> Scope:
    """``PIVOT (agg [AS a], … FOR cols IN (values))`` as Spark 2.4's ResolvePivot: GROUP BY every source column
    that neither an aggregate nor a pivot column reads; per (value, aggregate) one column holding the aggregate
    over the rows whose pivot columns equal the value (``agg(IF(cols = value, arg, NULL))`` — COUNT(*) counts the
    matching rows); columns are named by the value (its alias, else its string form) when there is one aggregate,
    else ``<value>_<aggregate alias or SQL text>``."""
    base = _relation(pv.source, catalog, ctx)
    simple = isinstance(pv.source, (A.TableRef, A.SubqueryRef))
    qual = (pv.source.alias or (pv.source.name.split(".")[-1] if isinstance(pv.source, A.TableRef) else None)) \
        if simple else None

    def unq(e):
        # a join's columns are flattened below: references keep their column name only
        return A.replace(e, lambda n: A.Ident((n.parts[-1],)) if isinstance(n, A.Ident) and not simple else None)
    aggs = [(unq(a), al) for a, al in pv.aggs]
    cols = [unq(c) for c in pv.columns]
    used = set()
    for e in [a for a, _ in aggs] + cols:
        for node in A.walk(e):
            if isinstance(node, A.Ident):
                used.add(node.parts[-1].lower() if (len(node.parts) > 1 and qual and
                                                    node.parts[0].lower() == qual.lower()) else node.parts[0].lower())
    for a, _ in aggs:
        if not _contains_agg(a, ctx):
            raise QueryError(f"PIVOT expects aggregate expressions, got {output_name(a)}")
    visible = [i for i, q in enumerate(base.quals) if not isinstance(q, HiddenQual)]
    group = [base.names[i] for i in visible if base.names[i].lower() not in used]
    tmp = f"__dxa_pivot_{id(pv)}"
    t = Table([base.names[i] for i in visible], [base.cols[i] for i in visible], base.length, base.device)
    t.dist = getattr(base, "dist", P.REPLICATED)
    cat = catalog.child()
    cat.register(tmp, t)

    def value_name(vs, alias):
        if alias:
            return alias
        strs = []
        for v in vs:
            if not isinstance(v, A.Literal):
                raise QueryError("PIVOT values must be literals")
            strs.append("null" if v.value is None else
                        ("true" if v.value is True else "false" if v.value is False else str(v.value)))
        return strs[0] if len(strs) == 1 else "[" + ",".join(strs) + "]"

    def cond(vs):
        c = None
        for col, v in zip(cols, vs):
            term = A.IsNull(col) if isinstance(v, A.Literal) and v.value is None else A.BinOp("=", col, v)
            c = term if c is None else A.BinOp("and", c, term)
        return c

    def masked(agg, cnd):
        def sub(node):
            if isinstance(node, A.Call) and (node.name in AGG_FUNCS or node.name in ctx.udafs):
                if node.star:
                    return A.Call(node.name, [A.Call("if", [cnd, A.Literal(1, "int"), A.Literal(None, "null")])],
                                  node.distinct)
                return A.Call(node.name, [A.Call("if", [cnd, x, A.Literal(None, "null")]) for x in node.args[:1]]
                              + list(node.args[1:]), node.distinct)
            return None
        return A.replace(agg, sub)
    def guarded(agg, cnd):
        # Spark 2.4 pivots numeric / boolean aggregates in two phases (GROUP BY groups + pivot column, then
        # PivotFirst): a group without rows for a value gets NULL there — also for COUNT, which the one-phase
        # rewrite alone would give as 0.  Collections keep the one-phase result (an empty array).
        m = masked(agg, cnd)
        if any(isinstance(n, A.Call) and n.name in ("collect_list", "collect_set") for n in A.walk(agg)):
            return m
        hits = A.Call("count", [A.Call("if", [cnd, A.Literal(1, "int"), A.Literal(None, "null")])])
        return A.Call("if", [A.BinOp(">", hits, A.Literal(0, "int")), m, A.Literal(None, "null")])
    items = [A.SelectItem(A.Ident((g,)), g) for g in group]
    single = len(aggs) == 1
    for vs, valias in pv.values:
        vname = value_name(vs, valias)
        c = cond(vs)
        for a, aalias in aggs:
            name = vname if single else f"{vname}_{aalias or output_name(a)}"
            items.append(A.SelectItem(guarded(a, c), name))
    sel = A.Select(items=items, from_=A.TableRef(tmp, qual), group_by=[A.Ident((g,)) for g in group])
    out, _ = _exec_select(sel, cat, ctx)
    sc = Scope.of_table(out, pv.alias)
    sc.dist = P.dist_of(out)
    return sc


class _Appended(LazyColumns):
    """``lazy + tail`` without resolving the lazy part."""

    def __init__(self, lazy, tail):
        super().__init__([None] * len(lazy) + list(tail))
        self._lazy = lazy

    def _make(self, i):
        return self._lazy[i]


def _split_and(e: Optional[A.Expr]) -> List[A.Expr]:
    if e is None:
        return []
    if isinstance(e, A.BinOp) and e.op == "and":
        return _split_and(e.left) + _split_and(e.right)
    return [e]


def _refs_resolvable(e: A.Expr, scope: Scope) -> bool:
    for node in A.walk(e):
        if isinstance(node, A.Ident) and scope.try_resolve(node.parts) is None:
            return False
    return True


def _static_table(src, catalog):
    """(name, table) when ``src`` names a resident reference table (``Table.static``)."""
    if isinstance(src, A.TableRef) and not src.timewindow:
        t = catalog.get(src.name)
        if t is not None and getattr(t, "static", False):
            return src.name, t
    return None


def _rel_names(rel) -> set:
    """Names a hint can use for a relation: its alias, or its table name."""
    if isinstance(rel, A.TableRef):
        return {(rel.alias or rel.name.split(".")[-1]).lower(), rel.name.lower()}
    if isinstance(rel, (A.SubqueryRef, A.Pivot)) and rel.alias:
        return {rel.alias.lower()}
    return set()


def _join(j: A.Join, catalog, ctx) -> Scope:
    out = _join_rows(j, catalog, ctx)
    using = getattr(out, "_using", None)
    if not using:
        return out
    return _merge_using(out, using, j.kind, ctx)


def _merge_using(out: Scope, using, kind: str, ctx) -> Scope:
    """A USING / NATURAL join's output: the key columns once, first (left's value; right's for RIGHT JOIN;
    ``coalesce(left, right)`` for FULL), then the remaining left and right columns (Spark's
    ``Join(..., UsingJoin)`` projection).  The per-side copies stay reachable qualified (``a.k``)."""
    keys = using
    names, cols, quals = [], [], []
    for nm, li, ri in keys:
        lc, rc = out.cols[li], out.cols[ri]
        if kind == "right":
            c = rc
        elif kind == "full":
            tmp = Scope(["__l", "__r"], [lc, rc], [None, None], out.length, out.device)
            c = evaluate(A.Call("coalesce", [A.Ident(("__l",)), A.Ident(("__r",))]), tmp, ctx)
        else:
            c = lc
        names.append(nm)
        cols.append(c)
        quals.append(None)
    key_idx = {i for _n, li, ri in keys for i in (li, ri)}
    merged = Scope(names + list(out.names), _Prefixed(cols, out.cols),
                   quals + [HiddenQual(q or "") if i in key_idx else q for i, q in enumerate(out.quals)],
                   out.length, out.device)
    merged.dist = getattr(out, "dist", P.REPLICATED)
    return merged


class _Prefixed(LazyColumns):
    """``head + tail`` where ``tail`` (a join's lazily gathered columns) stays unresolved until read."""

    def __init__(self, head, tail):
        super().__init__(list(head) + [None] * len(tail))
        self._n = len(head)
        self._tail = tail

    def _make(self, i):
        return self._tail[i - self._n]


class _ColRef(A.Expr):
    """A join key given by column position in its side's scope (USING / NATURAL keys)."""

    def __init__(self, idx: int):
        self.idx = idx

    def key(self):
        return ("colref", self.idx)

    def children(self):
        return []


def _visible_index(scope: Scope, name: str) -> Optional[int]:
    low = name.lower()
    hits = [i for i, (n, q) in enumerate(zip(scope.names, scope.quals))
            if n.lower() == low and not isinstance(q, HiddenQual)]
    if len(hits) > 1:
        raise QueryError(f"USING column '{name}' is ambiguous on one side of the join")
    return hits[0] if hits else None


def _key_col(e, scope: Scope, ctx) -> Column:
    if isinstance(e, _ColRef):
        return materialize(scope.cols[e.idx])
    return materialize(evaluate(e, scope, ctx))


def _join_rows(j: A.Join, catalog, ctx) -> Scope:
    left = _relation(j.left, catalog, ctx)
    right = _relation(j.right, catalog, ctx)
    n_l, n_r = left.length, right.length
    dev = left.device
    lkeys, rkeys, residual = [], [], []
    using = list(j.using or [])
    if j.natural:
        lvis = [n for n, q in zip(left.names, left.quals) if not isinstance(q, HiddenQual)]
        rvis = {n.lower() for n, q in zip(right.names, right.quals) if not isinstance(q, HiddenQual)}
        seen = set()
        for n in lvis:
            if n.lower() in rvis and n.lower() not in seen:
                seen.add(n.lower())
                using.append(n)
        if not using:
            j = A.Join(j.left, j.right, "cross" if j.kind == "inner" else j.kind, None, None,
                       broadcast=j.broadcast)
    using_idx = []
    for nm in using:
        li = _visible_index(left, nm)
        ri = _visible_index(right, nm)
        if li is None or ri is None:
            raise QueryError(f"USING column '{nm}' cannot be resolved on the "
                             f"{'left' if li is None else 'right'} side of the join")
        using_idx.append((left.names[li], li, len(left.names) + ri))
        lkeys.append(_ColRef(li))
        rkeys.append(_ColRef(ri))
    for c in _split_and(j.on):
        if isinstance(c, A.BinOp) and c.op == "=":
            if _refs_resolvable(c.left, left) and _refs_resolvable(c.right, right) and not \
                    _refs_resolvable(c.left, right):
                lkeys.append(c.left)
                rkeys.append(c.right)
                continue
            if _refs_resolvable(c.left, right) and _refs_resolvable(c.right, left) and not \
                    _refs_resolvable(c.right, right):
                lkeys.append(c.right)
                rkeys.append(c.left)
                continue
        residual.append(c)
    kind = j.kind
    ldist, rdist = getattr(left, "dist", P.REPLICATED), getattr(right, "dist", P.REPLICATED)
    out_dist = P.REPLICATED
    bc = j.broadcast or set()
    if P.active() and ldist != P.REPLICATED and rdist != P.REPLICATED and bc:
        # /*+ BROADCAST(x) */: replicate the named side (all-gather) instead of co-partitioning both by key hash —
        # the build side then need not be shuffled every batch (Spark's broadcast hash join)
        if (_rel_names(j.right) & bc) and kind in ("inner", "left", "semi", "anti", "cross"):
            right = _gather_scope(right)
            rdist = P.REPLICATED
        elif (_rel_names(j.left) & bc) and kind in ("inner", "right", "cross"):
            left = _gather_scope(left)
            ldist = P.REPLICATED
    if P.active() and (ldist != P.REPLICATED or rdist != P.REPLICATED):
        if ldist != P.REPLICATED and rdist != P.REPLICATED and lkeys:
            # co-partition both sides by the join-key hash (Spark's shuffle hash join)
            # (keys in the type both sides compare in, so equal keys hash alike: 3 vs 3.0, decimal(10,2) vs
            # decimal(38,4))
            lk0, rk0 = _coerce_keys([_key_col(e, left, ctx) for e in lkeys], [_key_col(e, right, ctx) for e in rkeys])
            left = _shuffle_scope(left, lk0)
            right = _shuffle_scope(right, rk0, ref=left)
            out_dist = P.HASHED
        elif ldist != P.REPLICATED and kind in ("inner", "left", "semi", "anti", "cross"):
            out_dist = ldist            # partitioned ⨝ replicated: rank-local
        elif rdist != P.REPLICATED and kind in ("inner", "right", "cross"):
            out_dist = rdist
        else:
            left = _gather_scope(left) if ldist != P.REPLICATED else left
            right = _gather_scope(right) if rdist != P.REPLICATED else right
        n_l, n_r = left.length, right.length
    if kind == "cross" or (not lkeys):
        if kind not in ("cross", "inner"):
            # outer / semi / anti join on non-equi terms only (Spark's broadcast nested-loop join): the pairs
            # that satisfy ON, in left-row chunks of at most 2^26 pairs, then the preserved side's unmatched rows
            lis, ris = [], []
            step = max(1, (1 << 26) // max(1, n_r))
            for s0 in range(0, n_l, step):
                s1 = min(n_l, s0 + step)
                cl = torch.arange(s0, s1, device=dev).repeat_interleave(n_r)
                cr = torch.arange(n_r, device=dev).repeat(s1 - s0)
                if residual:
                    cl, cr = _filter_pairs(left, right, cl, cr, residual, ctx)
                lis.append(cl)
                ris.append(cr)
            e = torch.zeros(0, dtype=torch.int64, device=dev)
            li, ri = _complete_join(torch.cat(lis) if lis else e, torch.cat(ris) if ris else e, kind, n_l, n_r, dev)
            residual = []
        else:
            li = torch.arange(n_l, device=dev).repeat_interleave(n_r)
            ri = torch.arange(n_r, device=dev).repeat(n_l)
    else:
        lk = [_key_col(e, left, ctx) for e in lkeys]
        built = None
        static = _static_table(j.right, catalog)
        if static is not None and kind in ("inner", "left", "semi", "anti") and rdist == P.REPLICATED:
            # stream–static join: the reference table's keys are evaluated and coerced, and its hash table built,
            # ONCE — every later batch only evaluates and coerces its own (stream) side
            ck = (static[0], id(static[1]), tuple(e.key() for e in rkeys), tuple(c.dtype for c in lk))

            def build():
                rk0 = [_key_col(e, right, ctx) for e in rkeys]
                types = [_join_key_type(a.dtype, b.dtype) for a, b in zip(lk, rk0)]
                rk1 = [b if b.dtype == t else cast_column(b, t) for b, t in zip(rk0, types)]
                return static[1], types, rk1, J.build_side(rk1)
            _t, types, rk, built = catalog.cached_build(ck, build)
            lk = [a if a.dtype == t else cast_column(a, t) for a, t in zip(lk, types)]
        else:
            rk = [_key_col(e, right, ctx) for e in rkeys]
            lk, rk = _coerce_keys(lk, rk)
        if residual and kind != "inner":
            # non-equi ON terms of an outer / semi / anti join decide which pairs *match*: filter the equi pairs
            # first, then add the unmatched rows of the preserved side(s)
            li, ri = J.hash_join(lk, rk, "inner", built)
            li, ri = _filter_pairs(left, right, li, ri, residual, ctx)
            li, ri = _complete_join(li, ri, kind, n_l, n_r, dev)
            residual = []
        else:
            li, ri = J.hash_join(lk, rk, kind if kind != "cross" else "inner", built)
    if kind in ("semi", "anti"):
        out = Scope(left.names, TakenColumns(left.cols, li), left.quals, int(li.shape[0]), dev)
        out.dist = out_dist
        return out
    # which side can carry -1 (no match) is known from the join kind: no per-column host check.  Columns are
    # gathered on first read (a join feeding a narrow SELECT touches few of them).
    l_miss, r_miss = kind in ("right", "full"), kind in ("left", "full")
    cols = _JoinColumns([(left.cols, i, li, l_miss) for i in range(len(left.cols))] +
                        [(right.cols, i, ri, r_miss) for i in range(len(right.cols))])
    out = Scope(left.names + right.names, cols, left.quals + right.quals, int(li.shape[0]), dev)
    if residual:
        pred = None
        for c in residual:
            m = predicate_mask(evaluate(c, out, ctx))
            pred = m if pred is None else pred & m
        idx = torch.nonzero(pred).flatten()
        out = Scope(out.names, TakenColumns(out.cols, idx), out.quals, int(idx.shape[0]), dev)
    out.dist = out_dist
    out._using = using_idx            # USING / NATURAL keys: (name, left index, right index in the joined scope)
    return out


def _filter_pairs(left: Scope, right: Scope, li, ri, residual, ctx):
    pairs = Scope(left.names + right.names,
                  _JoinColumns([(left.cols, i, li, False) for i in range(len(left.cols))] +
                               [(right.cols, i, ri, False) for i in range(len(right.cols))]),
                  left.quals + right.quals, int(li.shape[0]), left.device)
    keep = None
    for c in residual:
        m = predicate_mask(evaluate(c, pairs, ctx))
        keep = m if keep is None else keep & m
    return li[keep], ri[keep]


def _complete_join(li, ri, kind, n_l, n_r, dev):
    """Matched pairs → the rows of a left / right / full outer, semi or anti join (-1: no partner)."""
    matched_l = torch.zeros(n_l, dtype=torch.bool, device=dev)
    if li.numel():
        matched_l[li] = True
    if kind in ("semi", "anti"):
        idx = torch.nonzero(matched_l if kind == "semi" else ~matched_l).flatten()
        return idx, torch.full_like(idx, -1)
    parts_l, parts_r = [li], [ri]
    if kind in ("left", "full"):
        miss = torch.nonzero(~matched_l).flatten()
        parts_l.append(miss)
        parts_r.append(torch.full_like(miss, -1))
    if kind in ("right", "full"):
        matched_r = torch.zeros(n_r, dtype=torch.bool, device=dev)
        if ri.numel():
            matched_r[ri] = True
        rmiss = torch.nonzero(~matched_r).flatten()
        parts_l.append(torch.full_like(rmiss, -1))
        parts_r.append(rmiss)
    li, ri = torch.cat(parts_l), torch.cat(parts_r)
    if kind == "right":
        order = torch.argsort(ri * (n_l + 1) + torch.where(li >= 0, li, torch.full_like(li, n_l)), stable=True)
    else:
        order = torch.argsort(torch.where(li >= 0, li, torch.full_like(li, n_l)) * (n_r + 1) +
                              torch.where(ri >= 0, ri, torch.full_like(ri, n_r)), stable=True)
    return li[order], ri[order]


def _shuffle_scope(scope: Scope, keys, ref=None) -> Scope:
    """Repartition a scope's rows by the hash of ``keys`` (RCCL all-to-all)."""
    from .distagg import shuffle_rows_by_keys
    keys, _ = _coerce_keys(keys, keys)
    new_scope, _ = shuffle_rows_by_keys(scope, keys, None)
    new_scope.dist = P.HASHED
    return new_scope


def _gather_scope(scope: Scope) -> Scope:
    t = Table([f"__c{i}" for i in range(len(scope.cols))], scope.cols, scope.length, scope.device)
    g = P.allgather_table(t)
    out = Scope(scope.names, g.columns, scope.quals, g.length, scope.device)
    out.dist = P.REPLICATED
    return out


def _join_key_type(a, b):
    """Type both sides of an equi-join key are compared in.  Spark 2.4's PromoteStrings casts a string compared with
    a numeric / boolean value to the other side's type (so ``3 = '003'`` holds); otherwise the widest common type."""
    from .decimal import is_decimal
    if a != b:
        # string vs decimal: double (findCommonTypeForBinaryComparison, SPARK-22469)
        if a == "string" and (b in ("long", "int", "double", "boolean") or is_decimal(b)):
            return "double" if is_decimal(b) else b
        if b == "string" and (a in ("long", "int", "double", "boolean") or is_decimal(a)):
            return "double" if is_decimal(a) else a
    return common_type(a, b)


def _coerce_keys(lk, rk):
    lo, ro = [], []
    for a, b in zip(lk, rk):
        if a.dtype != b.dtype:
            t = _join_key_type(a.dtype, b.dtype)
            a = cast_column(a, t) if a.dtype != t else a
            b = cast_column(b, t) if b.dtype != t else b
        lo.append(a)
        ro.append(b)
    return lo, ro


def _take_nullable(col: Column, idx: torch.Tensor, may_miss: bool = True) -> Column:
    """Rows ``idx`` of ``col``; -1 entries (no join partner) become nulls.  No host synchronisation."""
    if not may_miss:
        return col.take(idx)
    if col.length == 0:
        return ConstColumn(None, col.dtype, int(idx.shape[0]), col.device)
    miss = idx < 0
    safe = torch.where(miss, torch.zeros_like(idx), idx)
    return col.take(safe).with_valid(~miss)


class _JoinColumns(LazyColumns):
    """A join's output columns, each gathered from its side on first read: entries (side columns, index, row
    index vector, may hold -1)."""

    def __init__(self, entries):
        super().__init__([None] * len(entries))
        self._e = entries

    def _make(self, i):
        src, j, idx, miss = self._e[i]
        return _take_nullable(src[j], idx, miss)

    def prefetch(self, idxs) -> None:
        """The requested columns of each join side in one multi-column gather; -1 (no partner) rows become nulls
        through one shared mask."""
        groups = {}
        for i in self._unresolved(idxs):
            src, j, idx, miss = self._e[i]
            groups.setdefault((id(src), id(idx), miss), (src, idx, miss, []))[3].append(i)
        for src, idx, miss, ii in groups.values():
            cols = [src[self._e[i][1]] for i in ii]
            if len(ii) < 2 or any(c.length == 0 for c in cols):
                continue                              # single columns / empty sides: resolved on access
            if miss:
                gone = idx < 0
                taken = take_columns(cols, torch.where(gone, torch.zeros_like(idx), idx))
                keep = ~gone
                taken = [c.with_valid(keep) for c in taken]
            else:
                taken = take_columns(cols, idx)
            for i, c in zip(ii, taken):
                list.__setitem__(self, i, c)


# ---------------------------------------------------------------------------------------------------------------
# SELECT
# ---------------------------------------------------------------------------------------------------------------

def _contains_agg(e: A.Expr, ctx) -> bool:
    calls = A.summary(e)[0]
    return any(n in AGG_FUNCS or n in ctx.udafs for n in calls)


def _collect_aggs(e: A.Expr, ctx, out: Dict):
    if isinstance(e, A.Call) and (e.name in AGG_FUNCS or e.name in ctx.udafs):
        out.setdefault(e.key(), e)
        return
    for c in e.children():
        _collect_aggs(c, ctx, out)


def _star_columns(st: A.Star, scope: Scope) -> List[Tuple[A.Expr, str]]:
    """(expression, name) of every column a ``*`` / ``q.*`` stands for in ``scope``."""
    out = []
    if not st.qualifier:
        for nm, q in zip(scope.names, scope.quals):
            if isinstance(q, HiddenQual):
                continue              # a USING join's per-side key copy: the merged key is listed instead
            out.append((A.Ident(((q,) if q and _dup(scope, nm) else ()) + (nm,)), nm))
        return out
    q = st.qualifier
    if len(q) == 1 and scope.has_qualifier(q[0]):
        for nm, qq in zip(scope.names, scope.quals):
            if (qq or "").lower() == q[0].lower():
                out.append((A.Ident((qq, nm)), nm))
        return out
    col = scope.resolve(q)
    if isinstance(col, StructColumn):
        return [(A.Ident(q + (nm,)), nm) for nm in col.names]
    raise QueryError(f"cannot expand {'.'.join(q)}.*")


def _expand_call_stars(e: A.Expr, scope: Scope) -> A.Expr:
    """``struct(*)``, ``to_json(struct(t.*))``, ``hash(*)``, ``concat_ws(',', *)``: a star argument of a function
    (not COUNT(*)) stands for every column it names, in order (Spark's ResolveReferences expands
    ``UnresolvedStar`` inside function arguments the same way)."""
    def fn(node):
        if not isinstance(node, A.Call):
            return None
        if not (node.star and node.name != "count") and not any(isinstance(a, A.Star) for a in node.args):
            return None
        args = []
        if node.star and node.name != "count":
            args += [x for x, _ in _star_columns(A.Star(()), scope)]
        for a in node.args:
            if isinstance(a, A.Star):
                args += [x for x, _ in _star_columns(a, scope)]
            else:
                args.append(_expand_call_stars(a, scope))
        return A.Call(node.name, args, distinct=node.distinct)
    return A.replace(e, fn)


def _has_call_star(e: A.Expr) -> bool:
    return A.summary(e)[2]


def _expand_items(sel: A.Select, scope: Scope) -> List[Tuple[A.Expr, str]]:
    items = []
    for it in sel.items:
        e = it.expr
        if not isinstance(e, A.Star) and _has_call_star(e):
            items.append((_expand_call_stars(e, scope), it.alias or output_name(e)))
            continue
        if isinstance(e, A.Star):
            if not e.qualifier:
                for nm, q in zip(scope.names, scope.quals):
                    if isinstance(q, HiddenQual):
                        continue              # a USING join's per-side key copy: the merged key is listed instead
                    items.append((A.Ident(((q,) if q and _dup(scope, nm) else ()) + (nm,)), nm))
                continue
            q = e.qualifier
            if len(q) == 1 and scope.has_qualifier(q[0]):
                for nm, qq in zip(scope.names, scope.quals):
                    if (qq or "").lower() == q[0].lower():
                        items.append((A.Ident((qq, nm)), nm))
                continue
            col = scope.resolve(q)
            if isinstance(col, StructColumn):
                for nm in col.names:
                    items.append((A.Ident(q + (nm,)), nm))
                continue
            raise QueryError(f"cannot expand {'.'.join(q)}.*")
        if isinstance(it.alias, tuple) and not (isinstance(e, A.Call) and e.name in _GENERATOR_NAMES):
            raise QueryError(f"a multi-alias AS ({', '.join(it.alias)}) is only allowed on a generator function")
        items.append((e, it.alias or output_name(e)))
    return items


def _dup(scope: Scope, nm: str) -> bool:
    low = nm.lower()
    return sum(1 for n, q in zip(scope.names, scope.quals) if n.lower() == low and not isinstance(q, HiddenQual)) > 1


NONDETERMINISTIC = {"rand", "random", "randn", "uuid", "now", "current_timestamp", "current_date",
                    "unix_timestamp", "monotonically_increasing_id", "spark_partition_id"}


BLOCK = 16


class _NotPaned(Exception):
    pass


class _EmptyPane:
    def __init__(self, table):
        self.table = table
        self.partials = {}


def _paned_aggregate(sel: A.Select, t, alias: str, ctx) -> Optional[Table]:
    """GROUP BY over a window view answered from per-pane partial aggregates (see ``windows.PanedTable``).
    Returns None when the query does not qualify (non-decomposable aggregates, no aggregation, …)."""
    from . import distagg as D
    from .windows import PanedTable
    if not t.panes:
        return None
    proto = t.panes[0].table
    # a zero-row table of the window's schema (resolves the select list); kept on the store while the schema holds
    sig = (tuple(proto.names), tuple(str(c.dtype) for c in proto.columns))
    cached = getattr(t.store, "_empty_proto", None)
    if cached is None or cached[0] != sig:
        cached = (sig, proto.take(torch.empty(0, dtype=torch.int64, device=proto.device)))
        t.store._empty_proto = cached
    empty = cached[1]
    # the statement's paned plan (select items, aggregates, cacheability, fingerprint) depends only on the
    # statement, the window's schema and the session's functions: derived once, not re-walked every batch
    plans = t.store.__dict__.setdefault("_paned_plans", {})
    pkey = (id(sel), alias, sig, id(ctx.udfs), id(ctx.udafs) if hasattr(ctx, "udafs") else None)
    plan_ent = plans.get(pkey)
    if plan_ent is None or plan_ent[0] is not sel:
        items = _expand_items(sel, Scope.of_table(empty, alias))
        aggs: Dict = {}
        for e, _ in items:
            _collect_aggs(e, ctx, aggs)
        if sel.having is not None:
            _collect_aggs(sel.having, ctx, aggs)
        ok = bool(aggs or sel.group_by) and not any(W.window_calls(e) for e, _ in items) and \
            D.decomposable(aggs, ctx)
        exprs = [e for e, _ in items] + list(sel.group_by) + ([sel.where] if sel.where is not None else []) + (
            [sel.having] if sel.having is not None else [])
        cacheable = True
        for e in exprs:
            for node in A.walk(e):
                if isinstance(node, A.Call) and (node.name in NONDETERMINISTIC or (
                        node.name in ctx.udfs and not getattr(ctx.udfs[node.name], "deterministic", False))):
                    cacheable = False
        fp = repr((alias, [e.key() for e in exprs], sel.where is not None, [nm for _, nm in items]))
        plan_ent = plans[pkey] = (sel, ok, items, aggs, cacheable, fp)
    _, ok, items, aggs, cacheable, fp = plan_ent
    if not ok:
        return None
    if cacheable and sel.group_by:
        # the dense ring (persistent group dictionary + per-pane accumulator rows in HBM, window_dense.py): one
        # combine kernel and one status read per batch instead of concatenating and re-grouping partial tables
        from .window_dense import dense_answer, dense_partials
        if P.active() and t.dist != P.REPLICATED:
            with host_section("paned:dense"):
                got = dense_partials(t, sel, alias, ctx, items, aggs, fp, empty)
            if got is not None:
                partial, plan, key_names, gexprs = got
                got, tag = D.exchange_partials(partial, key_names, True)
                with host_section("paned:merge"):
                    out_keys, finals, ng = D.merge_partials(got, plan, key_names, aggs, True)
                return _paned_output(sel, items, out_keys, finals, ng, gexprs, proto.device, tag, ctx)
        else:
            defer = ctx.defer_dense
            with host_section("paned:dense"):
                got = dense_answer(t, sel, alias, ctx, items, aggs, fp, defer=defer)
            if callable(got):
                def finish():
                    res = got()
                    if res is None:
                        return None                 # collision / overflow: the caller re-runs the paned path
                    out_keys, finals, ng, gexprs = res
                    return _paned_output(sel, items, out_keys, finals, ng, gexprs, proto.device, P.REPLICATED, ctx)
                return _PendingDense(finish)
            if got is not None:
                out_keys, finals, ng, gexprs = got
                return _paned_output(sel, items, out_keys, finals, ng, gexprs, proto.device, P.REPLICATED, ctx)
    state = {}

    def pane_partial(pane, full):
        cached = pane.partials.get(fp) if (full and cacheable) else None
        if cached is None:
            src = pane.table if full else t.clipped(pane)
            scope = Scope.of_table(src, alias)
            if sel.where is not None:
                mask = predicate_mask(evaluate(sel.where, scope, ctx))
                idx = torch.nonzero(mask).flatten()
                scope = Scope(scope.names, TakenColumns(scope.cols, idx), scope.quals, int(idx.shape[0]),
                              scope.device)
            gx = [_resolve_group_expr(g, scope, items) for g in sel.group_by]
            keys = [materialize(evaluate(g, scope, ctx)) for g in gx]
            if any(isinstance(k, (StructColumn, ArrayColumn)) for k in keys):
                raise _NotPaned()
            partial, pl, kn = D.local_partials(gx, keys, aggs, scope, ctx)
            cached = (partial, pl, kn, gx)
            if full and cacheable:
                pane.partials[fp] = cached
        state["meta"] = cached[1:]
        return cached[0]

    # complete blocks of BLOCK consecutive in-window panes are pre-combined once and reused until a member is
    # evicted, so a 300-pane window merges ~20 block partials + the loose panes at its edges instead of 300 tables.
    # (Measured and dropped, profiles/window_merge/: combining all complete blocks into one table was within noise;
    # additionally keeping the newest block's running combination and the oldest block's suffix combinations cost
    # more — a group-by pass per batch plus bursts — than the concat it saves.)
    store = t.store
    span = BLOCK * max(1, store.interval_us)
    parts = []
    by_block: Dict[int, list] = {}
    sec = host_section("paned:partials")
    sec.__enter__()
    # parts are ordered by event time (a block by its first slot): the merge input does not depend on the order
    # the views list their panes in, and from one batch to the next the list keeps one long common run (the newest
    # pane joins at the end, the oldest leave at the front) for _concat_panes to reuse
    keyed = []
    try:
        use_blocks = cacheable and store.interval_us
        for pane, full in t.pieces():
            if full and use_blocks:
                by_block.setdefault(pane.key // span, []).append(pane)
            else:
                keyed.append((pane.key, pane_partial(pane, full)))
        for bid, panes in by_block.items():
            if len(panes) == BLOCK:
                members = tuple(sorted(p.key for p in panes))
                ent = store.blocks.get((fp, bid))
                if ent is None or ent[0] != members:
                    ps = [pane_partial(p, True) for p in sorted(panes, key=lambda p: p.key)]
                    pl, kn, _ = state["meta"]
                    ent = (members, D.combine_partials(concat_tables(ps), pl, kn, bool(sel.group_by)), state["meta"])
                    store.blocks[(fp, bid)] = ent
                state.setdefault("meta", ent[2])
                keyed.append((bid * span, ent[1]))
            else:
                keyed.extend((p.key, pane_partial(p, True)) for p in panes)
        keyed.sort(key=lambda kv: kv[0])
        parts = [tb for _, tb in keyed]
        if "meta" not in state:
            # nothing of this rank's window is in range: still produce (empty) partials, so every rank runs the
            # same exchange — the choice of plan must not depend on a rank's data
            parts.append(pane_partial(_EmptyPane(empty), False))
    except _NotPaned:
        return None
    finally:
        sec.__exit__(None, None, None)
    plan, key_names, gexprs = state["meta"]
    parts = [p for p in parts if p.length] or parts[:1]
    dev = proto.device
    grouped = bool(sel.group_by)
    with host_section("paned:concat"):
        got = _concat_panes(parts, store, fp)
    tag = P.REPLICATED
    if P.active() and t.dist != P.REPLICATED:
        got, tag = D.exchange_partials(got, key_names, grouped)
    with host_section("paned:merge"):
        out_keys, finals, ng = D.merge_partials(got, plan, key_names, aggs, grouped)
    return _paned_output(sel, items, out_keys, finals, ng, gexprs, dev, tag if grouped else P.REPLICATED, ctx)


def _paned_output(sel, items, out_keys, finals, ng, gexprs, dev, tag, ctx) -> Table:
    """The select list (and HAVING) over a window statement's groups: aggregates and group keys enter as
    substitutions."""
    subst = dict(finals)
    for g, k in zip(gexprs, out_keys):
        subst[g.key()] = k
    escope = Scope([], [], [], ng, dev)
    cols = [evaluate(e, escope, ctx, subst) for e, _ in items]
    out = Table([nm for _, nm in items], cols, ng, dev)
    if sel.having is not None:
        out = out.filter(predicate_mask(evaluate(sel.having, escope, ctx, subst)))
    out.dist = tag
    return out


def _row_view(t: Table, a: int, b: int) -> Optional[Table]:
    """Rows [a, b) of a table of flat columns as views (no copy, no launch); None for other column kinds."""
    cols = []
    for c in t.columns:
        v = None if c.valid is None else c.valid[a:b]
        if type(c) is PrimColumn:
            cols.append(PrimColumn(c.dtype, c.data[a:b], v))
        elif type(c) is StrColumn:
            cols.append(StrColumn(c.arena, c.starts[a:b], c.lens[a:b], v, c.dtype))
        else:
            return None
    return Table(t.names, cols, b - a, t.device)


def _concat_panes(parts: List[Table], store, fp) -> Table:
    """``concat_tables(parts)`` for a window's partial tables, reusing last batch's concatenation: from one batch
    to the next only the edges change (the clipped oldest panes, the newest pane), so the run of parts that ended
    last batch's list and reappears here is taken as ONE row view of last batch's result instead of ~30 tables
    (a block completing or expiring breaks the run: then everything is concatenated afresh).  The cache holds the
    parts themselves, so no id is reused while it is alive."""
    cache = getattr(store, "concat_cache", None)
    if cache is None:
        cache = store.concat_cache = {}
    hit = cache.get(fp)
    pieces = parts
    if hit is not None and len(parts) >= 4:
        cparts, coffs, ctab = hit
        pos = {id(p): k for k, p in enumerate(cparts)}
        a = next((k for k, p in enumerate(parts) if id(p) in pos), None)
        if a is not None:
            j = pos[id(parts[a])]
            m = 0
            while a + m < len(parts) and j + m < len(cparts) and parts[a + m] is cparts[j + m]:
                m += 1
            if j + m == len(cparts) and m >= 3:
                mid = _row_view(ctab, coffs[j], coffs[j + m])
                if mid is not None:
                    pieces = parts[:a] + [mid] + parts[a + m:]
    got = concat_tables(pieces)
    offs = [0]
    for p in parts:
        offs.append(offs[-1] + p.length)
    cache[fp] = (list(parts), offs, got)
    return got


def _lookup(src: A.TableRef, catalog: Catalog):
    name = src.name
    if src.timewindow:
        name = f"{src.name}_{src.timewindow.replace(' ', '')}"
    return catalog.get(name)


def _rewrite_expr(e, fn):
    """Rebuild an expression tree bottom-up through ``fn(node) -> node | None`` (None: keep, descend)."""
    import dataclasses
    r = fn(e)
    if r is not None:
        return r
    if not dataclasses.is_dataclass(e) or not isinstance(e, A.Expr):
        return e
    changes = {}
    for f in dataclasses.fields(e):
        v = getattr(e, f.name)
        if isinstance(v, A.Expr):
            nv = _rewrite_expr(v, fn)
            if nv is not v:
                changes[f.name] = nv
        elif isinstance(v, list) and any(isinstance(x, A.Expr) for x in v):
            nv = [_rewrite_expr(x, fn) if isinstance(x, A.Expr) else x for x in v]
            if any(a is not b for a, b in zip(nv, v)):
                changes[f.name] = nv
    return dataclasses.replace(e, **changes) if changes else e


def _exec_grouping_sets(sel: A.Select, catalog, ctx):
    """GROUP BY ROLLUP / CUBE / GROUPING SETS: one aggregation per set, UNION ALL.  Group expressions outside the
    current set read as NULL in the select list and HAVING (not inside aggregates); ``grouping(c)`` /
    ``grouping_id(…)`` become the set's constant bits (Spark's semantics)."""
    if any(isinstance(it.expr, A.Star) for it in sel.items):
        raise QueryError("SELECT * is not supported with ROLLUP / CUBE / GROUPING SETS")
    all_keys = [g.key() for g in sel.group_by]
    parts = []
    for st in sel.grouping_sets:
        in_set = {g.key() for g in st}
        rolled = {k for k in all_keys if k not in in_set}

        def fn(node, rolled=rolled):
            if isinstance(node, A.Call):
                if node.name in AGG_FUNCS or node.name in ctx.udafs:
                    return node                                   # aggregates see the real values
                if node.name == "grouping":
                    return A.Literal(1 if node.args and node.args[0].key() in rolled else 0, "int")
                if node.name == "grouping_id":
                    cols = [a.key() for a in node.args] or all_keys
                    bits = 0
                    for k in cols:
                        bits = (bits << 1) | (1 if k in rolled else 0)
                    return A.Literal(bits, "long")
            if isinstance(node, A.Expr) and not isinstance(node, A.Literal) and node.key() in rolled:
                return A.Literal(None, "null")
            return None
        items = [A.SelectItem(_rewrite_expr(it.expr, fn), it.alias or output_name(it.expr)) for it in sel.items]
        sub = A.Select(items=items, from_=sel.from_, where=sel.where, group_by=list(st),
                       having=None if sel.having is None else _rewrite_expr(sel.having, fn))
        if not st and not any(_contains_agg(it.expr, ctx) for it in items):
            sub.group_by = []
        out, _ = _exec_select(sub, catalog, ctx)
        parts.append(out)
    out = parts[0]
    for p in parts[1:]:
        out = _set_op(A.SetOp("union", True, None, None), out, p)
    return distinct(out) if sel.distinct else out


class _Prefiltered:
    """A statement's WHERE mask evaluated at the start of the batch, its row count on its way to pinned memory."""
    __slots__ = ("sel", "table", "mask", "counts", "k", "event")

    def __init__(self, sel, table, mask, counts, k, event):
        self.sel, self.table, self.mask, self.counts, self.k, self.event = sel, table, mask, counts, k, event

    def indices(self) -> torch.Tensor:
        self.event.synchronize()          # long complete by the time the statement runs: no queue drain
        n = int(self.mask.shape[0]) - int(self.counts[self.k])       # counts: the mask's false rows
        return torch.nonzero_static(self.mask, size=n).flatten()


def _plain_predicate(e: A.Expr, ctx) -> bool:
    """A WHERE that reads only its row (no sub-query, window or aggregate): evaluable before its statement runs."""
    calls, wins, _star = A.summary(e)
    if wins or any(n in AGG_FUNCS or n in ctx.udafs for n in calls):
        return False
    return not any(isinstance(n, A.SubqueryExpr) for n in A.walk(e))


def prefilter(queries, catalog, ctx, min_group: int = 2) -> None:
    """Note the statements that filter a table already in ``catalog`` (the batch's input views, reference and state
    tables).  When the first of them runs, the WHERE masks of all of them over that same table are evaluated
    together and their row counts come to pinned memory in ONE copy (``_run_prefilters``): the statements after
    it take their rows without draining the stream.  Each predicate is still evaluated exactly once; a statement
    whose predicate fails there keeps the usual path (and reports its error there)."""
    from .windows import PanedTable
    cands: Dict[int, list] = {}
    for q in queries:
        if q is None or q.ctes or not isinstance(q.body, A.Select):
            continue
        sel = q.body
        src = sel.from_
        if sel.where is None or sel.grouping_sets is not None or not isinstance(src, A.TableRef) or src.sample or \
                src.timewindow:
            continue
        t = catalog.get(src.name)
        if t is None or t.device.type != "cuda" or not _plain_predicate(sel.where, ctx):
            continue
        if isinstance(t, PanedTable) and (sel.group_by or any(
                not isinstance(it.expr, A.Star) and _contains_agg(it.expr, ctx) for it in sel.items)):
            continue                       # a windowed aggregate: the paned / dense path applies WHERE per pane
        cands.setdefault(id(t), []).append((sel, t, src.alias or src.name.split(".")[-1]))
    # lazily run, one filter alone gains nothing (``min_group`` 2); run at once ahead of a window's kernels, it does
    ctx.prefilter_cands = {k: v for k, v in cands.items() if len(v) >= min_group}


def filter_readers(queries, ctx) -> Dict[str, list]:
    """Statements (index, SELECT, alias) whose plain WHERE filters a named table, by that name (lower case): the
    candidates ``prefilter_result`` starts as soon as a statement registers the table they read."""
    out: Dict[str, list] = {}
    for k, q in queries:
        if q is None or q.ctes or not isinstance(q.body, A.Select):
            continue
        sel = q.body
        src = sel.from_
        if sel.where is None or sel.grouping_sets is not None or not isinstance(src, A.TableRef) or src.sample or \
                src.timewindow or not _plain_predicate(sel.where, ctx):
            continue
        out.setdefault(src.name.lower(), []).append((k, sel, src.alias or src.name.split(".")[-1]))
    return out


def prefilter_result(table, readers, ctx) -> None:
    """A statement's result just registered: the WHERE masks of the later statements that filter it (``readers``)
    are queued now, their counts on the way to pinned memory — by the time those statements run, the statements in
    between have synchronised the stream, and they take their rows without a wait of their own."""
    if table.device.type != "cuda" or not table.length:
        return
    _run_prefilters([(sel, table, alias) for _, sel, alias in readers if id(sel) not in ctx.prefilter], ctx)


def _run_prefilters(cands, ctx) -> None:
    found = []
    for sel, t, alias in cands:
        try:
            mask = predicate_mask(evaluate(sel.where, Scope.of_table(t, alias), ctx))
        except Exception:  # noqa: BLE001 — the statement's own evaluation reports it
            continue
        found.append((sel, t, mask))
    if not found:
        return
    from ..ops import native as N
    dev = found[0][2].device
    st = N.stream_handle(dev)
    # false rows per mask (null_count_kernel: one small launch each, where a torch bool sum is a 50 us reduction)
    falses = torch.empty(len(found), dtype=torch.int64, device=dev)
    for k, (_, _, m) in enumerate(found):
        m = m.contiguous()
        N.call("dxa_null_counts", N.ptr(N.u8(m)), int(m.shape[0]), 1, falses[k:].data_ptr(), st)
    counts = torch.empty(len(found), dtype=torch.int64, pin_memory=True)
    counts.copy_(falses, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    for k, (sel, t, mask) in enumerate(found):
        ctx.prefilter[id(sel)] = _Prefiltered(sel, t, mask, counts, k, ev)


class _PendingDense:
    """A windowed GROUP BY whose dense-ring kernels are queued; ``finish()`` reads the status → Table or None."""
    __slots__ = ("finish",)

    def __init__(self, finish):
        self.finish = finish


def _deferred_select(sel: A.Select, catalog, ctx, pending: _PendingDense) -> DeferredTable:
    """The statement's result as a ``DeferredTable``, registered on ``ctx.pending`` (the processor completes any left
    at the end of the batch's statements).  When the dictionary reports a collision the statement runs again on
    the paned path — against the catalog as it was here, so statements planned meanwhile cannot change its
    inputs."""
    snap = catalog.child()

    def finish():
        prev_cat, prev_defer = ctx.catalog, ctx.defer_dense
        ctx.catalog, ctx.defer_dense = snap, False
        try:
            out = pending.finish()
            if out is None:
                out, _ = _exec_select(sel, snap, ctx)
        finally:
            ctx.catalog, ctx.defer_dense = prev_cat, prev_defer
        return out
    d = DeferredTable(finish)
    ctx.pending.append(d)
    return d


def _exec_select(sel: A.Select, catalog, ctx, want_scope=False):
    if sel.grouping_sets is not None:
        return _exec_grouping_sets(sel, catalog, ctx), None
    if isinstance(sel.from_, A.TableRef) and not want_scope:
        from .windows import PanedTable
        t = _lookup(sel.from_, catalog)
        if isinstance(t, PanedTable):
            alias = sel.from_.alias or sel.from_.name.split(".")[-1]
            try:
                out = _paned_aggregate(sel, t, alias, ctx)
            except EvalError:
                out = None
            if isinstance(out, _PendingDense):
                out = _deferred_select(sel, catalog, ctx, out)
                if not sel.distinct:
                    return out, None
            if out is not None:
                return (distinct(out) if sel.distinct else out), None
    scope = _relation(sel.from_, catalog, ctx)
    sdist = getattr(scope, "dist", P.REPLICATED)
    if sel.where is not None:
        pf = ctx.prefilter.pop(id(sel), None) if ctx.prefilter else None
        if pf is None and ctx.prefilter_cands and isinstance(sel.from_, A.TableRef):
            src_t = _lookup(sel.from_, catalog)
            cands = ctx.prefilter_cands.get(id(src_t))
            if cands and any(c[0] is sel and c[1] is src_t for c in cands):
                del ctx.prefilter_cands[id(src_t)]
                _run_prefilters(cands, ctx)
                pf = ctx.prefilter.pop(id(sel), None)
        if pf is not None and pf.sel is sel and pf.table is _lookup(sel.from_, catalog) and \
                pf.mask.shape[0] == scope.length:
            idx = pf.indices()
        else:
            scope.prefetch([sel.where])
            mask = predicate_mask(evaluate(sel.where, scope, ctx))
            idx = torch.nonzero(mask).flatten()
        scope = Scope(scope.names, TakenColumns(scope.cols, idx), scope.quals, int(idx.shape[0]), scope.device)
        scope.dist = sdist
    # the columns the statement reads in one gather (a SELECT * stays deferred: its consumer may read few columns)
    scope.prefetch([it.expr for it in sel.items if not isinstance(it.expr, A.Star)] +
                   list(sel.group_by) + [sel.having])
    sel = _window_column_refs(sel, scope)
    sel, scope = _sliding_windows(sel, scope, ctx)
    items = _expand_items(sel, scope)
    gen_at = [k for k, (e, _) in enumerate(items) if isinstance(e, A.Call) and e.name in _GENERATOR_NAMES]
    if gen_at:
        return _exec_generator_select(sel, items, gen_at, scope, ctx), None
    is_agg = bool(sel.group_by) or any(_contains_agg(e, ctx) for e, _ in items) or (
        sel.having is not None and _contains_agg(sel.having, ctx))
    wcalls = [w for e, _ in items for w in W.window_calls(e)]
    if wcalls and P.active() and sdist != P.REPLICATED:
        scope = _window_repartition(scope, wcalls, ctx, is_agg)
        sdist = scope.dist
    if is_agg:
        out = _aggregate(sel, items, scope, ctx)
        src = None
    else:
        subst = _window_columns(wcalls, lambda x: evaluate(x, scope, ctx), scope.length, scope.device, {})
        if not subst and isinstance(scope.cols, LazyColumns):
            # bare column references into a filtered scope stay deferred takes: a consumer reading few of them
            # (an alert view over ``SELECT * … WHERE``) never gathers the rest
            cols = DeferredColumns([_deferred_ref(e, scope) or evaluate(e, scope, ctx) for e, _ in items])
        else:
            cols = [evaluate(e, scope, ctx, subst or None) for e, _ in items]
        out = Table([nm for _, nm in items], cols, scope.length, scope.device)
        out.dist = sdist
        src = scope
    if sel.distinct:
        out = distinct(out)
        src = None
    return out, (src if want_scope else None)


_WINDOW_COL = "__dxa_window"


def _window_column_refs(sel: A.Select, scope: Scope) -> A.Select:
    """Spark's TimeWindowing names the grouped ``window(...)`` struct ``window``: with ``GROUP BY window(ts, …)``
    the SELECT list and HAVING may say ``window`` / ``window.start`` / ``window.end`` (when the input has no column of
    that name)."""
    calls = [g for g in sel.group_by if isinstance(g, A.Call) and g.name == "window"]
    if len(calls) != 1 or scope._find("window"):
        return sel
    call = calls[0]

    def sub(node):
        if isinstance(node, A.Ident) and node.parts[0].lower() == "window":
            e = call
            for part in node.parts[1:]:
                e = A.Subscript(e, A.Literal(part, "string"), dot=True)
            return e
        return None
    import dataclasses
    return dataclasses.replace(
        sel, items=[dataclasses.replace(it, expr=A.replace(it.expr, sub)) for it in sel.items],
        having=None if sel.having is None else A.replace(sel.having, sub))


def _sliding_windows(sel: A.Select, scope: Scope, ctx):
    """Spark's TimeWindowing for sliding ``window(ts, dur, slide)`` (slide < dur): each row is repeated once per
    window holding its timestamp (after WHERE, before grouping), and every occurrence of that window call in the
    SELECT list, GROUP BY and HAVING reads the expanded rows' window struct.  One distinct sliding window per
    SELECT, as in Spark."""
    from . import sqlfuncs as SF
    exprs = [it.expr for it in sel.items] + list(sel.group_by) + ([sel.having] if sel.having is not None else [])
    found = {}
    for e in exprs:
        if "window" not in A.summary(e)[0]:
            continue
        for node in A.walk(e):
            if isinstance(node, A.Call) and node.name == "window" and len(node.args) >= 3:
                size, slide, _ = SF.window_params(node, scope, ctx)
                if slide != size:
                    found.setdefault(node.key(), node)
    if not found:
        return sel, scope
    if len(found) > 1:
        raise QueryError("only one distinct sliding window() is allowed per SELECT")
    key, call = next(iter(found.items()))
    rows, wcol = SF.sliding_windows(call, scope, ctx)
    sdist = getattr(scope, "dist", P.REPLICATED)
    base = Scope(scope.names, TakenColumns(scope.cols, rows), scope.quals, int(rows.shape[0]), scope.device)
    out = base.with_bindings([_WINDOW_COL], [wcol])
    out.dist = sdist
    ref = A.Ident((_WINDOW_COL,))

    def sub(node):
        return ref if isinstance(node, A.Call) and node.name == "window" and node.key() == key else None
    import dataclasses
    sel2 = dataclasses.replace(
        sel, items=[dataclasses.replace(it, expr=A.replace(it.expr, sub),
                                        alias=it.alias or ("window" if sub(it.expr) is not None else None))
                    for it in sel.items],
        group_by=[A.replace(g, sub) for g in sel.group_by],
        having=None if sel.having is None else A.replace(sel.having, sub))
    return sel2, out


_GENERATOR_NAMES = {"explode", "explode_outer", "posexplode", "posexplode_outer", "inline", "inline_outer",
                    "stack", "json_tuple"}


def _exec_generator_select(sel: A.Select, items, gen_at, scope: Scope, ctx) -> Table:
    """``SELECT a, explode(arr) AS e FROM …``: the generator's rows replace the input rows; the other items are
    evaluated over the input rows they came from."""
    from . import generators as GEN
    if len(gen_at) > 1:
        raise QueryError("only one generator is allowed per SELECT clause")
    if sel.group_by or any(_contains_agg(e, ctx) for e, _ in items):
        # Spark's ExtractGenerator over an Aggregate: aggregate first (the generator's arguments become hidden
        # aggregate outputs, e.g. explode(collect_list(v))), then generate over the aggregated rows
        import dataclasses
        k = gen_at[0]
        call, alias = items[k]
        hidden = [f"__dxa_gen{i}" for i in range(len(call.args))]
        others = [(e, nm) for j, (e, nm) in enumerate(items) if j != k]
        agg = _aggregate(sel, others + list(zip(call.args, hidden)), scope, ctx)
        ascope = Scope.of_table(agg)
        ascope.dist = getattr(agg, "dist", P.REPLICATED)
        gcall = A.Call(call.name, [A.Ident((h,)) for h in hidden], call.distinct, call.star)
        items2 = [(A.Ident((nm,)), nm) for e, nm in others]
        items2.insert(k, (gcall, alias))
        plain = dataclasses.replace(sel, group_by=[], having=None, grouping_sets=None)
        return _exec_generator_select(plain, items2, [k], ascope, ctx)
    k = gen_at[0]
    call, alias = items[k]
    rows, names, gcols = GEN.generate(call, scope, ctx)
    if isinstance(alias, tuple):
        if len(alias) != len(names):
            raise QueryError(f"{call.name}() produces {len(names)} column(s), but {len(alias)} alias(es) were given")
        names = list(alias)
    elif alias != output_name(call):
        names = [alias] if len(names) == 1 else names
    sub = Scope(scope.names, TakenColumns(scope.cols, rows), scope.quals, int(rows.shape[0]), scope.device)
    sub.dist = getattr(scope, "dist", P.REPLICATED)
    out_names, out_cols = [], []
    for j, (e, nm) in enumerate(items):
        if j == k:
            out_names += names
            out_cols += gcols
        else:
            out_names.append(nm)
            out_cols.append(evaluate(e, sub, ctx))
    out = Table(out_names, out_cols, sub.length, scope.device)
    out.dist = sub.dist
    return distinct(out) if sel.distinct else out


def _deferred_ref(e: A.Expr, scope: Scope):
    """(scope.cols, index) for a bare, unambiguous column reference (no struct navigation), else None."""
    if not isinstance(e, A.Ident):
        return None
    parts = e.parts
    if len(parts) == 2 and scope.has_qualifier(parts[0]):
        hits = scope._find(parts[1], parts[0])
    elif len(parts) == 1:
        hits = scope._find(parts[0])
    else:
        return None
    return (scope.cols, hits[0]) if len(hits) == 1 else None


def _resolve_group_expr(g: A.Expr, scope: Scope, items) -> A.Expr:
    """GROUP BY may name a select-list alias when the name is not an input column (Spark groupByAliases)."""
    if isinstance(g, A.Ident) and scope.try_resolve(g.parts) is None and len(g.parts) == 1:
        for e, nm in items:
            if nm.lower() == g.parts[0].lower():
                return e
    if isinstance(g, A.Literal) and g.type in ("int", "long") and 1 <= g.value <= len(items):
        return items[g.value - 1][0]    # GROUP BY ordinal
    return g


def _aggregate(sel: A.Select, items, scope: Scope, ctx) -> Table:
    dev = scope.device
    n = scope.length
    gexprs = [_resolve_group_expr(g, scope, items) for g in sel.group_by]
    keys = []
    if gexprs:
        keys = [materialize(evaluate(g, scope, ctx)) for g in gexprs]
        keys = [k if not isinstance(k, (StructColumn, ArrayColumn)) else _nested_key(k) for k in keys]
    if P.active() and getattr(scope, "dist", P.REPLICATED) != P.REPLICATED:
        return _aggregate_distributed(sel, items, scope, ctx, gexprs, keys)
    if gexprs:
        with host_section("aggregate:group_rows"):
            groups = G.group_rows(keys)
    else:
        # global aggregate: one group, even over zero rows
        groups = G.Groups(torch.zeros(n, dtype=torch.int32 if dev.type == "cuda" else torch.int64, device=dev), 1,
                          torch.zeros(1, dtype=torch.int64, device=dev))
    aggs: Dict = {}
    for e, _ in items:
        _collect_aggs(e, ctx, aggs)
    if sel.having is not None:
        _collect_aggs(sel.having, ctx, aggs)
    with host_section("aggregate:aggs"):
        subst = _eval_aggs(aggs, scope, groups, ctx)
    ng = groups.ngroups
    if n == 0 and not gexprs:
        rep_scope = Scope(scope.names, [ConstColumn(None, c.dtype, 1, dev) for c in scope.cols], scope.quals, 1, dev)
    else:
        rep_scope = Scope(scope.names, TakenColumns(scope.cols, groups.rep), scope.quals, ng, dev)
    m = None
    if sel.having is not None:
        m = predicate_mask(evaluate(sel.having, rep_scope, ctx, subst))
    wcalls = [w for e, _ in items for w in W.window_calls(e)]
    if wcalls:
        # window functions see the grouped rows after HAVING (Spark evaluates them last)
        if m is not None:
            keep = torch.nonzero(m).flatten()
            rep_scope = Scope(rep_scope.names, TakenColumns(rep_scope.cols, keep), rep_scope.quals,
                              int(keep.shape[0]), dev)
            subst = {k: c.take(keep) for k, c in subst.items()}
            ng, m = rep_scope.length, None
        _window_columns(wcalls, lambda x: evaluate(x, rep_scope, ctx, subst), rep_scope.length, dev, subst)
    cols = [evaluate(e, rep_scope, ctx, subst) for e, _ in items]
    out = Table([nm for _, nm in items], cols, rep_scope.length, dev)
    if m is not None:
        out = out.filter(m)
    return out


def _window_columns(wcalls, ev, n, dev, subst: Dict) -> Dict:
    """Evaluate every window call once (keyed by expression) into ``subst``."""
    for w in wcalls:
        if w.key() not in subst:
            try:
                subst[w.key()] = W.evaluate_window(w, ev, n, dev)
            except W.WindowError as ex:
                raise QueryError(str(ex)) from ex
    return subst


def _window_repartition(scope: Scope, wcalls, ctx, is_agg: bool) -> Scope:
    """Make a partitioned scope exact for window functions: rows of one window partition must live on one rank.
    Shuffle by the PARTITION BY keys when every window call shares them; otherwise (no PARTITION BY, differing
    specs, or windows over aggregated rows) gather everything to every rank."""
    parts = {tuple(p.key() for p in w.partition) for w in wcalls}
    if is_agg or len(parts) != 1 or not wcalls[0].partition:
        return _gather_scope(scope)
    keys = [materialize(evaluate(p, scope, ctx)) for p in wcalls[0].partition]
    keys = [k if not isinstance(k, (StructColumn, ArrayColumn)) else _nested_key(k) for k in keys]
    return _shuffle_scope(scope, keys)


def _aggregate_distributed(sel, items, scope, ctx, gexprs, keys) -> Table:
    """GROUP BY over a partitioned input: two-phase RCCL aggregation (or a key shuffle for non-mergeable aggregates).
    Select expressions may only use group expressions and aggregates (Spark's rule)."""
    from . import distagg as D
    dev = scope.device
    aggs: Dict = {}
    for e, _ in items:
        _collect_aggs(e, ctx, aggs)
    if sel.having is not None:
        _collect_aggs(sel.having, ctx, aggs)
    if D.decomposable(aggs, ctx):
        out_keys, finals, ng, tag = D.distributed_aggregate(gexprs, keys, aggs, scope, ctx)
        subst = dict(finals)
        for g, k in zip(gexprs, out_keys):
            subst[g.key()] = k
        empty = Scope([], [], [], ng, dev)
        cols = [evaluate(e, empty, ctx, subst) for e, _ in items]
        out = Table([nm for _, nm in items], cols, ng, dev)
        if sel.having is not None:
            out = out.filter(predicate_mask(evaluate(sel.having, empty, ctx, subst)))
        out.dist = tag
        return out
    # non-decomposable: move rows to their key owner, then aggregate locally
    new_scope, new_keys = D.shuffle_rows_by_keys(scope, keys, ctx)
    new_scope.dist = P.REPLICATED    # rows of a key now live on one rank: local aggregation is exact
    sel2 = A.Select(sel.items, None, None, sel.group_by, sel.having, False)
    out = _aggregate(sel2, items, new_scope, ctx)
    out.dist = P.HASHED if gexprs else P.REPLICATED
    return out


def _nested_key(col):
    from .serialize import column_json_values
    from .column import strings_from_pylist
    return strings_from_pylist(column_json_values(col), col.device)


def _eval_aggs(aggs: Dict, scope: Scope, groups: G.Groups, ctx) -> Dict:
    """Evaluate a query's aggregate calls.  Plain COUNT / SUM / MIN / MAX / AVG calls are handed to
    ``G.aggregate_many`` together, so they can share one fused accumulation pass; the rest go one by one."""
    out = {}
    batch = []
    for k, call in aggs.items():
        name = "avg" if call.name == "mean" else call.name
        simple = (call.name not in ctx.udafs and not call.distinct and
                  (call.star or (name == "count" and not call.args) or
                   (name in ("count", "sum", "min", "max", "avg") and len(call.args) == 1)))
        if not simple:
            out[k] = _eval_agg(call, scope, groups, ctx)
            continue
        if call.star or not call.args:
            batch.append((k, None, "count_star"))
            continue
        arg = materialize(evaluate(call.args[0], scope, ctx))
        if isinstance(arg, ConstColumn):
            arg = arg.materialize()
        batch.append((k, arg, name))
    if batch:
        for (k, _, _), col in zip(batch, G.aggregate_many(groups, [(a, f) for _, a, f in batch], scope.length)):
            out[k] = col
    return out


def _eval_agg(call: A.Call, scope: Scope, groups: G.Groups, ctx) -> Column:
    name = call.name
    n = scope.length
    udaf = ctx.udafs.get(name)
    if udaf is not None:
        args = [materialize(evaluate(a, scope, ctx)) for a in call.args]
        return udaf.aggregate(args, groups, ctx)
    if call.star or (name == "count" and not call.args):
        return G.aggregate(groups, None, "count_star", n)
    if name == "count" and len(call.args) > 1:
        return _count_tuple([materialize(evaluate(a, scope, ctx)) for a in call.args], groups, n, call.distinct)
    if name in ("corr", "covar_pop", "covar_samp", "kurtosis", "skewness", "max_by", "min_by"):
        args = [materialize(evaluate(a, scope, ctx)) for a in call.args]
        args = [a.materialize() if isinstance(a, ConstColumn) else a for a in args]
        if name in ("max_by", "min_by"):
            return _arg_extreme(args, groups, n, name == "max_by")
        return _moments(name, args, groups)
    arg = materialize(evaluate(call.args[0], scope, ctx))
    if isinstance(arg, ConstColumn):
        arg = arg.materialize()
    if call.distinct:
        if name not in ("count", "sum", "avg", "approx_count_distinct"):
            name = name  # min/max(DISTINCT x) == min/max(x)
        else:
            return _distinct_agg(name, arg, groups, n)
    if name == "approx_count_distinct":
        return _distinct_agg("count", arg, groups, n)
    if name in ("first_value",):
        name = "first"
    if name in ("last_value",):
        name = "last"
    if name in ("collect_list", "collect_set"):
        return _collect(groups, arg, name == "collect_set")
    if name in ("percentile", "percentile_approx", "approx_percentile", "median"):
        p = 0.5 if name == "median" else evaluate(call.args[1], scope, ctx)
        return _percentile(groups, arg, p, exact=name in ("percentile", "median"))
    if name in ("count_if",):
        m = predicate_mask(arg)
        return G.aggregate(groups, PrimColumn("long", m.to(torch.int64)), "sum", n)
    if name in ("bool_and", "every", "bool_or", "any", "some"):
        v = arg
        r = G.aggregate(groups, PrimColumn("long", v.data.to(torch.int64), v.valid),
                        "min" if name in ("bool_and", "every") else "max", n)
        return PrimColumn("boolean", r.data != 0, r.valid)
    if name == "mean":
        name = "avg"
    return G.aggregate(groups, arg, name, n)


def _moments(name, args, groups: G.Groups):
    """corr / covar_pop / covar_samp (two arguments) and skewness / kurtosis (one) per group, from two device passes
    (group means, then centred co-moments with index_add): Spark's Corr / Covariance / CentralMomentAgg results —
    null for an empty group, NaN where Spark divides by zero (corr of a constant, covar_samp of one row), kurtosis
    as excess kurtosis."""
    ng = groups.ngroups
    xs = [cast_column(a, "double") if a.dtype != "double" else a for a in args]
    ok = xs[0].valid_mask()
    for a in xs[1:]:
        ok = ok & a.valid_mask()
    idx = torch.nonzero(ok).flatten()
    gid = groups.gid.to(torch.int64)[idx]
    vals = [a.data.to(torch.float64)[idx] for a in xs]
    dev = gid.device
    f64 = torch.float64

    def gsum(v):
        return torch.zeros(ng, dtype=f64, device=dev).index_add_(0, gid, v)
    cnt = gsum(torch.ones_like(vals[0]))
    safe = cnt.clamp(min=1)
    d = [v - (gsum(v) / safe)[gid] for v in vals]
    has = cnt > 0
    nan = torch.full_like(cnt, float("nan"))
    if name in ("corr", "covar_pop", "covar_samp"):
        if len(d) != 2:
            raise QueryError(f"{name} takes two arguments")
        cxy = gsum(d[0] * d[1])
        if name == "covar_pop":
            return PrimColumn("double", cxy / safe, has)
        if name == "covar_samp":
            return PrimColumn("double", torch.where(cnt > 1, cxy / (cnt - 1).clamp(min=1), nan), has)
        den = torch.sqrt(gsum(d[0] * d[0]) * gsum(d[1] * d[1]))
        return PrimColumn("double", torch.where(den > 0, cxy / torch.where(den > 0, den, torch.ones_like(den)), nan),
                          has)
    m2, m = gsum(d[0] * d[0]), cnt
    if name == "skewness":
        m3 = gsum(d[0] ** 3)
        r = torch.sqrt(m) * m3 / torch.where(m2 > 0, m2, torch.ones_like(m2)) ** 1.5
    else:
        m4 = gsum(d[0] ** 4)
        r = m * m4 / torch.where(m2 > 0, m2 * m2, torch.ones_like(m2)) - 3.0
    return PrimColumn("double", torch.where(m2 > 0, r, nan), has)


def _arg_extreme(args, groups: G.Groups, n, is_max: bool):
    """max_by(x, y) / min_by(x, y): x of the row with the largest / smallest non-null y per group (one device
    sort by (group, y); ties keep the first row in input order)."""
    if len(args) != 2:
        raise QueryError("max_by / min_by take two arguments")
    x, y = args
    from ..ops.sort import argsort_words, sort_spec_words
    ok = y.valid_mask()
    idx = torch.nonzero(ok).flatten()
    gid = groups.gid.to(torch.int64)[idx]
    ysub = y.take(idx)
    perm = argsort_words(sort_spec_words([(ysub, not is_max, False)]) + [gid])
    sg = gid[perm]
    first = torch.ones_like(sg, dtype=torch.bool)
    first[1:] = sg[1:] != sg[:-1]
    rows = idx[perm[first]]
    owner = sg[first]
    pick = torch.full((groups.ngroups,), -1, dtype=torch.int64, device=gid.device)
    pick[owner] = rows
    return _take_nullable(x, pick)


def _count_tuple(args, groups: G.Groups, n, distinct: bool):
    """count(a, b, …) — rows whose arguments are all non-null — and count(DISTINCT a, b, …), the distinct such
    tuples per group (Spark's Count over several children)."""
    args = [a.materialize() if isinstance(a, ConstColumn) else a for a in args]
    ok = args[0].valid_mask()
    for a in args[1:]:
        ok = ok & a.valid_mask()
    if not distinct:
        return G.aggregate(groups, PrimColumn("long", torch.zeros(n, dtype=torch.int64, device=ok.device), ok),
                           "count", n)
    gcol = PrimColumn("long", groups.gid.to(torch.int64))
    sub = G.group_rows([gcol] + args)
    first = sub.rep
    owner = G.Groups(groups.gid[first], groups.ngroups, groups.rep)
    m = int(first.shape[0])
    return G.aggregate(owner, PrimColumn("long", torch.zeros(m, dtype=torch.int64, device=ok.device), ok[first]),
                       "count", m)


def _distinct_agg(name, arg, groups: G.Groups, n):
    dev = groups.rep.device
    gcol = PrimColumn("long", groups.gid.to(torch.int64))
    sub = G.group_rows([gcol, arg])
    first_rows = sub.rep
    owner = G.Groups(groups.gid[first_rows], groups.ngroups, groups.rep)
    vals = arg.take(first_rows)
    if name == "count":
        return G.aggregate(owner, vals, "count", int(first_rows.shape[0]))
    return G.aggregate(owner, vals, "sum" if name == "sum" else "avg", int(first_rows.shape[0]))


def _percentile(groups: G.Groups, arg, p, exact: bool):
    """percentile / median (linear interpolation between the two nearest ranks) and percentile_approx (the
    smallest value whose rank reaches p·count — exact here) per group, from one device sort by (group, value).
    ``p`` may be a constant or an array of constants (→ array result)."""
    from .column import ArrayColumn
    dev = groups.rep.device
    ng = groups.ngroups
    if isinstance(p, ArrayColumn):
        ps = [float(e.value) if isinstance(e, ConstColumn) else float(e.to_pylist()[0]) for e in p.elements]
        return ArrayColumn([_percentile(groups, arg, ConstColumn(q, "double", 1, dev), exact) for q in ps], ng,
                           None, False, dev)
    q = float(p.value if isinstance(p, ConstColumn) else p)
    if not 0.0 <= q <= 1.0:
        raise QueryError("percentile must be in [0, 1]")
    if not isinstance(arg, PrimColumn):
        arg = cast_column(arg, "double")
    from .decimal import is_decimal, to_double
    dec = is_decimal(arg.dtype)
    # decimals: the exact percentile interpolates their double values (Spark's Percentile result is a double); the
    # approximate one returns an input VALUE, so it keeps the decimal type (ApproximatePercentile's dataType)
    x = to_double(arg).data if dec else arg.data.to(torch.float64)
    ok = arg.valid_mask()
    idx = torch.nonzero(ok).flatten()
    g = groups.gid.to(torch.int64)[idx]
    v = x[idx]
    o = torch.argsort(arg.data[idx] if (dec and arg.dtype.narrow) else v, stable=True)
    o = o[torch.argsort(g[o], stable=True)]
    g, v = g[o], v[o]
    cnt = torch.bincount(g, minlength=ng)
    start = torch.cumsum(cnt, 0) - cnt
    has = cnt > 0
    c1 = torch.clamp(cnt - 1, min=0)
    if exact:
        pos = q * c1.to(torch.float64)
        lo = torch.floor(pos).to(torch.int64)
        hi = torch.clamp(lo + 1, max=c1)
        fr = pos - lo.to(torch.float64)
        vl = v[torch.clamp(start + lo, max=max(0, v.numel() - 1))] if v.numel() else torch.zeros(ng, dtype=torch.float64,
                                                                                                device=dev)
        vh = v[torch.clamp(start + hi, max=max(0, v.numel() - 1))] if v.numel() else vl
        r = vl + fr * (vh - vl)
        return PrimColumn("double", r, has)
    k = torch.clamp(torch.ceil(q * cnt.to(torch.float64)).to(torch.int64) - 1, min=0)
    k = torch.minimum(k, c1)
    if dec:
        at = idx[o][torch.clamp(start + k, max=max(0, v.numel() - 1))] if v.numel() else \
            torch.zeros(ng, dtype=torch.int64, device=dev)
        return _take_nullable(arg, torch.where(has, at, torch.full_like(at, -1)))
    r = v[torch.clamp(start + k, max=max(0, v.numel() - 1))] if v.numel() else torch.zeros(ng, dtype=torch.float64,
                                                                                          device=dev)
    if arg.dtype in ("byte", "short", "int", "long"):
        return PrimColumn(arg.dtype, r.to(torch.int64), has)
    return PrimColumn(arg.dtype if arg.dtype in ("double", "float") else "double", r, has)


def _collect(groups: G.Groups, arg, as_set):
    """collect_list/collect_set → JSON array text per group (host-assisted)."""
    from .column import strings_from_pylist
    import json
    from .serialize import json_value
    vals = arg.to_pylist()
    gid = groups.gid.cpu().tolist()
    out = [[] for _ in range(groups.ngroups)]
    for v, g in zip(vals, gid):
        if v is None:
            continue
        if as_set and v in out[g]:
            continue
        out[g].append(v)
    from .types import ArrayType
    if isinstance(arg, (PrimColumn, StrColumn)) and isinstance(arg.dtype, str):
        # a real array column (fixed slots): explode, size, array functions and JSON output all take it
        from .sqlfuncs import array_from_pylist
        return array_from_pylist(out, arg.dtype, groups.rep.device)
    return strings_from_pylist([json.dumps([json_value(x, arg.dtype) for x in o], separators=(",", ":"))
                                for o in out], groups.rep.device, ArrayType(arg.dtype))


# ---------------------------------------------------------------------------------------------------------------
# ORDER BY
# ---------------------------------------------------------------------------------------------------------------

def _sort_key_tensor(col: Column) -> Tuple[torch.Tensor, torch.Tensor]:
    """(order key, valid): an int64 tensor whose *unsigned* order is the column's SQL order (dxa.ops.sort — device
    order-key kernels; strings are dense-ranked on the device)."""
    from ..ops.sort import column_order_key
    col = materialize(col)
    if not isinstance(col, (StrColumn, PrimColumn)):
        raise QueryError(f"cannot ORDER BY {col.dtype}")
    return column_order_key(col)


def _order_by(t: Table, items: List[A.OrderItem], ctx, src_scope: Optional[Scope],
              aliases: Optional[Dict] = None) -> Table:
    """One stable device radix argsort over all ORDER BY keys (dxa.ops.sort.argsort_words): per item an order key
    word and, when the column has nulls, a null-placement word above it."""
    from ..ops.sort import argsort_words, sort_spec_words
    if t.length <= 1:
        return t
    out_scope = Scope.of_table(t)
    specs = []
    for it in items:
        e = it.expr
        if isinstance(e, A.Literal) and e.type in ("int", "long"):
            col = t.columns[e.value - 1]
        else:
            try:
                col = evaluate(e, out_scope, ctx)
            except EvalError:
                named = (aliases or {}).get(e.key())
                if named is not None and t.column(named) is not None:
                    col = t.column(named)
                elif src_scope is None:
                    raise
                else:
                    col = evaluate(e, src_scope, ctx)
        col = materialize(col)
        if not isinstance(col, (StrColumn, PrimColumn, StructColumn)):
            raise QueryError(f"cannot ORDER BY {col.dtype}")
        nulls_first = it.nulls_first if it.nulls_first is not None else it.ascending
        specs.append((col, it.ascending, nulls_first))
    return t.take(argsort_words(sort_spec_words(specs)))
