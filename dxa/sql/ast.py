"""AST node types for the DataX-SQL dialect (the Spark-SQL subset the reference's flows use).

The reference hands every transform statement to ``spark.sql`` (DataProcessing/datax-host/src/main/scala/datax/
processor/CommonProcessorFactory.scala:249-294).  We own the whole front-end instead: these nodes are produced by
``dxa.sql.parser`` and consumed by the columnar planner in ``dxa.engine.query``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple, Any


class Expr:
    """Base expression node.  ``key()`` gives a structural identity used to match GROUP BY expressions."""

    def key(self):
        raise NotImplementedError

    def children(self) -> List["Expr"]:
        return []


@dataclass(eq=False)
class Literal(Expr):
    value: Any
    type: str  # 'long' | 'int' | 'short' | 'byte' | 'double' | 'string' | 'boolean' | 'null' | decimal(p,s)
    suffixed: bool = False      # typed by a suffix (10L, 10S, 10Y, 1.0D, 1BD): a folded minus keeps the type
    integral: bool = False      # an unsuffixed integer literal (its type follows its value, the sign included)

    def key(self):
        return ("lit", self.type, self.value)


@dataclass(eq=False)
class Ident(Expr):
    """Possibly-dotted identifier: ``a``, ``t.a``, ``Raw.deviceDetails.deviceId``."""
    parts: Tuple[str, ...]

    def key(self):
        return ("id",) + tuple(p.lower() for p in self.parts)

    @property
    def name(self):
        return self.parts[-1]


@dataclass(eq=False)
class Star(Expr):
    qualifier: Tuple[str, ...] = ()

    def key(self):
        return ("star",) + self.qualifier


@dataclass(eq=False)
class Call(Expr):
    name: str          # lower-cased function name
    args: List[Expr]
    distinct: bool = False
    star: bool = False  # COUNT(*)

    def key(self):
        return ("call", self.name, self.distinct, self.star) + tuple(a.key() for a in self.args)

    def children(self):
        return list(self.args)


@dataclass(eq=False)
class WindowCall(Expr):
    """``func(args) OVER (PARTITION BY ... ORDER BY ... [ROWS|RANGE frame])``.  ``frame`` is ``(kind, start, end)``
    with each bound ``(type, offset)``: type in unbounded_preceding / preceding / current / following /
    unbounded_following."""
    func: Call
    partition: List[Expr] = field(default_factory=list)
    order: List["OrderItem"] = field(default_factory=list)
    frame: Optional[tuple] = None
    ref: Optional[str] = None          # ``OVER w``: a window the query's WINDOW clause names (resolved by the parser)

    def key(self):
        return ("over", self.func.key(), tuple(p.key() for p in self.partition),
                tuple((o.expr.key(), o.ascending, o.nulls_first) for o in self.order), self.frame)

    def children(self):
        return list(self.func.args) + list(self.partition) + [o.expr for o in self.order]


@dataclass(eq=False)
class BinOp(Expr):
    op: str            # '+','-','*','/','%','=','!=','<','<=','>','>=','and','or','||','<=>','&','|','^','div'
    left: Expr
    right: Expr

    def key(self):
        return ("bin", self.op, self.left.key(), self.right.key())

    def children(self):
        return [self.left, self.right]


@dataclass(eq=False)
class UnaryOp(Expr):
    op: str            # 'not', '-', '+', '~'
    operand: Expr

    def key(self):
        return ("un", self.op, self.operand.key())

    def children(self):
        return [self.operand]


@dataclass(eq=False)
class IsNull(Expr):
    operand: Expr
    negated: bool = False

    def key(self):
        return ("isnull", self.negated, self.operand.key())

    def children(self):
        return [self.operand]


@dataclass(eq=False)
class InList(Expr):
    operand: Expr
    items: List[Expr]
    negated: bool = False

    def key(self):
        return ("in", self.negated, self.operand.key()) + tuple(i.key() for i in self.items)

    def children(self):
        return [self.operand] + list(self.items)


@dataclass(eq=False)
class Between(Expr):
    operand: Expr
    low: Expr
    high: Expr
    negated: bool = False

    def key(self):
        return ("between", self.negated, self.operand.key(), self.low.key(), self.high.key())

    def children(self):
        return [self.operand, self.low, self.high]


@dataclass(eq=False)
class Like(Expr):
    operand: Expr
    pattern: Expr
    negated: bool = False
    regex: bool = False  # RLIKE

    def key(self):
        return ("like", self.negated, self.regex, self.operand.key(), self.pattern.key())

    def children(self):
        return [self.operand, self.pattern]


@dataclass(eq=False)
class Case(Expr):
    operand: Optional[Expr]
    whens: List[Tuple[Expr, Expr]]
    default: Optional[Expr]

    def key(self):
        return ("case", self.operand.key() if self.operand else None,
                tuple((w.key(), t.key()) for w, t in self.whens), self.default.key() if self.default else None)

    def children(self):
        out = [self.operand] if self.operand else []
        for w, t in self.whens:
            out += [w, t]
        if self.default:
            out.append(self.default)
        return out


@dataclass(eq=False)
class Cast(Expr):
    operand: Expr
    to: str
    typed_literal: bool = False        # ``TIMESTAMP '…'`` / ``DATE '…'``: a literal of that type (Spark's typed literal)

    def key(self):
        return ("cast", self.to, self.operand.key())

    def children(self):
        return [self.operand]


@dataclass(eq=False)
class Subscript(Expr):
    """``base[index]`` on maps / arrays, and ``base.field`` on a non-identifier base (e.g. ``RuleObject.x`` after a call)."""
    base: Expr
    index: Expr
    dot: bool = False

    def key(self):
        return ("sub", self.dot, self.base.key(), self.index.key())

    def children(self):
        return [self.base, self.index]


@dataclass(eq=False)
class Interval(Expr):
    micros: int

    def key(self):
        return ("interval", self.micros)


# ----------------------------------------------------------------------------------------------------------------
# Relations / statements
# ----------------------------------------------------------------------------------------------------------------

@dataclass(eq=False)
class SelectItem:
    expr: Expr
    alias: Optional[str] = None      # a tuple of names: a generator's multi-alias ``AS (a, b)``


@dataclass(eq=False)
class TableRef:
    name: str
    alias: Optional[str] = None
    timewindow: Optional[str] = None   # DataX extension: FROM t TIMEWINDOW('5 minutes')
    sample: Optional[tuple] = None     # TABLESAMPLE: ("fraction", f) | ("rows", n)


@dataclass(eq=False)
class SubqueryRef:
    query: "Query"
    alias: Optional[str] = None
    sample: Optional[tuple] = None
    columns: Optional[tuple] = None        # ``(…) AS t(x, y)``: the output columns renamed positionally


@dataclass(eq=False)
class Join:
    left: Any
    right: Any
    kind: str          # 'inner' | 'left' | 'right' | 'full' | 'cross' | 'semi' | 'anti'
    on: Optional[Expr] = None
    using: Optional[List[str]] = None
    natural: bool = False              # NATURAL JOIN: USING every column name both sides share
    broadcast: Optional[set] = None    # relation names/aliases a BROADCAST hint names (lower case)


@dataclass(eq=False)
class Pivot:
    """``FROM src PIVOT (aggs FOR cols IN (values))``: group by every column of ``src`` that no aggregate and no
    pivot column reads, one output column per (value, aggregate)."""
    source: Any
    aggs: List[Tuple[Expr, Optional[str]]]
    columns: List[Expr]
    values: List[Tuple[List[Expr], Optional[str]]]
    alias: Optional[str] = None


@dataclass(eq=False)
class OrderItem:
    expr: Expr
    ascending: bool = True
    nulls_first: Optional[bool] = None


@dataclass(eq=False)
class Select:
    items: List[SelectItem]
    from_: Any = None
    where: Optional[Expr] = None
    group_by: List[Expr] = field(default_factory=list)
    having: Optional[Expr] = None
    distinct: bool = False
    grouping_sets: Optional[List[List[Expr]]] = None     # ROLLUP / CUBE / GROUPING SETS (subsets of group_by)
    hints: List[Tuple[str, List[str]]] = field(default_factory=list)    # /*+ NAME(args) */


@dataclass(eq=False)
class SetOp:
    op: str            # 'union' | 'intersect' | 'except'
    all: bool
    left: Any
    right: Any


@dataclass(eq=False)
class Query:
    body: Any          # Select | SetOp
    order_by: List[OrderItem] = field(default_factory=list)
    limit: Optional[int] = None
    ctes: List[Tuple[str, "Query"]] = field(default_factory=list)     # WITH name AS (query), …
    distribute_by: List[Expr] = field(default_factory=list)           # DISTRIBUTE BY / CLUSTER BY keys
    sort_by: List["OrderItem"] = field(default_factory=list)          # SORT BY (within each rank's partition)


@dataclass(eq=False)
class SubqueryExpr(Expr):
    """``(SELECT …)`` as a value (kind ``scalar``), ``EXISTS (SELECT …)`` (``exists``) or ``x [NOT] IN (SELECT …)``
    (``in``, with ``operand`` = x).  Uncorrelated: the sub-query is planned on its own."""
    kind: str
    query: Query
    operand: Optional[Expr] = None
    negated: bool = False

    def key(self):
        return ("subq", self.kind, id(self.query), self.negated,
                None if self.operand is None else self.operand.key())

    def children(self):
        return [self.operand] if self.operand is not None else []


@dataclass(eq=False)
class Lambda(Expr):
    """``x -> expr`` / ``(x, i) -> expr`` argument of a higher-order array function."""
    params: Tuple[str, ...]
    body: Expr

    def key(self):
        return ("lambda", tuple(p.lower() for p in self.params), self.body.key())

    def children(self):
        return [self.body]


@dataclass(eq=False)
class LateralView:
    """``FROM src LATERAL VIEW [OUTER] generator(args) alias AS c1[, c2]``."""
    source: Any
    generator: Call
    outer: bool = False
    alias: Optional[str] = None
    columns: List[str] = field(default_factory=list)


def walk(e: Expr):
    """Pre-order traversal of an expression tree (an explicit stack: no generator chain per tree level)."""
    stack = [e]
    pop, extend = stack.pop, stack.extend
    while stack:
        n = pop()
        yield n
        ch = n.children()
        if ch:
            extend(reversed(ch))


_SUMMARY: dict = {}


def summary(e: Expr):
    """(names of the calls in ``e``, its window calls, whether a call takes a ``*`` argument) — read by every
    statement of every batch, computed once per expression node (statement ASTs live for the flow)."""
    got = _SUMMARY.get(id(e))
    if got is not None and got[0] is e:
        return got[1]
    calls, wins, star = set(), [], False
    for n in walk(e):
        if isinstance(n, Call):
            calls.add(n.name)
            if not star and ((n.star and n.name != "count") or any(isinstance(a, Star) for a in n.args)):
                star = True
        elif isinstance(n, WindowCall):
            wins.append(n)
    out = (frozenset(calls), tuple(wins), star)
    if len(_SUMMARY) >= 8192:
        _SUMMARY.clear()
    _SUMMARY[id(e)] = (e, out)
    return out


def replace(e, fn):
    """Copy of expression ``e`` with every node for which ``fn(node)`` returns an Expr replaced by it (pre-order: a
    replaced node's subtree is not visited).  Fields holding expressions or lists of them are rebuilt; other fields
    are shared."""
    import dataclasses
    if not isinstance(e, Expr):
        return e
    r = fn(e)
    if r is not None:
        return r
    if not dataclasses.is_dataclass(e):
        return e
    changes = {}
    for f in dataclasses.fields(e):
        v = getattr(e, f.name)
        if isinstance(v, Expr):
            nv = replace(v, fn)
        elif isinstance(v, list) and any(isinstance(x, Expr) for x in v):
            nv = [replace(x, fn) for x in v]
        else:
            continue
        changes[f.name] = nv
    return dataclasses.replace(e, **changes) if changes else e
