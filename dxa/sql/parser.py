"""Tokenizer + recursive-descent parser for the DataX-SQL dialect.

Supported surface (everything the reference's fixtures and sample flows exercise, plus the usual Spark-SQL
operators): SELECT [DISTINCT] … FROM … [JOIN … ON …] [WHERE] [GROUP BY] [HAVING] [ORDER BY] [LIMIT];
UNION [ALL] / INTERSECT / EXCEPT; sub-queries in FROM; CASE, CAST, IN, BETWEEN, LIKE/RLIKE, IS [NOT] NULL;
back-ticked identifiers, nested field access (``a.b.c``), map/array subscripts, ``t.*``; the DataX
``TIMEWINDOW('5 minutes')`` FROM-suffix (reference rewrite: Services/DataX.Flow/DataX.Flow.CodegenRules/Engine.cs:595-627).

Anything outside the subset raises ``SqlError`` with the offending position — we fail loudly rather than guess.
"""
from __future__ import annotations

import re
from typing import List, Optional

from . import ast as A


class SqlError(Exception):
    pass


KEYWORDS = {
    "select", "distinct", "from", "where", "group", "by", "having", "order", "limit", "as", "and", "or", "not",
    "in", "is", "null", "true", "false", "case", "when", "then", "else", "end", "cast", "join", "inner", "left",
    "right", "full", "outer", "cross", "on", "using", "union", "all", "intersect", "except", "asc", "desc",
    "between", "like", "rlike", "regexp", "nulls", "first", "last", "semi", "anti", "timewindow", "interval", "div",
}

_TOKEN_RE = re.compile(r"""
    (?P<hint>/\*\+.*?\*/) |
    (?P<ws>\s+|--[^\n]*|/\*.*?\*/) |
    (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?[LlDdSsYy]?(?:BD)?) |
    (?P<str>'(?:[^'\\]|\\.|'')*'|"(?:[^"\\]|\\.|"")*") |
    (?P<bq>`(?:[^`]|``)*`) |
    (?P<id>[A-Za-z_][A-Za-z0-9_$]*) |
    (?P<op><=>|<>|!=|==|<=|>=|\|\||&&|[-+*/%=<>(),.;\[\]~&|^!:])
""", re.VERBOSE | re.DOTALL)


class Tok:
    __slots__ = ("kind", "text", "pos")

    def __init__(self, kind, text, pos):
        self.kind, self.text, self.pos = kind, text, pos

    def __repr__(self):
        return f"Tok({self.kind},{self.text!r})"


def _unquote(s: str) -> str:
    q = s[0]
    body = s[1:-1]
    out = []
    i = 0
    while i < len(body):
        c = body[i]
        if c == "\\" and i + 1 < len(body):
            n = body[i + 1]
            out.append({"n": "\n", "t": "\t", "r": "\r", "0": "\0", "b": "\b"}.get(n, n))
            i += 2
            continue
        if c == q and i + 1 < len(body) and body[i + 1] == q:
            out.append(q)
            i += 2
            continue
        out.append(c)
        i += 1
    return "".join(out)


def tokenize(sql: str) -> List[Tok]:
    toks: List[Tok] = []
    pos = 0
    while pos < len(sql):
        m = _TOKEN_RE.match(sql, pos)
        if not m:
            raise SqlError(f"unexpected character {sql[pos]!r} at {pos} in: {sql[max(0, pos - 30):pos + 30]!r}")
        kind = m.lastgroup
        text = m.group(kind)
        if kind == "ws":
            pass
        elif kind == "id":
            low = text.lower()
            toks.append(Tok("kw" if low in KEYWORDS else "id", text, pos))
        elif kind == "bq":
            toks.append(Tok("id", text[1:-1].replace("``", "`"), pos))
        elif kind == "str":
            toks.append(Tok("str", _unquote(text), pos))
        elif kind == "hint":
            toks.append(Tok("hint", text[3:-2], pos))
        else:
            toks.append(Tok(kind, text, pos))
        pos = m.end()
    toks.append(Tok("eof", "", pos))
    return toks


_INTERVAL_UNITS = {
    "microsecond": 1, "microseconds": 1, "millisecond": 1000, "milliseconds": 1000,
    "second": 1_000_000, "seconds": 1_000_000, "minute": 60_000_000, "minutes": 60_000_000,
    "hour": 3_600_000_000, "hours": 3_600_000_000, "day": 86_400_000_000, "days": 86_400_000_000,
    "week": 7 * 86_400_000_000, "weeks": 7 * 86_400_000_000,
}


def parse_duration_micros(text: str) -> int:
    """'5 minutes' / '60 second' / '1 hour 30 minutes' → microseconds (reference: SettingDictionary.getDuration)."""
    parts = text.strip().lower().split()
    if len(parts) == 1:
        m = re.match(r"^(\d+)\s*([a-z]+)$", parts[0])
        if m:
            parts = [m.group(1), m.group(2)]
        elif re.match(r"^\d+$", parts[0]):
            return int(parts[0]) * 1_000_000
    if len(parts) % 2:
        raise SqlError(f"bad duration {text!r}")
    total = 0
    for i in range(0, len(parts), 2):
        n = float(parts[i])
        unit = parts[i + 1]
        if unit not in _INTERVAL_UNITS:
            raise SqlError(f"bad duration unit {unit!r} in {text!r}")
        total += int(n * _INTERVAL_UNITS[unit])
    return total


_EXTRACT_FIELDS = {"year": "year", "years": "year", "yr": "year", "quarter": "quarter", "qtr": "quarter",
                   "month": "month", "months": "month", "mon": "month", "week": "weekofyear", "weeks": "weekofyear",
                   "day": "dayofmonth", "days": "dayofmonth", "d": "dayofmonth", "dayofweek": "dayofweek",
                   "dow": "dayofweek", "doy": "dayofyear", "dayofyear": "dayofyear", "hour": "hour", "hours": "hour",
                   "h": "hour", "minute": "minute", "minutes": "minute", "min": "minute", "second": "second",
                   "seconds": "second", "s": "second"}


class Parser:
    def __init__(self, sql: str):
        self.sql = sql
        self.toks = tokenize(sql)
        self.i = 0

    # -- token helpers -------------------------------------------------------------------------------------------
    @property
    def cur(self) -> Tok:
        return self.toks[self.i]

    def peek(self, k=1) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def is_kw(self, *words, tok=None) -> bool:
        t = tok or self.cur
        return t.kind == "kw" and t.text.lower() in words

    def is_op(self, *ops, tok=None) -> bool:
        t = tok or self.cur
        return t.kind == "op" and t.text in ops

    def advance(self) -> Tok:
        t = self.cur
        self.i += 1
        return t

    def accept_kw(self, *words) -> bool:
        if self.is_kw(*words):
            self.i += 1
            return True
        return False

    def accept_op(self, *ops) -> bool:
        if self.is_op(*ops):
            self.i += 1
            return True
        return False

    def expect_kw(self, word):
        if not self.accept_kw(word):
            self.error(f"expected {word.upper()}")

    def expect_op(self, op):
        if not self.accept_op(op):
            self.error(f"expected '{op}'")

    def error(self, msg):
        t = self.cur
        raise SqlError(f"{msg} at position {t.pos} near {self.sql[max(0, t.pos - 40):t.pos + 40]!r}")

    def ident(self) -> str:
        t = self.cur
        if t.kind == "id":
            self.i += 1
            return t.text
        # non-reserved keywords usable as identifiers
        if t.kind == "kw" and t.text.lower() in ("first", "last", "semi", "anti", "nulls", "timewindow", "interval",
                                                   "div", "regexp"):
            self.i += 1
            return t.text
        self.error("expected identifier")

    # -- statements ----------------------------------------------------------------------------------------------
    def parse_query(self) -> A.Query:
        ctes = []
        if self.is_word("with") and self.peek().kind in ("id", "kw") and not self.is_op("(", tok=self.peek()):
            self.advance()
            while True:
                name = self.ident()
                self.expect_kw("as")
                self.expect_op("(")
                ctes.append((name, self.parse_query()))
                self.expect_op(")")
                if not self.accept_op(","):
                    break
        body = self.parse_set_expr()
        q = A.Query(body=body, ctes=ctes)
        if self.accept_kw("order"):
            self.expect_kw("by")
            q.order_by = self.parse_order_items()
        if self.is_word("cluster") and self.is_kw("by", tok=self.peek()):
            self.advance()
            self.advance()
            q.distribute_by = self._expr_list()
            q.sort_by = [A.OrderItem(e) for e in q.distribute_by]
        else:
            if self.is_word("distribute") and self.is_kw("by", tok=self.peek()):
                self.advance()
                self.advance()
                q.distribute_by = self._expr_list()
            if self.is_word("sort") and self.is_kw("by", tok=self.peek()):
                self.advance()
                self.advance()
                q.sort_by = self.parse_order_items()
        if (q.distribute_by or q.sort_by) and q.order_by:
            self.error("ORDER BY cannot be combined with SORT BY / DISTRIBUTE BY / CLUSTER BY")
        if self.accept_kw("limit"):
            t = self.advance()
            if t.kind != "num":
                self.error("expected LIMIT count")
            q.limit = int(t.text)
        return q

    def _expr_list(self):
        out = [self.parse_expr()]
        while self.accept_op(","):
            out.append(self.parse_expr())
        return out

    def _alias_word_ok(self) -> bool:
        """An identifier right after a relation is its alias — unless it opens a clause that Spark does not reserve
        (NATURAL JOIN, PIVOT (…), TABLESAMPLE (…), DISTRIBUTE/SORT/CLUSTER BY, LATERAL VIEW)."""
        t, n = self.cur, self.peek()
        if t.kind != "id":
            return False
        w = t.text.lower()
        if w == "natural" and (self.is_kw("join", "inner", "left", "right", "full", tok=n)):
            return False
        if w in ("pivot", "tablesample") and self.is_op("(", tok=n):
            return False
        if w in ("distribute", "sort", "cluster") and self.is_kw("by", tok=n):
            return False
        if w == "lateral" and self.is_word("view", tok=n):
            return False
        if w == "window" and n.kind in ("id", "kw") and self.is_kw("as", tok=self.peek(2)):
            return False                 # WINDOW w AS (…) after the FROM clause
        return True

    def parse_order_items(self):
        items = []
        while True:
            e = self.parse_expr()
            asc = True
            if self.accept_kw("desc"):
                asc = False
            else:
                self.accept_kw("asc")
            nf = None
            if self.accept_kw("nulls"):
                if self.accept_kw("first"):
                    nf = True
                else:
                    self.expect_kw("last")
                    nf = False
            items.append(A.OrderItem(e, asc, nf))
            if not self.accept_op(","):
                return items

    def parse_set_expr(self):
        left = self.parse_set_term()
        while self.is_kw("union", "except") or (self.is_kw("intersect")):
            op = self.advance().text.lower()
            is_all = self.accept_kw("all")
            if not is_all:
                self.accept_kw("distinct")
            right = self.parse_set_term()
            left = A.SetOp(op, is_all, left, right)
        return left

    def parse_set_term(self):
        if self.is_word("values") and (self.is_op("(", tok=self.peek()) or self.peek().kind in ("num", "str")):
            return self._parse_values().body
        if self.is_op("("):
            # parenthesised query
            save = self.i
            self.advance()
            if self.is_kw("select") or self.is_op("(") or self.is_word("values"):
                q = self.parse_query()
                self.expect_op(")")
                if q.order_by or q.limit is not None:
                    return A.SetOp("wrap", True, q, None)
                return q.body
            self.i = save
        return self.parse_select()

    def parse_select(self) -> A.Select:
        self.expect_kw("select")
        hints = []
        while self.cur.kind == "hint":
            hints += _parse_hints(self.advance().text)
        distinct = self.accept_kw("distinct")
        if not distinct:
            self.accept_kw("all")
        items = []
        while True:
            items.append(self.parse_select_item())
            if not self.accept_op(","):
                break
        sel = A.Select(items=items, distinct=distinct, hints=hints)
        if self.accept_kw("from"):
            sel.from_ = self.parse_from()
            bc = {a.lower() for name, args in hints if name in _BROADCAST_HINTS for a in args}
            if bc:
                _mark_broadcast(sel.from_, bc)
        if self.accept_kw("where"):
            sel.where = self.parse_expr()
        if self.accept_kw("group"):
            self.expect_kw("by")
            self._parse_group_by(sel)
        if self.accept_kw("having"):
            sel.having = self.parse_expr()
        if self.is_word("window") and self.peek().kind in ("id", "kw"):
            self._parse_window_clause(sel)
        return sel

    def _parse_window_clause(self, sel: A.Select):
        """``WINDOW w AS (PARTITION BY … ORDER BY … frame), w2 AS w`` → every ``OVER w`` of the select list,
        HAVING and ORDER BY takes that specification."""
        self.advance()
        defs = {}
        while True:
            name = self.ident().lower()
            self.expect_kw("as")
            if self.accept_op("("):
                defs[name] = self._window_spec()
            else:
                other = self.ident().lower()
                if other not in defs:
                    self.error(f"window {other} is not defined")
                defs[name] = defs[other]
            if not self.accept_op(","):
                break

        def fill(node):
            if isinstance(node, A.WindowCall) and node.ref is not None:
                spec = defs.get(node.ref.lower())
                if spec is None:
                    self.error(f"window {node.ref} is not defined")
                part, order, frame = spec
                return A.WindowCall(A.replace(node.func, fill), list(part), list(order), frame)
            return None
        sel.items = [A.SelectItem(A.replace(it.expr, fill), it.alias) for it in sel.items]
        if sel.having is not None:
            sel.having = A.replace(sel.having, fill)
        self._window_defs = defs

    def _parse_group_by(self, sel: A.Select):
        """GROUP BY e, … [WITH ROLLUP | WITH CUBE] | ROLLUP(…) | CUBE(…) | GROUPING SETS ((…), …)."""
        def expr_list():
            self.expect_op("(")
            out = []
            if not self.is_op(")"):
                out.append(self.parse_expr())
                while self.accept_op(","):
                    out.append(self.parse_expr())
            self.expect_op(")")
            return out

        def uniq(exprs):
            seen, out = set(), []
            for e in exprs:
                if e.key() not in seen:
                    seen.add(e.key())
                    out.append(e)
            return out

        if self.is_word("rollup", "cube") and self.is_op("(", tok=self.peek()):
            kind = self.advance().text.lower()
            cols = expr_list()
            sel.group_by = cols
            sel.grouping_sets = _rollup(cols) if kind == "rollup" else _cube(cols)
            return
        if self.is_word("grouping") and self.is_word("sets", tok=self.peek()):
            self.advance()
            self.advance()
            self.expect_op("(")
            sets = []
            while True:
                if self.is_op("("):
                    sets.append(expr_list())
                else:
                    sets.append([self.parse_expr()])
                if not self.accept_op(","):
                    break
            self.expect_op(")")
            sel.group_by = uniq([e for st in sets for e in st])
            sel.grouping_sets = sets
            return
        while True:
            sel.group_by.append(self.parse_expr())
            if not self.accept_op(","):
                break
        if self.is_word("grouping") and self.is_word("sets", tok=self.peek()):
            # GROUP BY a, b GROUPING SETS ((a), (b), ()) — Spark 2.4's form: the list names the grouping columns
            self.advance()
            self.advance()
            self.expect_op("(")
            sets = []
            while True:
                if self.is_op("("):
                    sets.append(expr_list())
                else:
                    sets.append([self.parse_expr()])
                if not self.accept_op(","):
                    break
            self.expect_op(")")
            sel.group_by = uniq(sel.group_by + [e for st in sets for e in st])
            sel.grouping_sets = sets
            return
        if self.is_word("with") and self.is_word("rollup", "cube", tok=self.peek()):
            self.advance()
            kind = self.advance().text.lower()
            sel.grouping_sets = _rollup(sel.group_by) if kind == "rollup" else _cube(sel.group_by)

    def parse_select_item(self) -> A.SelectItem:
        if self.is_op("*"):
            self.advance()
            return A.SelectItem(A.Star())
        # qualified star  a.b.*
        j = self.i
        quals = []
        while self.toks[j].kind in ("id",) and self.toks[j + 1].kind == "op" and self.toks[j + 1].text == ".":
            quals.append(self.toks[j].text)
            if self.toks[j + 2].kind == "op" and self.toks[j + 2].text == "*":
                self.i = j + 3
                return A.SelectItem(A.Star(tuple(quals)))
            j += 2
        e = self.parse_expr()
        alias = None
        if self.accept_kw("as"):
            if self.accept_op("("):
                # multi-alias of a generator: stack(2, 1, 'a', 2, 'b') AS (x, y)
                names = [self.ident()]
                while self.accept_op(","):
                    names.append(self.ident())
                self.expect_op(")")
                alias = tuple(names)
            else:
                alias = self.ident()
        elif self.cur.kind == "id":
            alias = self.advance().text
        return A.SelectItem(e, alias)

    def parse_from(self):
        left = self.parse_table_primary()
        while True:
            if self.is_word("lateral") and self.is_word("view", tok=self.peek()):
                self.advance()
                self.advance()
                outer = self.accept_kw("outer")
                gen = self.parse_primary()
                if not isinstance(gen, A.Call):
                    self.error("LATERAL VIEW expects a generator function call")
                alias = None
                if not self.is_kw("as"):
                    alias = self.ident()
                cols = []
                if self.accept_kw("as"):
                    cols.append(self.ident())
                    while self.accept_op(","):
                        cols.append(self.ident())
                left = A.LateralView(left, gen, outer, alias, cols)
                continue
            if self.accept_op(","):
                right = self.parse_table_primary()
                left = A.Join(left, right, "cross")
                continue
            kind = None
            save = self.i
            natural = False
            if self.is_word("natural") and self.is_kw("join", "inner", "left", "right", "full", tok=self.peek()):
                self.advance()
                natural = True
            if self.accept_kw("join"):
                kind = "inner"
            elif self.accept_kw("inner"):
                self.expect_kw("join")
                kind = "inner"
            elif self.accept_kw("cross"):
                self.expect_kw("join")
                kind = "cross"
            elif self.is_kw("left", "right", "full"):
                side = self.advance().text.lower()
                if side == "left" and self.accept_kw("semi"):
                    kind = "semi"
                elif side == "left" and self.accept_kw("anti"):
                    kind = "anti"
                else:
                    self.accept_kw("outer")
                    kind = side
                self.expect_kw("join")
            if kind is None:
                self.i = save
                if self.is_word("pivot") and self.is_op("(", tok=self.peek()):
                    left = self.parse_pivot(left)
                    continue
                return left
            if natural and kind in ("semi", "anti", "cross"):
                self.error(f"NATURAL {kind.upper()} JOIN is not supported")
            right = self.parse_table_primary()
            on = None
            using = None
            if natural:
                left = A.Join(left, right, kind, None, None, natural=True)
                continue
            if self.accept_kw("on"):
                on = self.parse_expr()
            elif self.accept_kw("using"):
                self.expect_op("(")
                using = [self.ident()]
                while self.accept_op(","):
                    using.append(self.ident())
                self.expect_op(")")
            left = A.Join(left, right, kind, on, using)

    def _parse_values(self) -> A.Query:
        """``VALUES (1, 'a'), (2, 'b')`` / ``VALUES 1, 2`` (Spark's inline table) → a UNION ALL of one-row SELECTs
        named col1, col2, … (balanced, so a long list stays shallow); the set operation widens each column to the
        rows' common type as Spark's inline-table resolution does."""
        self.advance()                                   # VALUES
        rows = []
        while True:
            if self.is_op("(") and not self._at_query_after_paren():
                self.advance()
                row = [self.parse_expr()]
                while self.accept_op(","):
                    row.append(self.parse_expr())
                self.expect_op(")")
            else:
                row = [self.parse_expr()]
            rows.append(row)
            if not self.accept_op(","):
                break
        width = len(rows[0])
        if any(len(r) != width for r in rows):
            self.error("VALUES rows must have the same number of columns")
        names = [f"col{i + 1}" for i in range(width)]
        sels = [A.Select(items=[A.SelectItem(e, nm) for e, nm in zip(r, names)]) for r in rows]

        def tree(lo, hi):
            if hi - lo == 1:
                return sels[lo]
            mid = (lo + hi) // 2
            return A.SetOp("union", True, tree(lo, mid), tree(mid, hi))
        return A.Query(tree(0, len(sels)))

    def _at_query_after_paren(self) -> bool:
        t = self.peek()
        return t.kind in ("id", "kw") and t.text.lower() in ("select", "with", "values")

    def _alias_columns(self):
        """``AS t`` / ``t`` / ``AS t(x, y)`` after a derived table → (alias, column names or None)."""
        alias, cols = None, []
        if self.accept_kw("as"):
            alias = self.ident()
        elif self._alias_word_ok():
            alias = self.advance().text
        if alias is not None and self.accept_op("("):
            cols.append(self.ident())
            while self.accept_op(","):
                cols.append(self.ident())
            self.expect_op(")")
        return alias, (tuple(cols) or None)

    def parse_table_primary(self):
        if self.is_word("values") and (self.is_op("(", tok=self.peek()) or self.peek().kind in ("num", "str")):
            q = self._parse_values()
            alias, cols = self._alias_columns()
            return A.SubqueryRef(q, alias, None, cols)
        if self.accept_op("("):
            q = self.parse_query()
            self.expect_op(")")
            sample = self.parse_sample()
            alias, cols = self._alias_columns()
            return A.SubqueryRef(q, alias, sample, cols)
        name = self.ident()
        while self.accept_op("."):
            name += "." + self.ident()
        tw = None
        if self.accept_kw("timewindow"):
            self.expect_op("(")
            t = self.advance()
            if t.kind != "str":
                self.error("TIMEWINDOW expects a string literal")
            tw = t.text
            self.expect_op(")")
        sample = self.parse_sample()
        alias = None
        if self.accept_kw("as"):
            alias = self.ident()
        elif self._alias_word_ok():
            alias = self.advance().text
        return A.TableRef(name, alias, tw, sample)

    def parse_sample(self):
        """``TABLESAMPLE (x PERCENT | n ROWS | BUCKET x OUT OF y)`` → ("fraction", f) | ("rows", n)."""
        if not (self.is_word("tablesample") and self.is_op("(", tok=self.peek())):
            return None
        self.advance()
        self.advance()
        if self.is_word("bucket"):
            self.advance()
            x = self._sample_number()
            if not (self.accept_word("out") and self.accept_word("of")):
                self.error("expected OUT OF")
            y = self._sample_number()
            if y <= 0 or x <= 0 or x > y:
                self.error("TABLESAMPLE BUCKET x OUT OF y needs 0 < x <= y")
            out = ("fraction", x / y)
        else:
            v = self._sample_number()
            if self.accept_word("percent"):
                if not 0 <= v <= 100:
                    self.error("TABLESAMPLE percentage must be between 0 and 100")
                out = ("fraction", v / 100.0)
            elif self.accept_word("rows"):
                if v < 0 or v != int(v):
                    self.error("TABLESAMPLE row count must be a non-negative integer")
                out = ("rows", int(v))
            else:
                self.error("expected PERCENT or ROWS")
        self.expect_op(")")
        return out

    def _sample_number(self) -> float:
        t = self.advance()
        if t.kind != "num":
            self.error("expected a number")
        return float(t.text.rstrip("LlDdSsYy"))

    def parse_pivot(self, source):
        """``PIVOT (agg [AS a], … FOR col | (c1, c2) IN (v [AS x], (v1, v2) [AS x], …)) [alias]``
        (Spark 2.4 pivotClause; applies to the FROM clause's relation)."""
        self.advance()
        self.expect_op("(")
        aggs = []
        while True:
            e = self.parse_expr()
            alias = None
            if self.accept_kw("as"):
                alias = self.ident()
            elif self.cur.kind == "id" and not self.is_word("for"):
                alias = self.advance().text
            aggs.append((e, alias))
            if not self.accept_op(","):
                break
        if not self.accept_word("for"):
            self.error("expected FOR")
        if self.accept_op("("):
            cols = self._expr_list()
            self.expect_op(")")
        else:
            cols = [self.parse_postfix()]
        self.expect_kw("in")
        self.expect_op("(")
        values = []
        while True:
            if self.is_op("(") and len(cols) > 1:
                self.advance()
                vs = self._expr_list()
                self.expect_op(")")
            else:
                vs = [self.parse_expr()]
            if len(vs) != len(cols):
                self.error(f"PIVOT value has {len(vs)} parts for {len(cols)} column(s)")
            alias = None
            if self.accept_kw("as"):
                alias = self.ident()
            elif self.cur.kind == "id":
                alias = self.advance().text
            values.append((vs, alias))
            if not self.accept_op(","):
                break
        self.expect_op(")")
        self.expect_op(")")
        alias = None
        if self.accept_kw("as"):
            alias = self.ident()
        elif self._alias_word_ok():
            alias = self.advance().text
        return A.Pivot(source, aggs, cols, values, alias)

    # -- expressions ---------------------------------------------------------------------------------------------
    def parse_expr(self) -> A.Expr:
        return self.parse_or()

    def parse_or(self):
        e = self.parse_and()
        while self.accept_kw("or"):
            e = A.BinOp("or", e, self.parse_and())
        return e

    def parse_and(self):
        e = self.parse_not()
        while self.accept_kw("and") or self.accept_op("&&"):
            e = A.BinOp("and", e, self.parse_not())
        return e

    def parse_not(self):
        if self.accept_kw("not") or self.accept_op("!"):
            return A.UnaryOp("not", self.parse_not())
        return self.parse_predicate()

    def parse_predicate(self):
        e = self.parse_bitor()
        while True:
            if self.is_op("=", "==", "!=", "<>", "<", "<=", ">", ">=", "<=>"):
                op = self.advance().text
                op = {"==": "=", "<>": "!="}.get(op, op)
                e = A.BinOp(op, e, self.parse_bitor())
                continue
            neg = False
            save = self.i
            if self.accept_kw("not"):
                neg = True
            if self.accept_kw("in"):
                self.expect_op("(")
                if self._at_query():
                    q = self.parse_query()
                    self.expect_op(")")
                    e = A.SubqueryExpr("in", q, e, neg)
                    continue
                items = [self.parse_expr()]
                while self.accept_op(","):
                    items.append(self.parse_expr())
                self.expect_op(")")
                e = A.InList(e, items, neg)
                continue
            if self.accept_kw("between"):
                lo = self.parse_bitor()
                self.expect_kw("and")
                hi = self.parse_bitor()
                e = A.Between(e, lo, hi, neg)
                continue
            if self.accept_kw("like"):
                e = A.Like(e, self.parse_bitor(), neg, False)
                continue
            if self.accept_kw("rlike", "regexp"):
                e = A.Like(e, self.parse_bitor(), neg, True)
                continue
            if neg:
                self.i = save
                return e
            if self.accept_kw("is"):
                n = self.accept_kw("not")
                if self.accept_kw("null"):
                    e = A.IsNull(e, n)
                elif self.accept_kw("true"):
                    e = A.BinOp("<=>", e, A.Literal(True, "boolean"))
                    if n:
                        e = A.UnaryOp("not", e)
                elif self.accept_kw("false"):
                    e = A.BinOp("<=>", e, A.Literal(False, "boolean"))
                    if n:
                        e = A.UnaryOp("not", e)
                else:
                    self.error("expected NULL after IS")
                continue
            return e

    def parse_bitor(self):
        e = self.parse_bitxor()
        while self.is_op("|") and not self.is_op("||"):
            self.advance()
            e = A.BinOp("|", e, self.parse_bitxor())
        return e

    def parse_bitxor(self):
        e = self.parse_bitand()
        while self.accept_op("^"):
            e = A.BinOp("^", e, self.parse_bitand())
        return e

    def parse_bitand(self):
        e = self.parse_additive()
        while self.accept_op("&"):
            e = A.BinOp("&", e, self.parse_additive())
        return e

    def parse_additive(self):
        e = self.parse_mult()
        while self.is_op("+", "-", "||"):
            op = self.advance().text
            e = A.BinOp(op, e, self.parse_mult())
        return e

    def parse_mult(self):
        e = self.parse_unary()
        while self.is_op("*", "/", "%") or self.is_kw("div"):
            op = self.advance().text.lower()
            e = A.BinOp(op, e, self.parse_unary())
        return e

    def parse_unary(self):
        if self.is_op("-"):
            self.advance()
            operand = self.parse_unary()
            if isinstance(operand, A.Literal) and operand.integral:
                # Spark's grammar reads the minus into the literal (number: MINUS? INTEGER_VALUE), so the type is
                # that of the negative value: -2147483648 is an INT, -9223372036854775808 a BIGINT
                return _integer_literal(-int(operand.value))
            if isinstance(operand, A.Literal) and (operand.type in ("long", "int", "short", "byte", "double")
                                                   or str(operand.type).startswith("decimal(")):
                from ..engine.types import INT_RANGE
                if operand.type in INT_RANGE and not (INT_RANGE[operand.type][0] <= -operand.value
                                                      <= INT_RANGE[operand.type][1]):
                    self.error(f"numeric literal -{operand.value} does not fit in range of {operand.type}")
                return A.Literal(-operand.value, operand.type, suffixed=operand.suffixed)
            return A.UnaryOp("-", operand)
        if self.accept_op("+"):
            return self.parse_unary()
        if self.accept_op("~"):
            return A.UnaryOp("~", self.parse_unary())
        return self.parse_postfix()

    def parse_postfix(self):
        e = self.parse_primary()
        while True:
            if self.accept_op("["):
                idx = self.parse_expr()
                self.expect_op("]")
                e = A.Subscript(e, idx)
            elif self.is_op(".") and not isinstance(e, A.Ident):
                self.advance()
                name = self.ident()
                e = A.Subscript(e, A.Literal(name, "string"), dot=True)
            else:
                return e

    def parse_primary(self) -> A.Expr:
        t = self.cur
        if t.kind == "num":
            self.advance()
            return _number_literal(t.text)
        if t.kind == "str":
            self.advance()
            s = t.text
            # adjacent string literals concatenate
            while self.cur.kind == "str":
                s += self.advance().text
            return A.Literal(s, "string")
        if self.is_op("("):
            self.advance()
            if self._at_query():
                q = self.parse_query()
                self.expect_op(")")
                return A.SubqueryExpr("scalar", q)
            if self.cur.kind == "id" and self.is_op(",", tok=self.peek()):
                # (x, y) -> body: a multi-parameter lambda
                save = self.i
                params = [self.advance().text]
                while self.accept_op(","):
                    if self.cur.kind != "id":
                        break
                    params.append(self.advance().text)
                if self.accept_op(")") and self.is_op("-") and self.is_op(">", tok=self.peek()):
                    self.advance()
                    self.advance()
                    return A.Lambda(tuple(params), self.parse_expr())
                self.i = save
            e = self.parse_expr()
            self.expect_op(")")
            return e
        if t.kind == "id" and t.text.lower() == "exists" and self.is_op("(", tok=self.peek()):
            save = self.i
            self.advance()
            self.advance()
            if self._at_query():
                q = self.parse_query()
                self.expect_op(")")
                return A.SubqueryExpr("exists", q)
            self.i = save
        if t.kind == "id" and self.is_op("-", tok=self.peek()) and self.is_op(">", tok=self.peek(2)):
            self.advance()
            self.advance()
            self.advance()
            return A.Lambda((t.text,), self.parse_expr())
        if t.kind == "kw":
            w = t.text.lower()
            if w == "null":
                self.advance()
                return A.Literal(None, "null")
            if w in ("true", "false"):
                self.advance()
                return A.Literal(w == "true", "boolean")
            if w == "case":
                return self.parse_case()
            if w == "cast":
                self.advance()
                self.expect_op("(")
                e = self.parse_expr()
                self.expect_kw("as")
                ty = self.parse_type_name()
                self.expect_op(")")
                return A.Cast(e, ty)
            if w == "interval":
                self.advance()
                if self.cur.kind == "str":
                    return A.Interval(parse_duration_micros(self.advance().text))
                n = self.advance()
                unit = self.ident()
                return A.Interval(parse_duration_micros(f"{n.text} {unit}"))
            if w in ("left", "right", "first", "last") and self.is_op("(", tok=self.peek()):
                pass  # function named like a keyword
            elif w not in ("first", "last", "timewindow", "div", "regexp", "semi", "anti", "nulls"):
                self.error(f"unexpected keyword {t.text}")
        if t.kind in ("id", "kw") and t.text.lower() in ("timestamp", "date") and self.peek().kind == "str":
            # typed literal: TIMESTAMP '2020-01-01 00:00:00', DATE '2020-01-01'
            ty = self.advance().text.lower()
            return A.Cast(A.Literal(self.advance().text, "string"), ty, typed_literal=True)
        if t.kind in ("id", "kw"):
            name = self.advance().text
            if self.is_op("("):
                return self.parse_call(name)
            parts = [name]
            while self.is_op(".") and self.peek().kind in ("id", "kw") and not self.is_op("*", tok=self.peek()):
                self.advance()
                parts.append(self.advance().text)
            return A.Ident(tuple(parts))
        self.error("unexpected token")

    def parse_type_name(self) -> str:
        name = self.ident().lower()
        args = []
        if self.accept_op("("):
            depth = 1
            while depth:
                t = self.advance()
                if t.kind == "eof":
                    self.error("unterminated type")
                if self.is_op("(", tok=t):
                    depth += 1
                elif self.is_op(")", tok=t):
                    depth -= 1
                elif depth == 1 and t.kind == "num":
                    args.append(t.text)
        if name in ("decimal", "numeric", "dec"):
            from ..engine.decimal import DecimalType
            try:
                return DecimalType(*(int(a) for a in args[:2])) if args else DecimalType(10, 0)
            except ValueError:
                self.error(f"invalid decimal type {name}({', '.join(args)})")
        return {"integer": "int", "bigint": "long", "smallint": "short", "tinyint": "byte", "real": "float",
                "varchar": "string", "char": "string", "text": "string", "bool": "boolean",
                "numeric": "decimal", "dec": "decimal"}.get(name, name)

    def parse_case(self):
        self.expect_kw("case")
        operand = None
        if not self.is_kw("when"):
            operand = self.parse_expr()
        whens = []
        while self.accept_kw("when"):
            c = self.parse_expr()
            self.expect_kw("then")
            whens.append((c, self.parse_expr()))
        default = None
        if self.accept_kw("else"):
            default = self.parse_expr()
        self.expect_kw("end")
        return A.Case(operand, whens, default)

    def parse_call(self, name):
        self.expect_op("(")
        low = name.lower()
        if self.accept_op(")"):
            return self._maybe_over(A.Call(low, []))
        if self.is_op("*") and self.is_op(")", tok=self.peek()):
            self.advance()
            self.advance()
            return self._maybe_over(A.Call(low, [], star=True))
        if low == "extract" and self.peek().kind in ("id", "kw") and self.is_word("from", tok=self.peek()):
            # EXTRACT(field FROM source) → the field's function (Spark's Extract)
            field = self.advance().text.lower()
            self.advance()
            src = self.parse_expr()
            self.expect_op(")")
            fn = _EXTRACT_FIELDS.get(field)
            if fn is None:
                self.error(f"unknown EXTRACT field {field!r}")
            return A.Call(fn, [src])
        if low == "position":
            # POSITION(substr IN str) → locate(substr, str); the comma form falls through
            save = self.i
            sub = self.parse_bitor()
            if self.accept_kw("in"):
                src = self.parse_expr()
                self.expect_op(")")
                return A.Call("locate", [sub, src])
            self.i = save
        if low == "overlay":
            # OVERLAY(input PLACING replace FROM pos [FOR len])
            save = self.i
            inp = self.parse_expr()
            if self.accept_word("placing"):
                rep = self.parse_expr()
                if not self.accept_kw("from"):
                    self.error("expected FROM in OVERLAY")
                pos = self.parse_expr()
                args = [inp, rep, pos]
                if self.accept_word("for"):
                    args.append(self.parse_expr())
                self.expect_op(")")
                return A.Call("overlay", args)
            self.i = save
        distinct = self.accept_kw("distinct")
        args = [self._parse_call_arg()]
        while self.accept_op(","):
            args.append(self._parse_call_arg())
        self.expect_op(")")
        return self._maybe_over(A.Call(low, args, distinct=distinct))

    def _parse_call_arg(self):
        """A function argument; ``*`` and ``q.*`` (e.g. ``struct(*)``, ``to_json(struct(t.*))``) become Star nodes
        that the select list expands to the columns they name."""
        if self.is_op("*") and (self.is_op(",", tok=self.peek()) or self.is_op(")", tok=self.peek())):
            self.advance()
            return A.Star(())
        save = self.i
        quals = []
        while self.cur.kind in ("id", "qid") and self.is_op(".", tok=self.peek()):
            quals.append(self.advance().text)
            self.advance()
            if self.is_op("*"):
                self.advance()
                return A.Star(tuple(quals))
        self.i = save
        return self.parse_expr()

    def _at_query(self) -> bool:
        return self.is_kw("select") or (self.is_word("with") and self.peek().kind in ("id", "kw"))

    def is_word(self, *words, tok=None) -> bool:
        t = tok or self.cur
        return t.kind in ("id", "kw") and t.text.lower() in words

    def accept_word(self, *words) -> bool:
        if self.is_word(*words):
            self.i += 1
            return True
        return False

    def _maybe_over(self, call):
        """``call OVER (PARTITION BY ... ORDER BY ... frame)`` (Spark window functions); ``call OVER w`` names a
        window of the query's WINDOW clause."""
        if self.is_word("over") and self.peek().kind in ("id", "kw") and not self.is_op("(", tok=self.peek()):
            self.advance()
            return A.WindowCall(call, ref=self.ident())
        if not (self.is_word("over") and self.is_op("(", tok=self.peek())):
            return call
        self.advance()
        self.expect_op("(")
        part, order, frame = self._window_spec()
        return A.WindowCall(call, part, order, frame)

    def _window_spec(self):
        """The inside of ``( … )`` of a window: (partition, order, frame); consumes the closing parenthesis."""
        part, order, frame = [], [], None
        if self.accept_word("partition"):
            self.expect_kw("by")
            part.append(self.parse_expr())
            while self.accept_op(","):
                part.append(self.parse_expr())
        if self.is_kw("order") or self.is_word("sort"):
            self.advance()
            self.expect_kw("by")
            order = self.parse_order_items()
        if self.is_word("rows", "range"):
            kind = self.advance().text.lower()
            if self.accept_kw("between"):
                lo = self._frame_bound()
                self.expect_kw("and")
                hi = self._frame_bound()
            else:
                lo, hi = self._frame_bound(), ("current", 0)
            frame = (kind, lo, hi)
        self.expect_op(")")
        return part, order, frame

    def _frame_bound(self):
        if self.accept_word("unbounded"):
            if self.accept_word("preceding"):
                return ("unbounded_preceding", 0)
            if self.accept_word("following"):
                return ("unbounded_following", 0)
            self.error("expected PRECEDING or FOLLOWING")
        if self.accept_word("current"):
            if not self.accept_word("row"):
                self.error("expected ROW")
            return ("current", 0)
        if self.is_word("interval"):              # RANGE offsets over timestamps: INTERVAL '5' MINUTES → micros
            self.advance()
            if self.cur.kind == "str":
                k = parse_duration_micros(self.advance().text)
            else:
                n = self.advance()
                k = parse_duration_micros(f"{n.text} {self.ident()}")
        else:
            t = self.advance()
            if t.kind != "num":
                self.error("expected a frame offset")
            txt = t.text.rstrip("lLdD")
            k = float(txt) if any(c in txt for c in ".eE") else int(txt)
        if self.accept_word("preceding"):
            return ("preceding", k)
        if self.accept_word("following"):
            return ("following", k)
        self.error("expected PRECEDING or FOLLOWING")


_BROADCAST_HINTS = ("broadcast", "broadcastjoin", "mapjoin")
_KNOWN_HINTS = _BROADCAST_HINTS + ("merge", "shuffle_merge", "mergejoin", "shuffle_hash", "shuffle_replicate_nl",
                                   "coalesce", "repartition", "repartition_by_range")
_HINT_RE = re.compile(r"\s*([A-Za-z_][A-Za-z0-9_]*)\s*(?:\(([^)]*)\))?\s*,?")


def _parse_hints(text: str):
    """``/*+ BROADCAST(a, b) COALESCE(3) */`` → [("broadcast", ["a", "b"]), ("coalesce", ["3"])].  Join-strategy
    hints steer the distributed join (BROADCAST replicates the named relation instead of co-partitioning both
    sides); the others are accepted and ignored, as Spark ignores hints it cannot apply; an unparsable hint body is
    ignored with it (Spark logs a warning)."""
    out, pos = [], 0
    text = text.strip()
    while pos < len(text):
        m = _HINT_RE.match(text, pos)
        if not m or m.end() == pos:
            return out
        args = [a.strip().strip("`") for a in (m.group(2) or "").split(",") if a.strip()]
        out.append((m.group(1).lower(), args))
        pos = m.end()
    return out


def _mark_broadcast(rel, names):
    if isinstance(rel, A.Join):
        rel.broadcast = set(names) | set(getattr(rel, "broadcast", ()) or ())
        _mark_broadcast(rel.left, names)
        _mark_broadcast(rel.right, names)
    elif isinstance(rel, (A.LateralView, A.Pivot)):
        _mark_broadcast(rel.source, names)


def _rollup(cols):
    return [cols[:k] for k in range(len(cols), -1, -1)]


def _cube(cols):
    n = len(cols)
    sets = []
    for mask in range((1 << n) - 1, -1, -1):
        sets.append([c for i, c in enumerate(cols) if mask >> (n - 1 - i) & 1])
    return sets


def _number_literal(text: str) -> A.Literal:
    up = text.upper()
    if up.endswith("BD"):
        from ..engine.decimal import literal_type
        import decimal as _pd
        t = literal_type(text[:-2])
        if t is None:
            raise SqlError(f"decimal literal {text} exceeds 38 digits")
        return A.Literal(_pd.Decimal(text[:-2]), t)
    suffix = up[-1]
    if suffix in "LSY":
        # 10L BIGINT, 10S SMALLINT, 10Y TINYINT (Spark: a value outside the type's range is a parse error)
        from ..engine.types import INT_RANGE
        t = {"L": "long", "S": "short", "Y": "byte"}[suffix]
        v = int(text[:-1])
        if not (INT_RANGE[t][0] <= v <= INT_RANGE[t][1] + 1):     # +1: the minus sign folds in afterwards
            raise SqlError(f"numeric literal {text} does not fit in range of {t}")
        return A.Literal(v, t, suffixed=True)
    if suffix == "D":
        return A.Literal(float(text[:-1]), "double", suffixed=True)
    if "." in text or "e" in text.lower():
        # Spark 2.4: an unsuffixed fractional or exponent literal (DECIMAL_VALUE) is an exact decimal of its own
        # digits, BigDecimal(text); 1e20 is 10^20 as decimal(21,0) (Spark's decimal(1,-20) holds the same value);
        # over 38 digits it is a double.  (Exponent literals became doubles only in Spark 3.0, SPARK-29956.)
        from ..engine.decimal import literal_type
        import decimal as _pd
        t = literal_type(text)
        if t is None:
            return A.Literal(float(text), "double")
        v = _pd.Decimal(text)
        return A.Literal(v if t.scale else _pd.Decimal(int(v)), t)
    return _integer_literal(int(text))


def _integer_literal(v: int) -> A.Literal:
    """Spark's visitIntegerLiteral: INT when the value fits, else BIGINT, else decimal(digits, 0)."""
    if -2**31 <= v < 2**31:
        return A.Literal(v, "int", integral=True)
    if -2**63 <= v < 2**63:
        return A.Literal(v, "long", integral=True)
    from ..engine.decimal import DecimalType
    import decimal as _pd
    nd = len(str(abs(v)))
    if nd > 38:
        return A.Literal(float(v), "double")
    return A.Literal(_pd.Decimal(v), DecimalType(nd, 0), integral=True)


def parse_query(sql: str) -> A.Query:
    p = Parser(sql.strip().rstrip(";"))
    q = p.parse_query()
    if p.cur.kind != "eof":
        p.error("unexpected trailing input")
    return q


def parse_expression(sql: str) -> A.Expr:
    p = Parser(sql)
    e = p.parse_expr()
    if p.cur.kind != "eof":
        p.error("unexpected trailing input")
    return e


def parse_select_item(sql: str) -> A.SelectItem:
    """One projection line (reference projection files hold one ``selectExpr`` per line,
    DataProcessing/datax-host/src/main/scala/datax/handler/ProjectionHandler.scala:23-36)."""
    p = Parser(sql)
    it = p.parse_select_item()
    if p.cur.kind != "eof":
        p.error("unexpected trailing input")
    return it
