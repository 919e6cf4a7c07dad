"""Array built-ins as slot-matrix tensor operations (dxa/engine/arrayfuncs.py) against the row-wise host functions
(the oracle, ``arrayfuncs.rowwise()``) and hand-computed Spark 2.4 results; on the GPU over 1 M rows in < 10 ms."""
import random
import time

import pytest
import torch

from dxa.engine import arrayfuncs
from dxa.engine.column import Table
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql
from dxa.engine.types import StructField, StructType

S = StructType((StructField("g", "long"), StructField("v", "long"), StructField("w", "long"),
                StructField("s", "string"), StructField("d", "double")))
BASE = ("WITH A AS (SELECT g, collect_list(v) a, collect_list(w) b, collect_list(s) s, collect_list(d) d "
        "FROM T GROUP BY g) ")
EXPRS = ["array_max(a)", "array_min(a)", "array_position(a, 2)", "sort_array(a)", "sort_array(a, false)",
         "array_sort(a)", "array_distinct(a)", "slice(a, 2, 2)", "slice(a, -2, 5)", "array_union(a, b)",
         "array_intersect(a, b)", "array_except(a, b)", "array_distinct(s)", "array_position(s, 'y')",
         "array_max(d)", "array_min(d)", "sort_array(d)", "array_join(s, '-')", "array_union(s, s)",
         "array_except(s, array('x'))", "array_remove(a, 3)", "array_remove(s, 'x')", "arrays_overlap(a, b)"]


def _table(rows, device):
    cat = Catalog()
    cat.register("T", Table.from_pylist([dict(zip("gvwsd", r)) for r in rows], S, device))
    return cat


def _eval(rows, device, exprs=EXPRS):
    sql = BASE + "SELECT g, " + ", ".join(f"{e} AS c{i}" for i, e in enumerate(exprs)) + " FROM A ORDER BY g"
    return run_sql(sql, _table(rows, device), EvalContext(device=torch.device(device))).to_pylist()


ROWS = [(1, 3, 2, "x", 1.5), (1, 1, 5, "y", float("nan")), (1, 2, None, "x", -2.0), (1, 3, None, None, None),
        (1, 1, None, None, None), (2, 7, None, "q", 0.0), (3, None, 1, None, None)]


def _same(a, b):
    import math
    if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
        return True
    if isinstance(a, list) and isinstance(b, list):
        return len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, dict) and isinstance(b, dict):
        return a.keys() == b.keys() and all(_same(a[k], b[k]) for k in a)
    return a == b


def test_hand_computed_cpu():
    got = _eval(ROWS, "cpu")
    r1 = got[0]
    assert r1["c3"] == [1, 1, 2, 3, 3] and r1["c4"] == [3, 3, 2, 1, 1] and r1["c6"] == [3, 1, 2]
    assert r1["c7"] == [1, 2] and r1["c8"] == [3, 1] and r1["c9"] == [3, 1, 2, 5]
    assert r1["c10"] == [2] and r1["c11"] == [3, 1] and r1["c12"] == ["x", "y"] and r1["c13"] == 2
    assert r1["c2"] == 3 and r1["c17"] == "x-y-x" and r1["c19"] == ["y"]
    assert got[1]["c7"] == [] and got[1]["c8"] == []           # slice past the end / before the start: empty
    assert got[2]["c0"] is None and got[2]["c2"] == 0          # empty array: max null, position 0
    with pytest.raises(Exception, match="start at 1"):
        _eval(ROWS, "cpu", ["slice(a, 0, 1)"])


def test_matches_rowwise_cpu():
    rnd = random.Random(3)
    rows = [(rnd.randrange(200), rnd.choice([None, rnd.randrange(12)]), rnd.choice([None, rnd.randrange(12)]),
             rnd.choice([None, "x", "y", "zz", ""]), rnd.choice([None, rnd.uniform(-5, 5), float("nan")]))
            for _ in range(3000)]
    fast = _eval(rows, "cpu")
    with arrayfuncs.rowwise():
        slow = _eval(rows, "cpu")
    assert all(_same(a, b) for a, b in zip(fast, slow))


@pytest.mark.gpu
def test_gpu_matches_rowwise_and_is_fast(gpu):
    rnd = random.Random(5)
    rows = [(rnd.randrange(2000), rnd.choice([None, rnd.randrange(12)]), rnd.choice([None, rnd.randrange(12)]),
             rnd.choice([None, "x", "y", "zz", ""]), rnd.choice([None, rnd.uniform(-5, 5), float("nan")]))
            for _ in range(20000)]
    # build the arrays once: collect_list's element order on the GPU is whatever the atomics produced, so two
    # group-bys may order elements differently; both evaluators then run over the same arrays
    cat = _table(rows, gpu)
    cat.register("A", run_sql(BASE[len("WITH A AS ("):-2], cat, EvalContext(device=gpu)))
    sql = "SELECT g, " + ", ".join(f"{e} AS c{i}" for i, e in enumerate(EXPRS)) + " FROM A ORDER BY g"
    dev = run_sql(sql, cat, EvalContext(device=gpu)).to_pylist()
    with arrayfuncs.rowwise():
        host = run_sql(sql, cat, EvalContext(device=gpu)).to_pylist()
    bad = [(EXPRS[int(k[1:])], a[k], b[k]) for a, b in zip(dev, host) for k in a if k != "g" and not _same(a[k], b[k])]
    assert not bad, bad[:5]
    # 1 M arrays of up to 8 elements, one function at a time
    n = 1_000_000
    g = torch.arange(n * 8, device=gpu) // 8
    vals = torch.randint(0, 20, (n * 8,), device=gpu)
    from dxa.engine.column import PrimColumn
    t = Table(["g", "v", "w"], [PrimColumn("long", g), PrimColumn("long", vals),
                                PrimColumn("long", torch.flip(vals, [0]))], n * 8, gpu)
    cat = Catalog()
    cat.register("T", t)
    arrs = run_sql("SELECT g, collect_list(v) a, collect_list(w) b FROM T GROUP BY g", cat, EvalContext(device=gpu))
    cat.register("A", arrs)
    from dxa.engine.expr import Scope, evaluate
    from dxa.sql.parser import parse_expression
    sc = Scope.of_table(arrs)
    for expr in ["array_max(a)", "array_position(a, 3)", "sort_array(a)", "array_distinct(a)", "slice(a, 2, 3)",
                 "array_union(a, b)", "array_intersect(a, b)", "array_except(a, b)"]:
        e = parse_expression(expr)
        evaluate(e, sc, EvalContext(device=gpu))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        col = evaluate(e, sc, EvalContext(device=gpu))
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        assert col.length == arrs.length
        assert ms < 10.0, f"{expr}: {ms:.2f} ms for 1M arrays"
