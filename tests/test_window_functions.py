"""SQL window functions (``OVER``): hand-computed Spark results plus a brute-force row-by-row reference over random
data (partitions, ties, nulls, ROWS/RANGE frames)."""
import json
import random

import pytest

from dxa.engine.column import Table
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, QueryError, run_sql
from dxa.engine.serialize import table_to_json_lines
from dxa.engine.types import StructField, StructType

SCHEMA = StructType((StructField("id", "long"), StructField("k", "string"), StructField("t", "long"),
                     StructField("v", "double")))


def _cat(rows):
    c = Catalog()
    c.register("T", Table.from_pylist(rows, SCHEMA))
    return c


def q(cat, sql):
    return [json.loads(l) for l in table_to_json_lines(run_sql(sql, cat, EvalContext(now_us=0)))]


ROWS = [
    {"id": 1, "k": "a", "t": 10, "v": 1.0},
    {"id": 2, "k": "a", "t": 20, "v": 2.0},
    {"id": 3, "k": "a", "t": 20, "v": None},
    {"id": 4, "k": "a", "t": 30, "v": 4.0},
    {"id": 5, "k": "b", "t": 5, "v": 10.0},
    {"id": 6, "k": "b", "t": None, "v": 20.0},
    {"id": 7, "k": None, "t": 1, "v": 7.0},
]


def test_ranking_functions():
    got = q(_cat(ROWS), "SELECT id, row_number() OVER (PARTITION BY k ORDER BY t) AS rn, "
                        "rank() OVER (PARTITION BY k ORDER BY t) AS rk, "
                        "dense_rank() OVER (PARTITION BY k ORDER BY t) AS dr FROM T ORDER BY id")
    rn = {r["id"]: (r["rn"], r["rk"], r["dr"]) for r in got}
    # partition a: t=10 → 1; t=20 tie → rows 2,3 (row_number 2/3, rank 2, dense 2); t=30 → rn 4, rank 4, dense 3
    assert rn[1] == (1, 1, 1)
    assert {rn[2][0], rn[3][0]} == {2, 3} and rn[2][1:] == (2, 2) and rn[3][1:] == (2, 2)
    assert rn[4] == (4, 4, 3)
    # partition b: NULL t sorts first ascending
    assert rn[6] == (1, 1, 1) and rn[5] == (2, 2, 2)
    assert rn[7] == (1, 1, 1)


def test_running_and_whole_partition_aggregates():
    got = q(_cat(ROWS), "SELECT id, sum(v) OVER (PARTITION BY k ORDER BY t) AS run, "
                        "sum(v) OVER (PARTITION BY k) AS tot, count(v) OVER (PARTITION BY k) AS nv, "
                        "count(*) OVER () AS n_all, avg(v) OVER (PARTITION BY k ORDER BY t) AS ravg FROM T ORDER BY id")
    by = {r["id"]: r for r in got}
    # RANGE UNBOUNDED PRECEDING..CURRENT ROW: ties (t=20) share the running total
    assert [by[i]["run"] for i in (1, 2, 3, 4)] == [1.0, 3.0, 3.0, 7.0]
    assert all(by[i]["tot"] == 7.0 and by[i]["nv"] == 3 for i in (1, 2, 3, 4))
    assert by[6]["run"] == 20.0 and by[5]["run"] == 30.0
    assert all(r["n_all"] == 7 for r in got)
    assert by[2]["ravg"] == 1.5


def test_lag_lead_first_last():
    got = q(_cat(ROWS), "SELECT id, lag(v) OVER (PARTITION BY k ORDER BY id) AS pv, "
                        "lead(v, 2, -1.0) OVER (PARTITION BY k ORDER BY id) AS n2, "
                        "first_value(v) OVER (PARTITION BY k ORDER BY id) AS fv, "
                        "last_value(id) OVER (PARTITION BY k ORDER BY id ROWS BETWEEN UNBOUNDED PRECEDING AND "
                        "UNBOUNDED FOLLOWING) AS lid FROM T ORDER BY id")
    by = {r["id"]: r for r in got}
    assert "pv" not in by[1] and by[2]["pv"] == 1.0 and by[4].get("pv") is None   # id3's v is NULL
    assert by[2]["n2"] == 4.0 and by[3]["n2"] == -1.0 and by[4]["n2"] == -1.0
    assert "n2" not in by[1]                   # lead 2 of id1 is id3 whose v is NULL (default only off the end)
    assert all(by[i]["fv"] == 1.0 for i in (1, 2, 3, 4))
    assert by[1]["lid"] == 4 and by[5]["lid"] == 6 and by[7]["lid"] == 7


def test_sliding_rows_frame_min_max():
    got = q(_cat(ROWS), "SELECT id, min(v) OVER (PARTITION BY k ORDER BY id ROWS BETWEEN 1 PRECEDING AND 1 FOLLOWING)"
                        " AS mn, max(v) OVER (PARTITION BY k ORDER BY id ROWS 1 PRECEDING) AS mx FROM T ORDER BY id")
    by = {r["id"]: r for r in got}
    assert [by[i]["mn"] for i in (1, 2, 3, 4)] == [1.0, 1.0, 2.0, 4.0]
    assert [by[i]["mx"] for i in (1, 2, 3, 4)] == [1.0, 2.0, 2.0, 4.0]


def test_ntile_percent_rank_cume_dist():
    rows = [{"id": i, "k": "a", "t": i, "v": float(i)} for i in range(1, 8)]
    got = q(_cat(rows), "SELECT id, ntile(3) OVER (ORDER BY t) AS nt, percent_rank() OVER (ORDER BY t) AS pr, "
                        "cume_dist() OVER (ORDER BY t) AS cd FROM T ORDER BY id")
    assert [r["nt"] for r in got] == [1, 1, 1, 2, 2, 3, 3]
    assert [r["pr"] for r in got] == [i / 6 for i in range(7)]
    assert [r["cd"] for r in got] == [i / 7 for i in range(1, 8)]


def test_window_over_grouped_rows_and_having():
    got = q(_cat(ROWS), "SELECT k, sum(v) AS s, rank() OVER (ORDER BY sum(v) DESC) AS r FROM T "
                        "GROUP BY k HAVING count(*) > 1 ORDER BY r")
    assert got == [{"k": "b", "s": 30.0, "r": 1}, {"k": "a", "s": 7.0, "r": 2}]


def test_unsupported_window_function():
    with pytest.raises(QueryError):
        q(_cat(ROWS), "SELECT upper(k) OVER () AS x FROM T")


# -- brute-force reference ------------------------------------------------------------------------------------------

def _ref_window(rows, func, arg, part, order_desc, frame):
    """Row-by-row reference: partition by ``part``, order by (t, id) with nulls first (asc) / last (desc)."""
    def okey(r):
        t = r["t"]
        if order_desc:
            return (t is None, -(t or 0), -r["id"])
        return (t is not None, t or 0, r["id"])
    out = {}
    groups = {}
    for r in rows:
        groups.setdefault(r[part], []).append(r)
    for g in groups.values():
        g = sorted(g, key=okey)
        n = len(g)
        for i, r in enumerate(g):
            if frame is None:
                lo, hi = 0, n - 1
            else:
                lo, hi = max(0, i - frame[0]), min(n - 1, i + frame[1])
            vals = [x[arg] for x in g[lo:hi + 1] if x[arg] is not None] if lo <= hi else []
            if func == "row_number":
                out[r["id"]] = i + 1
            elif func == "sum":
                out[r["id"]] = sum(vals) if vals else None
            elif func == "count":
                out[r["id"]] = len(vals)
            elif func == "min":
                out[r["id"]] = min(vals) if vals else None
            elif func == "max":
                out[r["id"]] = max(vals) if vals else None
            elif func == "lag":
                out[r["id"]] = g[i - 1][arg] if i >= 1 else None
    return out


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("func", ["row_number", "sum", "count", "min", "max", "lag"])
def test_random_vs_bruteforce(seed, func):
    rnd = random.Random(seed)
    rows = []
    for i in range(300):
        rows.append({"id": i, "k": rnd.choice(["p", "q", "r", None]),
                     "t": rnd.choice([None] + list(range(20))),
                     "v": None if rnd.random() < 0.15 else float(rnd.randint(-50, 50))})
    cat = _cat(rows)
    desc = seed % 2 == 1
    frame = None if func in ("row_number", "lag") else (rnd.randint(0, 4), rnd.randint(0, 4))
    frame_sql = "" if frame is None else f" ROWS BETWEEN {frame[0]} PRECEDING AND {frame[1]} FOLLOWING"
    d = " DESC" if desc else ""
    call = {"row_number": "row_number()", "lag": "lag(v)"}.get(func, f"{func}(v)")
    got = q(cat, f"SELECT id, {call} OVER (PARTITION BY k ORDER BY t{d}, id{d}{frame_sql}) AS w FROM T")
    ref = _ref_window(rows, func, "v", "k", desc, frame)
    for r in got:
        assert r.get("w") == ref[r["id"]], (r, ref[r["id"]])


@pytest.mark.gpu
def test_window_functions_gpu_match_cpu():
    import torch
    assert torch.cuda.is_available()
    rnd = random.Random(7)
    rows = [{"id": i, "k": rnd.choice(["p", "q", "r", None]), "t": rnd.choice([None] + list(range(50))),
             "v": None if rnd.random() < 0.1 else float(rnd.randint(-500, 500))} for i in range(20000)]
    sql = ("SELECT id, row_number() OVER (PARTITION BY k ORDER BY t, id) AS rn, rank() OVER (PARTITION BY k ORDER BY t) "
           "AS rk, sum(v) OVER (PARTITION BY k ORDER BY t) AS run, min(v) OVER (PARTITION BY k ORDER BY id ROWS "
           "BETWEEN 3 PRECEDING AND 2 FOLLOWING) AS mn, lag(v, 2) OVER (PARTITION BY k ORDER BY id) AS lg, "
           "max(v) OVER (PARTITION BY k ORDER BY t DESC RANGE BETWEEN 4 PRECEDING AND 1 FOLLOWING) AS rg FROM T "
           "ORDER BY id")
    out = {}
    for dev in ("cpu", "cuda"):
        c = Catalog()
        c.register("T", Table.from_pylist(rows, SCHEMA, dev))
        out[dev] = [json.loads(l) for l in table_to_json_lines(run_sql(sql, c, EvalContext(now_us=0)))]
    assert out["cpu"] == out["cuda"]


def _brute_range(rows, lo, hi, desc=False, func="sum"):
    """RANGE BETWEEN lo AND hi (offsets, None = unbounded) over ORDER BY t per k, in Spark's terms: rows are placed
    on the ordering axis (s·t, nulls at -inf for ASC NULLS FIRST / +inf for DESC NULLS LAST); an unbounded side
    reaches the partition's end, an offset side is the current row's position + offset (a null row's own position)."""
    inf = float("inf")
    s = -1 if desc else 1

    def ov(x):
        return (inf if desc else -inf) if x["t"] is None else s * x["t"]
    out = {}
    for r in rows:
        peers = [x for x in rows if x["k"] == r["k"]]
        c = ov(r)
        lower = -inf if lo is None else (c if r["t"] is None else c + lo)
        upper = inf if hi is None else (c if r["t"] is None else c + hi)
        frame = [x for x in peers if lower <= ov(x) <= upper]
        vals = [x["v"] for x in frame if x["v"] is not None]
        if func == "sum":
            out[r["id"]] = sum(vals) if vals else None
        elif func == "count":
            out[r["id"]] = len(vals)
        else:
            out[r["id"]] = max(vals) if vals else None
    return out


@pytest.mark.parametrize("desc", [False, True])
def test_range_frames_with_value_offsets(desc):
    """RANGE frames with numeric offsets (Spark: one ORDER BY expression; frame = rows whose ORDER BY value lies
    within [v - lo, v + hi]; a null key's frame is its null peers) against a row-by-row reference."""
    rnd = random.Random(5)
    rows = [{"id": i, "k": rnd.choice(["a", "b", None]), "t": None if rnd.random() < 0.1 else rnd.randint(0, 40),
             "v": None if rnd.random() < 0.1 else float(rnd.randint(-5, 9))} for i in range(300)]
    cat = _cat(rows)
    d = " DESC" if desc else ""
    for lo_sql, hi_sql, lo, hi in (("5 PRECEDING", "CURRENT ROW", -5, 0), ("3 PRECEDING", "2 FOLLOWING", -3, 2),
                                   ("UNBOUNDED PRECEDING", "4 PRECEDING", None, -4),
                                   ("2 FOLLOWING", "UNBOUNDED FOLLOWING", 2, None)):
        for func in ("sum", "count", "max"):
            got = q(cat, f"SELECT id, {func}(v) OVER (PARTITION BY k ORDER BY t{d} RANGE BETWEEN {lo_sql} AND "
                         f"{hi_sql}) AS x FROM T")
            want = _brute_range(rows, lo, hi, desc, func)
            assert {g["id"]: g.get("x") for g in got} == want, (lo_sql, hi_sql, func)


def test_range_interval_offsets_over_timestamps():
    from dxa.engine.column import column_from_pylist
    c = Catalog()
    h = 3_600_000_000
    c.register("E", Table(["ts", "x"], [column_from_pylist([0, h // 2, h, 3 * h, 3 * h + 1], "timestamp"),
                                        column_from_pylist([1, 2, 3, 4, 5], "long")]))
    got = q(c, "SELECT x, sum(x) OVER (ORDER BY ts RANGE BETWEEN INTERVAL 1 HOUR PRECEDING AND CURRENT ROW) AS s "
               "FROM E")
    assert [(g["x"], g["s"]) for g in got] == [(1, 1), (2, 3), (3, 6), (4, 4), (5, 9)]
    with pytest.raises(Exception):
        q(c, "SELECT sum(x) OVER (ORDER BY ts, x RANGE BETWEEN 1 PRECEDING AND CURRENT ROW) AS s FROM E")


def test_lag_lead_generated_names_spark24():
    """Un-aliased lag / lead columns are named as Spark 2.4 names them: the defaulted offset and default printed
    (``lag(v, 1, NULL)``) and the frame from OffsetWindowFunction — lag's boundary is the folded literal -offset,
    printed by boundarySql as ``-1 FOLLOWING`` (a computed expression, not a literal, from the reference's Spark;
    parity unpinned by any reference fixture)."""
    out = run_sql("SELECT lag(v) OVER (PARTITION BY k ORDER BY id), lead(v) OVER (ORDER BY id), "
                  "lag(v, 2, 0) OVER (ORDER BY id) FROM T", _cat(ROWS), EvalContext())
    assert out.names == [
        "lag(v, 1, NULL) OVER (PARTITION BY k ORDER BY id ASC NULLS FIRST ROWS BETWEEN -1 FOLLOWING AND -1 FOLLOWING)",
        "lead(v, 1, NULL) OVER (ORDER BY id ASC NULLS FIRST ROWS BETWEEN 1 FOLLOWING AND 1 FOLLOWING)",
        "lag(v, 2, 0) OVER (ORDER BY id ASC NULLS FIRST ROWS BETWEEN -2 FOLLOWING AND -2 FOLLOWING)"]
