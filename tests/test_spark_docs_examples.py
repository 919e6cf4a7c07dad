"""Window functions, frames, ``window()`` and aggregates pinned to Spark's own documented examples — not to this
engine's CPU evaluator.  The ``employees`` table and the expected result tables are the ones printed in the Spark SQL
reference (sql-ref-syntax-qry-select-window: RANK / DENSE_RANK / CUME_DIST / MIN OVER / LAG / LEAD); the frame,
``window()`` and aggregate expectations are hand-computed from the documented semantics (RANGE frames are value
ranges over the ORDER BY key; ``window(ts, d, s)`` buckets are aligned to the epoch, [start, end)).  The user SQL
the reference runs goes through Spark 2.4 (CommonProcessorFactory.scala:257-275)."""
import datetime as dt

import pytest
import torch

from dxa.engine.column import Table
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql
from dxa.engine.types import StructField, StructType

EMP = StructType((StructField("name", "string"), StructField("dept", "string"), StructField("salary", "int"),
                  StructField("age", "int")))
EMPLOYEES = [("Lisa", "Sales", 10000, 35), ("Evan", "Sales", 32000, 38), ("Fred", "Engineering", 21000, 28),
             ("Alex", "Sales", 30000, 33), ("Tom", "Engineering", 23000, 33), ("Jane", "Marketing", 29000, 28),
             ("Jeff", "Marketing", 35000, 38), ("Paul", "Engineering", 29000, 23),
             ("Chloe", "Engineering", 23000, 25)]


def _q(sql, device="cpu"):
    cat = Catalog()
    cat.register("employees", Table.from_pylist([dict(zip(("name", "dept", "salary", "age"), r)) for r in EMPLOYEES],
                                                EMP, device))
    return run_sql(sql, cat, EvalContext(device=torch.device(device))).to_pylist()


def _by_name(rows, col):
    return {r["name"]: r[col] for r in rows}


DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("device", DEVICES)
def test_rank(device):
    got = _q("SELECT name, dept, salary, RANK() OVER (PARTITION BY dept ORDER BY salary) AS rank FROM employees",
             device)
    assert _by_name(got, "rank") == {"Lisa": 1, "Alex": 2, "Evan": 3, "Fred": 1, "Tom": 2, "Chloe": 2, "Paul": 4,
                                     "Jane": 1, "Jeff": 2}


@pytest.mark.parametrize("device", DEVICES)
def test_dense_rank(device):
    got = _q("SELECT name, DENSE_RANK() OVER (PARTITION BY dept ORDER BY salary ROWS BETWEEN UNBOUNDED PRECEDING "
             "AND CURRENT ROW) AS dense_rank FROM employees", device)
    assert _by_name(got, "dense_rank") == {"Lisa": 1, "Alex": 2, "Evan": 3, "Fred": 1, "Tom": 2, "Chloe": 2,
                                           "Paul": 3, "Jane": 1, "Jeff": 2}


@pytest.mark.parametrize("device", DEVICES)
def test_cume_dist(device):
    got = _q("SELECT name, CUME_DIST() OVER (PARTITION BY dept ORDER BY age RANGE BETWEEN UNBOUNDED PRECEDING AND "
             "CURRENT ROW) AS cume_dist FROM employees", device)
    exp = {"Alex": 1 / 3, "Lisa": 2 / 3, "Evan": 1.0, "Paul": 0.25, "Chloe": 0.5, "Fred": 0.75, "Tom": 1.0,
           "Jane": 0.5, "Jeff": 1.0}
    assert _by_name(got, "cume_dist") == pytest.approx(exp, rel=1e-15)


@pytest.mark.parametrize("device", DEVICES)
def test_min_over_default_frame(device):
    got = _q("SELECT name, MIN(salary) OVER (PARTITION BY dept ORDER BY salary) AS min FROM employees", device)
    assert _by_name(got, "min") == {"Lisa": 10000, "Alex": 10000, "Evan": 10000, "Paul": 21000, "Tom": 21000,
                                    "Fred": 21000, "Chloe": 21000, "Jane": 29000, "Jeff": 29000}


@pytest.mark.parametrize("device", DEVICES)
def test_lag_lead(device):
    got = _q("SELECT name, LAG(salary) OVER (PARTITION BY dept ORDER BY salary) AS lag, "
             "LEAD(salary, 1, 0) OVER (PARTITION BY dept ORDER BY salary) AS lead FROM employees", device)
    lag, lead = _by_name(got, "lag"), _by_name(got, "lead")
    # Tom and Chloe tie on salary (their relative order is unspecified in Spark too): check the rest exactly
    assert {k: lag[k] for k in ("Lisa", "Alex", "Evan", "Fred", "Paul", "Jane", "Jeff")} == \
        {"Lisa": None, "Alex": 10000, "Evan": 30000, "Fred": None, "Paul": 23000, "Jane": None, "Jeff": 29000}
    assert {k: lead[k] for k in ("Lisa", "Alex", "Evan", "Fred", "Paul", "Jane", "Jeff")} == \
        {"Lisa": 30000, "Alex": 32000, "Evan": 0, "Fred": 23000, "Paul": 0, "Jane": 35000, "Jeff": 0}
    assert sorted([lag["Tom"], lag["Chloe"]]) == [21000, 23000]
    assert sorted([lead["Tom"], lead["Chloe"]]) == [23000, 29000]


@pytest.mark.parametrize("device", DEVICES)
def test_range_and_rows_frames(device):
    got = _q("SELECT name, "
             "SUM(salary) OVER (PARTITION BY dept ORDER BY salary RANGE BETWEEN 2000 PRECEDING AND CURRENT ROW) AS r, "
             "SUM(salary) OVER (PARTITION BY dept ORDER BY salary, name ROWS BETWEEN 1 PRECEDING AND 1 FOLLOWING) "
             "AS w, COUNT(*) OVER (PARTITION BY dept) AS c, "
             "MAX(age) OVER (PARTITION BY dept ORDER BY salary RANGE BETWEEN CURRENT ROW AND UNBOUNDED FOLLOWING) "
             "AS m FROM employees", device)
    # RANGE 2000 PRECEDING: every row whose salary is in [salary - 2000, salary] (ties included)
    assert _by_name(got, "r") == {"Lisa": 10000, "Alex": 30000, "Evan": 62000, "Fred": 21000, "Tom": 67000,
                                  "Chloe": 67000, "Paul": 29000, "Jane": 29000, "Jeff": 35000}
    # ROWS 1 PRECEDING .. 1 FOLLOWING over (salary, name): Engineering = Fred 21000, Chloe 23000, Tom 23000,
    # Paul 29000
    assert _by_name(got, "w") == {"Lisa": 40000, "Alex": 72000, "Evan": 62000, "Fred": 44000, "Chloe": 67000,
                                  "Tom": 75000, "Paul": 52000, "Jane": 64000, "Jeff": 64000}
    assert _by_name(got, "c") == {"Lisa": 3, "Alex": 3, "Evan": 3, "Fred": 4, "Tom": 4, "Chloe": 4, "Paul": 4,
                                  "Jane": 2, "Jeff": 2}
    # CURRENT ROW .. UNBOUNDED FOLLOWING in value order: the peers of the current row are included
    assert _by_name(got, "m") == {"Lisa": 38, "Alex": 38, "Evan": 38, "Fred": 33, "Tom": 33, "Chloe": 33,
                                  "Paul": 23, "Jane": 38, "Jeff": 38}


@pytest.mark.parametrize("device", DEVICES)
def test_ntile_percent_rank_row_number(device):
    got = _q("SELECT name, NTILE(2) OVER (PARTITION BY dept ORDER BY salary, name) AS nt, "
             "PERCENT_RANK() OVER (PARTITION BY dept ORDER BY salary) AS pr, "
             "ROW_NUMBER() OVER (PARTITION BY dept ORDER BY salary, name) AS rn FROM employees", device)
    # NTILE(2) of 4 rows → 1,1,2,2; of 3 rows → 1,1,2; of 2 rows → 1,2
    assert _by_name(got, "nt") == {"Fred": 1, "Chloe": 1, "Tom": 2, "Paul": 2, "Lisa": 1, "Alex": 1, "Evan": 2,
                                   "Jane": 1, "Jeff": 2}
    # (rank - 1) / (rows - 1)
    assert _by_name(got, "pr") == pytest.approx({"Fred": 0.0, "Chloe": 1 / 3, "Tom": 1 / 3, "Paul": 1.0,
                                                 "Lisa": 0.0, "Alex": 0.5, "Evan": 1.0, "Jane": 0.0, "Jeff": 1.0})
    assert _by_name(got, "rn") == {"Fred": 1, "Chloe": 2, "Tom": 3, "Paul": 4, "Lisa": 1, "Alex": 2, "Evan": 3,
                                   "Jane": 1, "Jeff": 2}


TS = StructType((StructField("ts", "timestamp"), StructField("v", "long")))


def _ts_rows():
    base = dt.datetime(2024, 1, 1, 12, 0, 0)
    return [{"ts": base + dt.timedelta(minutes=m), "v": v} for m, v in ((0, 1), (3, 2), (7, 3), (12, 4), (14, 5))]


@pytest.mark.parametrize("device", DEVICES)
def test_window_function_tumbling_and_sliding(device):
    cat = Catalog()
    cat.register("T", Table.from_pylist(_ts_rows(), TS, device))
    ctx = EvalContext(device=torch.device(device))
    tumble = run_sql("SELECT window.start AS s, window.end AS e, SUM(v) AS total FROM T "
                     "GROUP BY window(ts, '10 minutes') ORDER BY s", cat, ctx).to_pylist()
    b = dt.datetime(2024, 1, 1, 12, 0, 0)
    m = lambda k: b + dt.timedelta(minutes=k)
    assert [(r["s"], r["e"], r["total"]) for r in tumble] == [(m(0), m(10), 6), (m(10), m(20), 9)]
    # 10-minute windows sliding every 5: each event falls into two windows [k*5, k*5+10)
    slide = run_sql("SELECT window.start AS s, SUM(v) AS total, COUNT(*) AS c FROM T "
                    "GROUP BY window(ts, '10 minutes', '5 minutes') ORDER BY s", cat, ctx).to_pylist()
    assert [(r["s"], r["total"], r["c"]) for r in slide] == [(m(-5), 3, 2), (m(0), 6, 3), (m(5), 12, 3),
                                                            (m(10), 9, 2)]


@pytest.mark.parametrize("device", DEVICES)
def test_aggregates_documented_values(device):
    got = _q("SELECT dept, COUNT(*) AS c, SUM(salary) AS s, AVG(age) AS a, MAX(name) AS mx, MIN(name) AS mn, "
             "COLLECT_SET(age) AS ages, STDDEV_POP(salary) AS sp, VAR_SAMP(salary) AS vs, "
             "APPROX_COUNT_DISTINCT(salary) AS acd, FIRST(name) AS f, COUNT(DISTINCT salary) AS cd "
             "FROM employees GROUP BY dept ORDER BY dept", device)
    eng, mkt, sales = got
    assert (eng["dept"], eng["c"], eng["s"], eng["a"]) == ("Engineering", 4, 96000, 27.25)
    assert (eng["mx"], eng["mn"], sorted(eng["ages"]), eng["cd"], eng["acd"]) == \
        ("Tom", "Chloe", [23, 25, 28, 33], 3, 3)
    # salaries 21000, 23000, 23000, 29000: mean 24000, squared deviations 9e6 + 1e6 + 1e6 + 25e6 = 36e6
    assert eng["sp"] == pytest.approx((36e6 / 4) ** 0.5) and eng["vs"] == pytest.approx(36e6 / 3)
    assert (mkt["c"], mkt["s"], mkt["a"]) == (2, 64000, 33.0) and mkt["f"] in ("Jane", "Jeff")
    assert (sales["c"], sales["s"], sales["mx"], sales["mn"]) == (3, 72000, "Lisa", "Alex")
