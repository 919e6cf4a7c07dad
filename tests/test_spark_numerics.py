"""Spark 2.4-pinned numerics of aggregates, window frames and scalar built-ins (round 5 fixes).

The reference hands every transform statement to ``spark.sql`` on Spark 2.4.5 (CommonProcessorFactory.scala:257-275,
datax-host/pom.xml:57).  Expected values are computed by hand from Spark's documented rules — DecimalPrecision
(SUM → decimal(p+10, s), AVG → decimal(p+4, s+4) HALF_UP), CentralMomentAgg ((n, mean, M2), NaN for one row),
RoundBase (``BigDecimal(Double.toString(x)).setScale(d, mode)``; decimal(p, min(s, d))), Murmur3Hash of decimals
(hashLong(unscaled) for p <= 18) — or with Python's exact ``decimal`` / ``math.fsum`` over the same inputs; pyspark
is not importable here, so parity beyond those documents is unpinned.  ``cuda`` runs the same statements on the
device."""
import decimal
import math
import random

import pytest
import torch

from dxa.engine.column import Table
from dxa.engine.decimal import DecimalType
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql
from dxa.engine.types import StructField, StructType

D = decimal.Decimal
DEV = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]

S = StructType((StructField("k", "long"), StructField("s", "string"), StructField("d", DecimalType(10, 2)),
                StructField("w", DecimalType(30, 4)), StructField("v", "double")))
ROWS = [{"k": 1, "s": "b1", "d": D("1.25"), "w": D("12345678901234567890.1234"), "v": 1e9 + 1},
        {"k": 1, "s": "a", "d": D("2.50"), "w": D("-1.0001"), "v": 1e9 + 2},
        {"k": 2, "s": "bb", "d": D("3.75"), "w": D("0.5000"), "v": 1e9 + 3},
        {"k": 2, "s": None, "d": None, "w": None, "v": None},
        {"k": 3, "s": "c", "d": D("5.00"), "w": D("7"), "v": 7.0}]


def _dev(device):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    return device


def q(sql, device="cpu", rows=ROWS, schema=S):
    cat = Catalog()
    cat.register("T", Table.from_pylist(rows, schema, device))
    out = run_sql(sql, cat, EvalContext(device=torch.device(device)))
    cols = [c.to_pylist() for c in out.columns]
    return out.names, [str(c.dtype) for c in out.columns], list(zip(*cols)) if cols else []


# ---- decimal window aggregates ---------------------------------------------------------------------------------

@pytest.mark.parametrize("device", DEV)
def test_decimal_window_sum_avg_whole_partition(device):
    _, types, rows = q("SELECT SUM(d) OVER () AS s, AVG(d) OVER () AS a FROM T", _dev(device))
    assert types == ["decimal(20,2)", "decimal(14,6)"]
    assert set(rows) == {(D("12.50"), D("3.125000"))}


@pytest.mark.parametrize("device", DEV)
def test_decimal_window_running_and_sliding(device):
    _, types, rows = q("SELECT k, d, SUM(d) OVER (ORDER BY d ROWS BETWEEN UNBOUNDED PRECEDING AND CURRENT ROW) AS rs, "
                       "MIN(d) OVER (ORDER BY d ROWS BETWEEN 1 PRECEDING AND CURRENT ROW) AS m, "
                       "MAX(d) OVER (PARTITION BY k) AS mx, "
                       "AVG(d) OVER (ORDER BY d ROWS BETWEEN 1 PRECEDING AND 1 FOLLOWING) AS av FROM T", _dev(device))
    assert types == ["long", "decimal(10,2)", "decimal(20,2)", "decimal(10,2)", "decimal(10,2)", "decimal(14,6)"]
    got = {r[1]: r[2:] for r in rows}
    # ORDER BY d ascending: NULL first (a frame of only the null row sums to NULL)
    assert got[None] == (None, None, D("3.75"), D("1.250000"))
    assert got[D("1.25")] == (D("1.25"), D("1.25"), D("2.50"), D("1.875000"))
    assert got[D("2.50")] == (D("3.75"), D("1.25"), D("2.50"), D("2.500000"))
    assert got[D("3.75")] == (D("7.50"), D("2.50"), D("3.75"), D("3.750000"))
    assert got[D("5.00")] == (D("12.50"), D("3.75"), D("5.00"), D("4.375000"))


@pytest.mark.parametrize("device", DEV)
def test_wide_decimal_window_aggregates(device):
    _, types, rows = q("SELECT SUM(w) OVER () AS s, MAX(w) OVER () AS mx, MIN(w) OVER () AS mn, "
                       "AVG(w) OVER () AS a FROM T", _dev(device))
    assert types == ["decimal(38,4)", "decimal(30,4)", "decimal(30,4)", "decimal(34,8)"]
    total = D("12345678901234567890.1234") + D("-1.0001") + D("0.5000") + D("7")
    avg = (total / 4).quantize(D("1e-8"), rounding=decimal.ROUND_HALF_UP)
    assert set(rows) == {(total, D("12345678901234567890.1234"), D("-1.0001"), avg)}


@pytest.mark.parametrize("device", DEV)
def test_decimal_percentiles(device):
    _, types, rows = q("SELECT percentile_approx(d, 0.5) AS pa, percentile(d, 0.5) AS p, median(d) AS m, "
                       "percentile(d, 0.25) AS p25 FROM T", _dev(device))
    # percentile_approx returns an input value (its type); percentile interpolates doubles
    assert types == ["decimal(10,2)", "double", "double", "double"]
    assert rows == [(D("2.50"), 3.125, 3.125, 2.1875)]


# ---- variance family -------------------------------------------------------------------------------------------

@pytest.mark.parametrize("device", DEV)
def test_stddev_no_catastrophic_cancellation(device):
    _, _, rows = q("SELECT stddev(v) AS sd, variance(v) AS va, var_pop(v) AS vp FROM T WHERE k <= 2", _dev(device))
    assert rows == [(1.0, 1.0, pytest.approx(2 / 3, rel=1e-12))]
    rows2 = [{"k": 1, "s": None, "d": None, "w": None, "v": 1.6e12 + x} for x in (0, 10, 20, 30)]
    _, _, r = q("SELECT stddev(v) AS sd FROM T", _dev(device), rows=rows2)
    assert r[0][0] == pytest.approx(math.sqrt(500 / 3), rel=1e-12)          # 12.909944…


@pytest.mark.parametrize("device", DEV)
def test_sample_statistics_of_one_row_are_nan(device):
    _, _, rows = q("SELECT k, stddev(v) AS sd, var_samp(v) AS vs, stddev_pop(v) AS sp FROM T GROUP BY k ORDER BY k",
                   _dev(device))
    assert rows[0] == (1, pytest.approx(math.sqrt(0.5)), pytest.approx(0.5), pytest.approx(0.5))
    k2, sd, vs, sp = rows[1]                              # one non-null value: NaN (Spark 2.4), pop 0
    assert math.isnan(sd) and math.isnan(vs) and sp == 0.0
    assert rows[2][0] == 3 and math.isnan(rows[2][1])


@pytest.mark.parametrize("device", DEV)
def test_sliding_double_frame_sum_is_exact_for_two_rows(device):
    rnd = random.Random(3)
    n = 20000
    vals = [1.6e12 + rnd.randrange(0, 10**6) / 8.0 for _ in range(n)]
    rows = [{"k": i, "s": None, "d": None, "w": None, "v": x} for i, x in enumerate(vals)]
    _, _, r = q("SELECT k, SUM(v) OVER (ORDER BY k ROWS BETWEEN 1 PRECEDING AND CURRENT ROW) AS s2, "
                "SUM(v) OVER (ORDER BY k ROWS BETWEEN 3 PRECEDING AND 3 FOLLOWING) AS s7 FROM T", _dev(device),
                rows=rows)
    for k, s2, s7 in r:
        want2 = vals[k] + (vals[k - 1] if k else 0.0)
        assert s2 == (vals[k - 1] + vals[k] if k else vals[0]), (k, s2, want2)
        want7 = math.fsum(vals[max(0, k - 3):k + 4])
        assert abs(s7 - want7) <= 4 * 2.0 ** -52 * want7, (k, s7, want7)


# ---- round / bround --------------------------------------------------------------------------------------------

@pytest.mark.parametrize("device", DEV)
def test_round_bround_doubles_follow_double_tostring(device):
    _, types, rows = q("SELECT round(CAST(1.005 AS DOUBLE), 2) AS a, bround(CAST(2.5 AS DOUBLE), 0) AS b, "
                       "bround(CAST(3.5 AS DOUBLE), 0) AS c, round(CAST(0.125 AS DOUBLE), 2) AS d2, "
                       "bround(CAST(0.125 AS DOUBLE), 2) AS e, round(CAST(-2.5 AS DOUBLE), 0) AS f, "
                       "round(CAST(1234.5678 AS DOUBLE), -2) AS g, round(1250, -2) AS h, bround(1250, -2) AS i "
                       "FROM T WHERE k = 3", _dev(device))
    assert types[:7] == ["double"] * 7 and types[7:] == ["int", "int"]
    assert rows == [(1.01, 2.0, 4.0, 0.13, 0.12, -3.0, 1200.0, 1300, 1200)]


@pytest.mark.parametrize("device", DEV)
def test_round_bround_decimals_keep_decimal_type(device):
    _, types, rows = q("SELECT round(1.005, 2) AS a, bround(1.005, 2) AS b, round(d, 1) AS c, bround(d, 1) AS e, "
                       "round(2.5) AS f, bround(2.5) AS g FROM T WHERE k = 1 ORDER BY d", _dev(device))
    assert types == ["decimal(4,2)", "decimal(4,2)", "decimal(10,1)", "decimal(10,1)", "decimal(2,0)", "decimal(2,0)"]
    assert rows == [(D("1.01"), D("1.00"), D("1.3"), D("1.2"), D("3"), D("2")),
                    (D("1.01"), D("1.00"), D("2.5"), D("2.5"), D("3"), D("2"))]


# ---- struct(*), auto names, arrays ---------------------------------------------------------------------------

@pytest.mark.parametrize("device", DEV)
def test_struct_star_and_to_json(device):
    names, types, rows = q("SELECT to_json(struct(*)) AS j, struct(t.*) AS st FROM T t WHERE k = 3", _dev(device))
    assert rows[0][0] == '{"k":3,"s":"c","d":5.00,"w":7.0000,"v":7.0}'
    assert types[1] == "struct<k:long,s:string,d:decimal(10,2),w:decimal(30,4),v:double>"


def test_spark_auto_names():
    names, _, _ = q("SELECT s LIKE 'b%', s RLIKE 'b', CASE WHEN k > 1 THEN 1 ELSE 0 END, k BETWEEN 1 AND 2, "
                    "s IS NULL, s IS NOT NULL, -k, NOT (k > 1), ROW_NUMBER() OVER (ORDER BY k), SUM(k) OVER (), "
                    "CAST(k AS BIGINT), k IN (1, 2), ucase(s), count(*), "
                    "SUM(k) OVER (PARTITION BY s ORDER BY k DESC) FROM T")
    assert names == ["s LIKE b%", "s RLIKE b", "CASE WHEN (k > 1) THEN 1 ELSE 0 END", "((k >= 1) AND (k <= 2))",
                     "(s IS NULL)", "(s IS NOT NULL)", "(- k)", "(NOT (k > 1))",
                     "row_number() OVER (ORDER BY k ASC NULLS FIRST ROWS BETWEEN UNBOUNDED PRECEDING AND CURRENT "
                     "ROW)", "sum(k) OVER (ROWS BETWEEN UNBOUNDED PRECEDING AND UNBOUNDED FOLLOWING)",
                     "CAST(k AS BIGINT)", "(k IN (1, 2))", "upper(s)", "count(1)",
                     "sum(k) OVER (PARTITION BY s ORDER BY k DESC NULLS LAST RANGE BETWEEN UNBOUNDED PRECEDING AND "
                     "CURRENT ROW)"]
    assert len(set(names)) == len(names)


@pytest.mark.parametrize("device", DEV)
def test_array_literals_in_array_contains_and_if(device):
    _, types, rows = q("SELECT k, array_contains(array(1, 2), 1) AS a, array_contains(array(1, 2), k) AS b, "
                       "IF(k > 1, array(1), array(2, 3)) AS c, size(IF(k > 1, array(1), array(2, 3))) AS n, "
                       "to_json(IF(k > 1, array(1), array(2, CAST(NULL AS INT)))) AS j, "
                       "size(IF(k > 2, array(1), NULL)) AS sn FROM T ORDER BY k, s", _dev(device))
    assert types[1:5] == ["boolean", "boolean", "array<int>", "int"]
    assert rows[0] == (1, True, True, [2, 3], 2, "[2,null]", -1)
    assert rows[-1] == (3, True, False, [1], 1, "[1]", 1)


@pytest.mark.parametrize("device", DEV)
def test_round_of_huge_doubles_is_identity(device):
    """round(x, d) on a double whose |x|·10^d passes 2^53 (or overflows) is x: BigDecimal(x).setScale(d) keeps a
    value with no digits below 10^-d (the scaled form must not become ±Infinity or NaN); far left of every digit the
    result is 0.0."""
    _, _, rows = q("SELECT round(1e300D, 10) a, round(1.5e300D, 400) b, round(123.456D, -400) c, "
                   "round(-1e300D, 2) d, bround(9007199254740993D, 1) e FROM T", _dev(device))
    assert rows[0] == (1e300, 1.5e300, 0.0, -1e300, 9007199254740992.0)
