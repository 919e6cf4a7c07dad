"""SQL semantics of the columnar engine (Spark SQL behaviour the reference's transforms rely on), on CPU tensors.
Expected values are hand-computed Spark results."""
import json

import pytest

from dxa.engine.column import Table
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql
from dxa.engine.serialize import table_to_json_lines
from dxa.engine.types import ArrayType, MapType, StructField, StructType

SCHEMA = StructType((StructField("id", "long"), StructField("kind", "string"), StructField("temp", "double"),
                     StructField("home", "long"), StructField("ts", "timestamp"),
                     StructField("d", StructType((StructField("a", "long"), StructField("b", "string"))))))
ROWS = [
    {"id": 1, "kind": "door", "temp": 20.5, "home": 150, "ts": None, "d": {"a": 1, "b": "x"}},
    {"id": 2, "kind": "heat", "temp": 35.0, "home": 150, "ts": None, "d": {"a": 2, "b": None}},
    {"id": 3, "kind": "door", "temp": None, "home": 32, "ts": None, "d": None},
    {"id": 4, "kind": None, "temp": -4.25, "home": 32, "ts": None, "d": {"a": None, "b": "y"}},
    {"id": 5, "kind": "heat", "temp": 99.5, "home": 150, "ts": None, "d": {"a": 5, "b": "z"}},
]
REF = [{"home": 150, "owner": "ann"}, {"home": 32, "owner": "bob"}, {"home": 7, "owner": "cid"}]


@pytest.fixture(scope="module")
def cat():
    c = Catalog()
    c.register("T", Table.from_pylist(ROWS, SCHEMA))
    c.register("R", Table.from_pylist(REF, StructType((StructField("home", "long"), StructField("owner", "string")))))
    return c


def q(cat, sql):
    return [json.loads(l) for l in table_to_json_lines(run_sql(sql, cat, EvalContext(now_us=0)))]


def test_projection_and_filter(cat):
    assert q(cat, "SELECT id, temp * 2 AS t2 FROM T WHERE temp > 0 AND home = 150") == [
        {"id": 1, "t2": 41.0}, {"id": 2, "t2": 70.0}, {"id": 5, "t2": 199.0}]


def test_three_valued_logic(cat):
    # NULL comparisons are unknown → filtered out; NOT of unknown stays unknown
    assert [r["id"] for r in q(cat, "SELECT id FROM T WHERE NOT (temp > 30)")] == [1, 4]
    assert [r["id"] for r in q(cat, "SELECT id FROM T WHERE temp IS NULL OR kind IS NULL")] == [3, 4]
    assert q(cat, "SELECT id, (temp > 30 OR TRUE) AS x, (temp > 30 AND FALSE) AS y FROM T WHERE id = 3") == [
        {"id": 3, "x": True, "y": False}]


def test_group_by_aggregates(cat):
    got = q(cat, "SELECT home, COUNT(*) AS n, COUNT(temp) AS nt, SUM(temp) AS s, MIN(temp) AS mn, MAX(temp) AS mx, "
                 "AVG(temp) AS av FROM T GROUP BY home ORDER BY home")
    assert got == [{"home": 32, "n": 2, "nt": 1, "s": -4.25, "mn": -4.25, "mx": -4.25, "av": -4.25},
                   {"home": 150, "n": 3, "nt": 3, "s": 155.0, "mn": 20.5, "mx": 99.5, "av": 155.0 / 3}]


def test_group_by_null_key_and_having(cat):
    got = q(cat, "SELECT kind, COUNT(*) AS n FROM T GROUP BY kind HAVING COUNT(*) >= 1 ORDER BY kind")
    assert got == [{"n": 1}, {"kind": "door", "n": 2}, {"kind": "heat", "n": 2}]     # nulls first, key omitted


def test_global_aggregate_over_empty_input(cat):
    assert q(cat, "SELECT COUNT(*) AS n, SUM(temp) AS s FROM T WHERE id > 100") == [{"n": 0}]


def test_count_distinct_and_collect(cat):
    assert q(cat, "SELECT COUNT(DISTINCT kind) AS k, COUNT(DISTINCT home) AS h FROM T") == [{"k": 2, "h": 2}]


def test_inner_and_left_join(cat):
    assert q(cat, "SELECT T.id, R.owner FROM T JOIN R ON T.home = R.home WHERE T.id <= 3 ORDER BY T.id") == [
        {"id": 1, "owner": "ann"}, {"id": 2, "owner": "ann"}, {"id": 3, "owner": "bob"}]
    got = q(cat, "SELECT R.owner, COUNT(T.id) AS n FROM R LEFT JOIN T ON R.home = T.home GROUP BY R.owner "
                 "ORDER BY R.owner")
    assert got == [{"owner": "ann", "n": 3}, {"owner": "bob", "n": 2}, {"owner": "cid", "n": 0}]


def test_semi_anti_join(cat):
    assert q(cat, "SELECT owner FROM R LEFT SEMI JOIN T ON R.home = T.home ORDER BY owner") == [
        {"owner": "ann"}, {"owner": "bob"}]
    assert q(cat, "SELECT owner FROM R LEFT ANTI JOIN T ON R.home = T.home") == [{"owner": "cid"}]


def test_union_distinct_and_all(cat):
    assert len(q(cat, "SELECT home FROM T UNION ALL SELECT home FROM R")) == 8
    assert sorted(r["home"] for r in q(cat, "SELECT home FROM T UNION SELECT home FROM R")) == [7, 32, 150]
    assert q(cat, "SELECT DISTINCT home FROM T ORDER BY home DESC") == [{"home": 150}, {"home": 32}]


def test_order_by_limit_nulls(cat):
    assert [r.get("temp") for r in q(cat, "SELECT temp FROM T ORDER BY temp")] == [None, -4.25, 20.5, 35.0, 99.5]
    assert [r.get("temp") for r in q(cat, "SELECT temp FROM T ORDER BY temp DESC LIMIT 2")] == [99.5, 35.0]


def test_case_if_coalesce(cat):
    got = q(cat, "SELECT id, CASE WHEN temp > 50 THEN 'hot' WHEN temp > 0 THEN 'warm' ELSE 'cold' END AS c, "
                 "IF(kind IS NULL, 'none', kind) AS k, COALESCE(temp, 0.0) AS t FROM T ORDER BY id")
    assert [(r["c"], r["k"], r["t"]) for r in got] == [("warm", "door", 20.5), ("warm", "heat", 35.0),
                                                       ("cold", "door", 0.0), ("cold", "none", -4.25),
                                                       ("hot", "heat", 99.5)]


def test_string_functions(cat):
    got = q(cat, "SELECT CONCAT(kind, '-', id) AS c, UPPER(kind) AS u, LENGTH(kind) AS l, "
                 "SUBSTRING(kind, 2, 2) AS s FROM T WHERE id = 1")
    assert got == [{"c": "door-1", "u": "DOOR", "l": 4, "s": "oo"}]
    assert q(cat, "SELECT id FROM T WHERE kind LIKE 'h%' ORDER BY id") == [{"id": 2}, {"id": 5}]
    assert q(cat, "SELECT CONCAT(kind, 'x') AS c FROM T WHERE id = 4") == [{}]      # null input → null


def test_struct_access_and_construction(cat):
    assert q(cat, "SELECT d.a AS a, d.b AS b FROM T WHERE id IN (1, 2, 3)") == [
        {"a": 1, "b": "x"}, {"a": 2}, {}]
    got = q(cat, "SELECT STRUCT(id, kind) AS s, MAP('k', kind) AS m, ARRAY(id, home) AS a FROM T WHERE id = 1")
    assert got == [{"s": {"id": 1, "kind": "door"}, "m": {"k": "door"}, "a": [1, 150]}]


def test_filter_null_rules_shape(cat):
    """The rules codegen's filterNull(Array(IF(cond, MAP(...), NULL), ...)) shape."""
    got = q(cat, "SELECT id, filterNull(Array(IF(temp > 30, MAP('ruleId', 'hot'), NULL), "
                 "IF(home = 150, MAP('ruleId', 'h150'), NULL))) AS Rules FROM T ORDER BY id")
    assert [r["Rules"] for r in got] == [[{"ruleId": "h150"}], [{"ruleId": "hot"}, {"ruleId": "h150"}], [], [],
                                         [{"ruleId": "hot"}, {"ruleId": "h150"}]]


def test_cast_and_arithmetic(cat):
    got = q(cat, "SELECT CAST(temp AS INT) AS i, CAST(id AS STRING) AS s, id / 2 AS h, id % 2 AS m, "
                 "CAST('12' AS LONG) + 1 AS p FROM T WHERE id = 5")
    assert got == [{"i": 99, "s": "5", "h": 2.5, "m": 1, "p": 13}]


def test_subquery_and_views(cat):
    c2 = Catalog()
    for n in ("T", "R"):
        c2.register(n, cat.get(n))
    c2.register("V", run_sql("SELECT home, COUNT(*) AS n FROM T GROUP BY home", c2, EvalContext()))
    assert q(c2, "SELECT owner, n FROM V JOIN R ON V.home = R.home ORDER BY n") == [
        {"owner": "bob", "n": 2}, {"owner": "ann", "n": 3}]
    assert q(c2, "SELECT MAX(n) AS m FROM (SELECT home, COUNT(*) AS n FROM T GROUP BY home) x") == [{"m": 3}]


def test_group_by_alias_and_ordinal(cat):
    assert q(cat, "SELECT home AS h, COUNT(*) AS n FROM T GROUP BY h ORDER BY h") == [
        {"h": 32, "n": 2}, {"h": 150, "n": 3}]
    assert q(cat, "SELECT home, COUNT(*) AS n FROM T GROUP BY 1 ORDER BY 1") == [
        {"home": 32, "n": 2}, {"home": 150, "n": 3}]


def test_timestamp_functions():
    c = Catalog()
    sch = StructType((StructField("s", "string"),))
    c.register("S", Table.from_pylist([{"s": "2019-02-28T22:45:10Z"}, {"s": "03/01/2019 01:02:03"}], sch))
    got = q(c, "SELECT stringToTimestamp(s) AS t, hour(stringToTimestamp(s)) AS h, "
               "date_trunc('hour', stringToTimestamp(s)) AS d FROM S")
    assert got == [{"t": "2019-02-28T22:45:10.000Z", "h": 22, "d": "2019-02-28T22:00:00.000Z"},
                   {"t": "2019-03-01T01:02:03.000Z", "h": 1, "d": "2019-03-01T01:00:00.000Z"}]
