"""Spark 2.4 integer widths and the round-5 review's silent-wrong-answer probes (VERDICT r5 Missing #1-2, Weak #2).

The reference runs every transform statement through ``spark.sql`` on Spark 2.4.5 (CommonProcessorFactory.scala:
257-275, datax-host/pom.xml:57) and reads user schemas with ``DataType.fromJson`` (SchemaFile.scala:22-26), which
has byte / short / integer / long types.  pyspark is not importable here and the reference ships no fixture for these
values, so parity is unpinned by any reference output: every expected value below is computed by hand from the JVM
rules Spark 2.4 applies —

* TINYINT / SMALLINT / INT / BIGINT arithmetic (``+ - *``, unary ``-``, ``abs``) wraps two's-complement at its width
  (Java ``int`` / ``long`` overflow; Spark's Add/Multiply on ByteType use ``(a + b).toByte``);
* narrowing casts keep the low bits (``Long.toInt``), double → integral is the JVM's saturating d2i / d2l with
  NaN → 0 (Scala ``Double.toInt``; ``toShort`` / ``toByte`` narrow the int), decimal → integral truncates then keeps
  the low bits (``Decimal.toLong``), string → integral is NULL out of range (``UTF8String.toInt`` etc.);
* integer literals are INT when they fit, else BIGINT, else decimal (AstBuilder.visitIntegerLiteral, the minus
  folded in); exponent literals are decimals (DECIMAL_VALUE; doubles only from Spark 3.0, SPARK-29956);
* ``CAST(array/map/struct AS STRING)`` is Cast.castToString of 2.4: ``[a, b]``, ``[k -> v]``, ``[f1, f2]``, NULL
  elements omitted with their separator kept (the behaviour Spark 3.0 keeps behind
  ``spark.sql.legacy.castComplexTypesToString.enabled``);
* ``ceil`` / ``floor`` of decimal(p, s) is decimal(p - s + 1, 0).

One bracketed value of the review differs from the JVM: ``CAST(3 AS INT) * 2147483647`` is 6442450941 mod 2^32 =
2147483645 in Java (Integer.MAX_VALUE * 3), not -2147483645.  ``cuda`` runs the same statements on the MI355X (the
tensor evaluator and, above 64 K rows, the fused hipRTC kernels, ``test_jit.py``)."""
import decimal

import pytest
import torch

from dxa.engine.column import Table
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql
from dxa.engine.types import StructField, StructType, schema_from_json

D = decimal.Decimal
DEV = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]
S = StructType((StructField("id", "long"), StructField("v", "double"), StructField("i", "int"),
                StructField("h", "short"), StructField("t", "byte")))
ROWS = [{"id": 3, "v": 0.5, "i": 2147483647, "h": 32767, "t": 127},
        {"id": -2, "v": 1e9, "i": -2147483648, "h": -32768, "t": -128}]


def _dev(device):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    return device


def q(sql, device="cpu", rows=ROWS):
    cat = Catalog()
    cat.register("T", Table.from_pylist(rows, S, device))
    out = run_sql(sql, cat, EvalContext(device=torch.device(device)))
    return {n: (str(c.dtype), c.to_pylist()) for n, c in zip(out.names, out.columns)}


def one(sql, device="cpu"):
    """First row of every output column: name → (type, value)."""
    return {k: (t, v[0]) for k, (t, v) in q(sql, device).items()}


@pytest.mark.parametrize("device", DEV)
def test_narrowing_casts_truncate(device):
    r = one("SELECT CAST(300 AS TINYINT) a, CAST(70000 AS SMALLINT) b, CAST(3000000000 AS INT) c, "
            "CAST(-129 AS TINYINT) d, CAST(id * 100 AS TINYINT) e FROM T", _dev(device))
    assert r == {"a": ("byte", 44), "b": ("short", 4464), "c": ("int", -1294967296), "d": ("byte", 127),
                 "e": ("byte", 44)}


@pytest.mark.parametrize("device", DEV)
def test_int_arithmetic_wraps(device):
    got = q("SELECT CAST(id AS INT) * 2147483647 a, 2147483647 + 1 b, abs(CAST(-2147483648 AS INT)) c, "
            "i + 1 d, i * 2 e, -i f, abs(i) g, i - 1 h2 FROM T", _dev(device))
    assert got["a"] == ("int", [2147483645, 2])                      # 3 * MAX = MAX - 2; -2 * MAX = 2
    assert got["b"] == ("int", [-2147483648] * 2)
    assert got["c"] == ("int", [-2147483648] * 2)
    assert got["d"] == ("int", [-2147483648, -2147483647])
    assert got["e"] == ("int", [-2, 0])
    assert got["f"] == ("int", [-2147483647, -2147483648])
    assert got["g"] == ("int", [2147483647, -2147483648])
    assert got["h2"] == ("int", [2147483646, 2147483647])


@pytest.mark.parametrize("device", DEV)
def test_small_types_keep_their_width(device):
    got = q("SELECT h + h a, t + t b, t * t c, h + t d, -t e, t + 1 f, h * 2L g, typeof(h + t) th, "
            "typeof(t + t) tt, typeof(t + 1) t1 FROM T", _dev(device))
    assert got["a"] == ("short", [-2, 0])
    assert got["b"] == ("byte", [-2, 0])
    assert got["c"] == ("byte", [1, 0])                              # 127^2 = 16129 = 0x3F01; 128^2 = 0x4000
    assert got["d"] == ("short", [-32642, 32640])                    # smallint + tinyint → smallint
    assert got["e"] == ("byte", [-127, -128])
    assert got["f"] == ("int", [128, -127])                          # tinyint + INT literal → int
    assert got["g"] == ("long", [65534, -65536])
    assert got["th"][1][0] == "smallint" and got["tt"][1][0] == "tinyint" and got["t1"][1][0] == "int"


@pytest.mark.parametrize("device", DEV)
def test_long_overflow_and_literal_folding(device):
    r = one("SELECT -CAST(-9223372036854775808 AS BIGINT) a, 9223372036854775807 + 1 b, "
            "-9223372036854775808 c, typeof(-9223372036854775808) tc, typeof(-2147483648) td, "
            "typeof(2147483648) te, typeof(9223372036854775808) tf, id * 9223372036854775807 g FROM T",
            _dev(device))
    assert r["a"] == ("long", -9223372036854775808)
    assert r["b"] == ("long", -9223372036854775808)
    assert r["c"] == ("long", -9223372036854775808)
    assert (r["tc"][1], r["td"][1], r["te"][1], r["tf"][1]) == ("bigint", "int", "bigint", "decimal(19,0)")
    assert r["g"] == ("long", 9223372036854775805)                   # 3 * MAX wraps to MAX - 2


@pytest.mark.parametrize("device", DEV)
def test_double_to_integral_saturates_like_d2i(device):
    got = q("SELECT CAST(v * 1e12 AS INT) a, CAST(v * 1e30 AS BIGINT) b, CAST(-v * 1e30 AS INT) c, "
            "CAST(CAST('NaN' AS DOUBLE) AS INT) d, CAST(v * 1e6 AS SMALLINT) e, CAST(1e20 AS INT) f, "
            "CAST(CAST('Infinity' AS DOUBLE) AS BIGINT) g FROM T", _dev(device))
    assert got["a"] == ("int", [2147483647, 2147483647])
    assert got["b"] == ("long", [9223372036854775807] * 2)
    assert got["c"] == ("int", [-2147483648] * 2)
    assert got["d"] == ("int", [0, 0])
    # d2i first (500000 / 1e15 → MAX_INT), then the low 16 bits: 500000 = 0x7A120 → 0xA120 = -24288; 0x7FFFFFFF → -1
    assert got["e"] == ("short", [-24288, -1])
    # 1e20 is a decimal literal: Decimal.toLong keeps the low 64 bits, toInt the low 32 → 10^20 mod 2^32
    assert got["f"] == ("int", [1661992960] * 2)
    assert got["g"] == ("long", [9223372036854775807] * 2)


@pytest.mark.parametrize("device", DEV)
def test_string_to_integral_is_null_out_of_range(device):
    r = one("SELECT CAST('200' AS TINYINT) a, CAST('-128' AS TINYINT) b, CAST(' 32767 ' AS SMALLINT) c, "
            "CAST('32768' AS SMALLINT) d, CAST('2147483648' AS INT) e, CAST('12.9' AS TINYINT) f FROM T",
            _dev(device))
    assert r == {"a": ("byte", None), "b": ("byte", -128), "c": ("short", 32767), "d": ("short", None),
                 "e": ("int", None), "f": ("byte", 12)}


def test_string_column_to_small_types_on_each_device():
    """The device string → number kernel parses as int, then the narrow range check nulls the rest."""
    rows = [{"id": 1, "v": 0.0, "i": 0, "h": 0, "t": 0}]
    cat = Catalog()
    cat.register("T", Table.from_pylist(rows, S, "cpu"))
    out = run_sql("SELECT CAST(s AS TINYINT) a, CAST(s AS SMALLINT) b FROM (SELECT explode(array('127', '128', "
                  "'-32768', 'x')) s FROM T)", cat, EvalContext())
    assert [c.to_pylist() for c in out.columns] == [[127, None, None, None], [127, 128, -32768, None]]


def test_exponent_literals_are_decimals():
    r = one("SELECT 1e20 a, 1.5e0 b, 15e-4 c, typeof(1.5e0) tb, 1e2D d, 2.5 e FROM T")
    assert r["a"] == ("decimal(21,0)", D("100000000000000000000"))
    assert r["b"] == ("decimal(2,1)", D("1.5"))
    assert r["c"] == ("decimal(4,4)", D("0.0015"))
    assert r["tb"][1] == "decimal(2,1)"
    assert r["d"] == ("double", 100.0)
    assert r["e"] == ("decimal(2,1)", D("2.5"))


def test_suffixed_literals():
    r = one("SELECT 10Y a, -128Y b, 300S c, 7L d, typeof(10Y) ta, typeof(300S) tc FROM T")
    assert r["a"] == ("byte", 10) and r["b"] == ("byte", -128) and r["c"] == ("short", 300)
    assert r["d"] == ("long", 7) and r["ta"][1] == "tinyint" and r["tc"][1] == "smallint"
    from dxa.sql.parser import SqlError
    with pytest.raises(SqlError):
        one("SELECT 200Y a FROM T")


@pytest.mark.parametrize("device", DEV)
def test_aggregates_of_small_types(device):
    got = q("SELECT sum(t) s, typeof(sum(t)) ts, max(h) m, typeof(max(h)) tm, min(t) n, avg(i) a, "
            "sum(i) si FROM T", _dev(device))
    assert got["s"] == ("long", [-1])
    assert got["ts"][1] == ["bigint"]
    assert got["m"] == ("short", [32767]) and got["tm"][1] == ["smallint"]
    assert got["n"] == ("byte", [-128])
    assert got["a"] == ("double", [-0.5])
    assert got["si"] == ("long", [-1])                               # SUM(int) is a BIGINT: no 32-bit wrap


@pytest.mark.parametrize("device", DEV)
def test_shifts_on_int_are_32_bit(device):
    r = one("SELECT shiftleft(i, 1) a, shiftleft(CAST(1 AS INT), 33) b, shiftrightunsigned(CAST(-1 AS INT), 28) c,"
            " shiftleft(id, 62) d, typeof(shiftleft(t, 1)) e FROM T", _dev(device))
    assert r == {"a": ("int", -2), "b": ("int", 2), "c": ("int", 15), "d": ("long", -4611686018427387904),
                 "e": ("string", "int")}


def test_schema_json_small_types_round_trip():
    sch = schema_from_json('{"type":"struct","fields":[{"name":"a","type":"byte","nullable":true,"metadata":{}},'
                           '{"name":"b","type":"short","nullable":true,"metadata":{}},'
                           '{"name":"c","type":"integer","nullable":true,"metadata":{}}]}')
    assert [f.dtype for f in sch.fields] == ["byte", "short", "int"]
    from dxa.engine.types import schema_to_json
    assert '"byte"' in schema_to_json(sch) and '"short"' in schema_to_json(sch) and '"integer"' in schema_to_json(sch)


@pytest.mark.parametrize("device", DEV)
def test_json_parse_small_types_range(device):
    """from_json of byte / short fields: values outside the type's range are NULL (the host parser and the device
    kernel + range check agree)."""
    from dxa.ops.jsonparse import ParsePlan, frame_records, parse
    sch = StructType((StructField("a", "byte"), StructField("b", "short")))
    recs = [b'{"a": 127, "b": -32768}', b'{"a": 128, "b": 32768}', b'{"a": -129, "b": 5}', b'{"a": "x", "b": 1.5}']
    want = [[127, None, None, None], [-32768, None, 5, None]]
    bg, og = frame_records(recs, device=torch.device(_dev(device)))
    col, _ = parse(bg, og, ParsePlan(sch))
    assert [col.child("a").to_pylist(), col.child("b").to_pylist()] == want
    assert col.child("a").dtype == "byte" and col.child("b").dtype == "short"


# ---- review Weak #2: complex casts, reverse(array), concat_ws NULLs, ceil / floor of decimals ---------------------

@pytest.mark.parametrize("device", DEV)
def test_complex_types_cast_to_string_spark24(device):
    r = one("SELECT CAST(array(1, NULL) AS STRING) a, CAST(map('a', 1) AS STRING) b, "
            "CAST(struct(1, 'x') AS STRING) c, CAST(array(NULL, 2) AS STRING) d, "
            "CAST(map('a', 1, 'b', NULL) AS STRING) e, CAST(struct(1, NULL, 'z') AS STRING) f, "
            "CAST(array(array(1.5D, 2.0D), NULL) AS STRING) g, CAST(array() AS STRING) h FROM T", _dev(device))
    assert {k: v for k, (_, v) in r.items()} == {"a": "[1,]", "b": "[a -> 1]", "c": "[1, x]", "d": "[, 2]",
                                                 "e": "[a -> 1, b ->]", "f": "[1,, z]", "g": "[[1.5, 2.0],]",
                                                 "h": "[]"}


@pytest.mark.parametrize("device", DEV)
def test_reverse_of_arrays(device):
    got = q("SELECT reverse(array(1, 2, 3)) a, reverse(array(1, NULL, 3)) b, reverse('abc') c, "
            "reverse(filter(array(1, 2, 3, 4), x -> x % 2 = 0)) d FROM T", _dev(device))
    assert got["a"] == ("array<int>", [[3, 2, 1]] * 2)
    assert got["b"] == ("array<int>", [[3, None, 1]] * 2)
    assert got["c"] == ("string", ["cba"] * 2)
    assert got["d"][1] == [[4, 2]] * 2


@pytest.mark.parametrize("device", DEV)
def test_concat_ws_skips_nulls_on_every_device(device):
    got = q("SELECT concat_ws('-', 'a', NULL, 'b') a, concat_ws(',', array('x', NULL, 'y'), 'z') b, "
            "concat_ws(NULL, 'a') c, concat_ws('-', 'a', CAST(NULL AS STRING), 1.5) d, "
            "concat_ws('/', CAST(id AS STRING), IF(id > 0, NULL, 'neg')) e FROM T", _dev(device))
    assert got["a"][1] == ["a-b"] * 2
    assert got["b"][1] == ["x,y,z"] * 2
    assert got["c"][1] == [None] * 2
    assert got["d"][1] == ["a-1.5"] * 2
    assert got["e"][1] == ["3", "-2/neg"]


@pytest.mark.parametrize("device", DEV)
def test_ceil_floor_of_decimals_stay_decimal(device):
    r = one("SELECT ceil(CAST(1.5 AS DECIMAL(3,1))) a, floor(CAST(-1.5 AS DECIMAL(3,1))) b, "
            "ceil(CAST(-1.5 AS DECIMAL(3,1))) c, floor(CAST(2.0 AS DECIMAL(3,1))) d, "
            "to_json(named_struct('x', ceil(CAST(1.25 AS DECIMAL(5,2))))) e, ceil(2.5D) f, floor(-2.5D) g, "
            "ceil(CAST(7 AS INT)) h, typeof(ceil(5)) ti FROM T", _dev(device))
    assert r["a"] == ("decimal(3,0)", D(2)) and r["b"] == ("decimal(3,0)", D(-2))
    assert r["c"] == ("decimal(3,0)", D(-1)) and r["d"] == ("decimal(3,0)", D(2))
    assert r["e"][1] == '{"x":2}'
    assert r["f"] == ("long", 3) and r["g"] == ("long", -3) and r["h"] == ("long", 7)
    assert r["ti"][1] == "bigint"


@pytest.mark.parametrize("device", DEV)
def test_decimal_column_ceil_floor(device):
    sch = StructType((StructField("d", __import__("dxa.engine.decimal", fromlist=["x"]).DecimalType(10, 3)),))
    rows = [{"d": D(x)} for x in ("1.001", "-1.001", "5.000", "-0.500", "0.000")] + [{"d": None}]
    cat = Catalog()
    cat.register("T", Table.from_pylist(rows, sch, _dev(device)))
    out = run_sql("SELECT ceil(d) c, floor(d) f FROM T", cat, EvalContext(device=torch.device(device)))
    c, f = (x.to_pylist() for x in out.columns)
    assert str(out.columns[0].dtype) == "decimal(8,0)"
    assert c == [D(2), D(-1), D(5), D(0), D(0), None]
    assert f == [D(1), D(-2), D(5), D(-1), D(0), None]


# ---- review Missing #2: Spark 2.4 built-ins and syntax ---------------------------------------------------------

@pytest.mark.parametrize("device", DEV)
def test_new_builtins(device):
    got = q("SELECT arrays_zip(array(1, 2), array('a', 'b', 'c')) z, map_from_entries(array(struct('k', 1), "
            "struct('m', 2))) m, space(3) s, size(shuffle(array(1, 2, 3))) n, sort_array(shuffle(array(3, 1, 2))) o "
            "FROM T", _dev(device))
    assert got["z"][1][0] == [{"0": 1, "1": "a"}, {"0": 2, "1": "b"}, {"0": None, "1": "c"}]
    assert got["m"][1][0] == {"k": 1, "m": 2}
    assert got["s"][1] == ["   "] * 2
    assert got["n"][1] == [3] * 2
    assert got["o"][1] == [[1, 2, 3]] * 2


def test_arrays_zip_names_from_columns():
    got = q("SELECT arrays_zip(x, y) z FROM (SELECT array(1, 2) x, array(3) y FROM T)")
    assert got["z"] == ("array<struct<x:int,y:int>>", [[{"x": 1, "y": 3}, {"x": 2, "y": None}]] * 2)


def test_stack_multi_alias_and_u_pattern():
    got = q("SELECT stack(2, 1, 'a', 2, 'b') AS (x, y) FROM T WHERE id > 0")
    assert got == {"x": ("int", [1, 2]), "y": ("string", ["a", "b"])}
    got = q("SELECT posexplode(array(5, 6)) AS (p, v) FROM T WHERE id > 0")
    assert got == {"p": ("int", [0, 1]), "v": ("int", [5, 6])}
    r = one("SELECT date_format(CAST('2024-05-06 07:08:09' AS TIMESTAMP), 'u') a, "
            "date_format(CAST('2024-05-12 00:08:09' AS TIMESTAMP), 'u F k K w W') b, "
            "date_format(CAST('2024-12-30 00:00:00' AS TIMESTAMP), 'w') c FROM T")
    assert (r["a"][1], r["b"][1], r["c"][1]) == ("1", "7 2 24 0 20 3", "1")
    from dxa.engine.query import QueryError
    with pytest.raises(QueryError):
        q("SELECT id AS (a, b) FROM T")
