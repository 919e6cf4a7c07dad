"""Spark 2.4 syntax and built-ins added in round 5: GROUP BY … GROUPING SETS, VALUES inline
tables (bare and parenthesised, with positional column aliases), TIMESTAMP / DATE typed literals, the named WINDOW
clause, ORDER BY a struct, Java short zone ids, str_to_map, map_concat, array_repeat, encode / decode (binary),
sentences, xpath_*, assert_true.  Expected rows are worked out by hand from Spark 2.4's documented behaviour (no Spark
here: parity unpinned by a reference fixture); the GPU test runs the same statements on the device and compares."""
import datetime as dt

import pytest

from test_sql_extended import q

SYNTAX_QUERIES = [
    "SELECT id, COUNT(*) AS c FROM T GROUP BY id GROUPING SETS ((id), ()) ORDER BY c, id",
    "SELECT a, b FROM VALUES (1, 'x'), (2, 'y') AS t(a, b)",
    "SELECT p FROM (VALUES (1, 2.5), (3, NULL)) AS v(p, q)",
    "SELECT COUNT(*) AS c FROM T WHERE ts < TIMESTAMP '2019-03-01 00:00:00'",
    "SELECT id, SUM(v) OVER w AS s FROM T WINDOW w AS (PARTITION BY id ORDER BY ts) ORDER BY id, ts",
    "SELECT id, rank() OVER w AS r, SUM(v) OVER w2 AS s FROM T WINDOW w AS (ORDER BY id), w2 AS (PARTITION BY id) "
    "ORDER BY id, r",
    "SELECT id, named_struct('a', id, 'b', v) AS st FROM T ORDER BY st DESC",
    "SELECT from_utc_timestamp(ts, 'PST') AS a, to_utc_timestamp(ts, 'EST') AS b, from_utc_timestamp(ts, 'CTT') AS c "
    "FROM T",
    "SELECT id, array_repeat(id, 2) AS b, str_to_map(name, ',', ':')['c'] AS m FROM T",
    "SELECT hex(encode(name, 'UTF-16BE')) AS h, decode(encode(name, 'UTF-8'), 'UTF-8') AS d FROM T",
]


def test_grouping_sets_after_group_list():
    assert q(SYNTAX_QUERIES[0])[0] == [(1, 1), (3, 1), (2, 2), (None, 4)]


def test_values_inline_tables():
    assert q(SYNTAX_QUERIES[1]) == ([(1, "x"), (2, "y")], ["a", "b"])
    assert q(SYNTAX_QUERIES[2]) == ([(1,), (3,)], ["p"])
    assert q("SELECT col1 FROM VALUES 1, 2") == ([(1,), (2,)], ["col1"])            # Spark's default names
    assert q("SELECT * FROM (SELECT 1, 2) AS v(p, q)") == ([(1, 2)], ["p", "q"])
    with pytest.raises(Exception, match="names 3 columns"):
        q("SELECT * FROM (SELECT 1, 2) AS v(p, q, r)")


def test_typed_literals():
    # T0 = 2019-02-28 23:00 UTC: rows at +0, +61 s, +1 h 0.123 s, +1 day → two before midnight
    assert q(SYNTAX_QUERIES[3])[0] == [(2,)]
    rows, names = q("SELECT datediff(DATE '2019-03-01', DATE '2019-02-01') AS d, DATE '2019-03-01', "
                    "TIMESTAMP '2019-03-01 00:00:00'")
    assert rows == [(28, dt.date(2019, 3, 1), dt.datetime(2019, 3, 1))]
    assert names == ["d", "DATE '2019-03-01'", "TIMESTAMP('2019-03-01 00:00:00')"]      # Literal.sql


def test_named_window_clause():
    # running SUM per id in ts order: id 2's first row has v NULL → NULL, then 4.0
    assert q(SYNTAX_QUERIES[4])[0] == [(1, 1.5), (2, None), (2, 4.0), (3, 3.25)]
    assert q(SYNTAX_QUERIES[5])[0] == [(1, 1, 1.5), (2, 2, 4.0), (2, 2, 4.0), (3, 4, 3.25)]


def test_order_by_struct():
    # field by field, a NULL field sorting below any value (so last under DESC)
    rows = q(SYNTAX_QUERIES[6])[0]
    assert [r[1] for r in rows] == [{"a": 3, "b": 3.25}, {"a": 2, "b": 4.0}, {"a": 2, "b": None},
                                    {"a": 1, "b": 1.5}]


def test_java_short_zone_ids():
    rows = q(SYNTAX_QUERIES[7])[0]
    # PST = America/Los_Angeles (UTC-8 in February), EST = fixed -05:00, CTT = Asia/Shanghai (+8)
    assert rows[0] == (dt.datetime(2019, 2, 28, 15), dt.datetime(2019, 3, 1, 4), dt.datetime(2019, 3, 1, 7))
    assert rows[3][0] == dt.datetime(2019, 3, 1, 15)


def test_map_and_array_builders():
    assert q("SELECT str_to_map('a:1,b:2') AS m, str_to_map('k=v;x=y', ';', '=') AS n")[0] == \
        [({"a": "1", "b": "2"}, {"k": "v", "x": "y"})]
    assert q("SELECT str_to_map('a:1,b') AS m")[0] == [({"a": "1", "b": None},)]          # no delimiter → NULL
    assert q("SELECT map_concat(map('a', 1), map('b', 2)) AS m")[0] == [({"a": 1, "b": 2},)]
    assert q("SELECT array_repeat('ab', 3) AS a, array_repeat('x', 0) AS b, array_repeat('x', -1) AS c, "
             "array_repeat('x', CAST(NULL AS INT)) AS d")[0] == [(["ab", "ab", "ab"], [], [], None)]
    # per row: 'a,b' has no 'c' key, 'c' maps to NULL (no ':'), NULL text → NULL map
    assert q(SYNTAX_QUERIES[8])[0] == [(1, [1, 1], None), (2, [2, 2], None), (3, [3, 3], None),
                                       (2, [2, 2], None)]


def test_encode_decode_binary():
    rows, _ = q("SELECT encode('héllo', 'UTF-8') AS a, hex(encode('hé', 'ISO-8859-1')) AS b, "
                "length(encode('hé', 'UTF-16')) AS c, decode(encode('hé', 'UTF-16LE'), 'UTF-16LE') AS d, "
                "typeof(encode('a', 'UTF-8')) AS t, base64(encode('hi', 'UTF-8')) AS e")
    # Java's UTF-16 encoder writes a big-endian BOM: FE FF 00 68 00 E9 → 6 bytes
    assert rows == [(b"h\xc3\xa9llo", "68E9", 6, "hé", "binary", "aGk=")]
    assert q(SYNTAX_QUERIES[9])[0] == [("0061002C0062", "a,b"), ("0063", "c"), (None, None),
                                       ("0061002C0062002C002C0064", "a,b,,d")]
    with pytest.raises(Exception, match="charset"):
        q("SELECT encode('a', 'EBCDIC') AS x")


def test_sentences_xpath_assert_true():
    assert q("SELECT sentences('Hi there! How are you?') AS s, sentences(NULL) AS n")[0] == \
        [([["Hi", "there"], ["How", "are", "you"]], None)]
    assert q("SELECT xpath_string('<a><b>x</b></a>', 'a/b') AS a, xpath_int('<a><b>3</b></a>', 'a/b') AS b, "
             "xpath('<a><b>1</b><b>2</b></a>', 'a/b/text()') AS c, "
             "xpath_double('<a><b>1.5</b><b>2</b></a>', 'sum(a/b)') AS d, "
             "xpath_boolean('<a><b/></a>', 'a/b') AS e")[0] == [("x", 3, ["1", "2"], 3.5, True)]
    assert q("SELECT assert_true(id > 0) AS a FROM T")[0] == [(None,)] * 4
    with pytest.raises(Exception, match="is not true"):
        q("SELECT assert_true(id > 1) AS a FROM T")


@pytest.mark.gpu
def test_spark24_syntax_gpu_match_cpu(gpu):
    """Same statements on the device (grouping-set expansion, typed-literal filter, window clause, struct sort,
    zone conversion, array / map builders, binary digests) = the CPU rows."""
    for sql in SYNTAX_QUERIES:
        assert q(sql, gpu) == q(sql, "cpu"), sql
