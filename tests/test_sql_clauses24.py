"""Spark 2.4 clauses the reference's user SQL may use (it runs arbitrary ``spark.sql``, CommonProcessorFactory.scala:
257-275 on Spark 2.4.5, datax-host/pom.xml:57): PIVOT, NATURAL JOIN, DISTRIBUTE BY / SORT BY / CLUSTER BY,
TABLESAMPLE and ``/*+ … */`` hints.  Expected rows are hand-computed from Spark's documented semantics (pyspark is
not importable here: parity unpinned beyond those documents); a 2-rank gloo run checks the distributed paths and a
GPU differential checks the device paths against the CPU evaluator."""
import os
import socket
import traceback

import pytest
import torch
import torch.multiprocessing as mp

from dxa.engine.column import Table
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql
from dxa.engine.types import StructField, StructType
from dxa.sql.parser import SqlError, parse_query

S = StructType((StructField("k", "long"), StructField("s", "string"), StructField("v", "double")))
ROWS = [{"k": 1, "s": "a", "v": 1.0}, {"k": 1, "s": "bb", "v": 2.0}, {"k": 2, "s": "a", "v": 3.0},
        {"k": 2, "s": None, "v": 4.0}, {"k": 3, "s": "bb", "v": 5.0}]
S2 = StructType((StructField("k", "long"), StructField("name", "string")))
ROWS2 = [{"k": 1, "name": "one"}, {"k": 3, "name": "three"}, {"k": 4, "name": "four"}]


def _cat(device="cpu", rows=ROWS, rows2=ROWS2):
    cat = Catalog()
    cat.register("T", Table.from_pylist(rows, S, device))
    cat.register("T2", Table.from_pylist(rows2, S2, device))
    return cat


def _rows(t):
    return [tuple(c.to_pylist()[i] for c in t.columns) for i in range(t.length)]


def qq(sql, device="cpu"):
    out = run_sql(sql, _cat(device), EvalContext(device=torch.device(device)))
    return out.names, _rows(out)


# ---- PIVOT ----------------------------------------------------------------------------------------------------

def test_pivot_single_aggregate_names_columns_by_value():
    names, rows = qq("SELECT * FROM T PIVOT (SUM(v) FOR s IN ('a', 'bb' AS b2, NULL))")
    assert names == ["k", "a", "b2", "null"]          # group by every column the pivot does not read
    assert sorted(rows) == [(1, 1.0, 2.0, None), (2, 3.0, None, 4.0), (3, None, 5.0, None)]


def test_pivot_several_aggregates_and_count_nulls():
    names, rows = qq("SELECT * FROM T PIVOT (SUM(v) AS sv, COUNT(*) AS c FOR s IN ('a', 'bb'))")
    assert names == ["k", "a_sv", "a_c", "bb_sv", "bb_c"]
    # a group without rows for a value is NULL there, COUNT included (Spark's two-phase PivotFirst)
    assert sorted(rows) == [(1, 1.0, 1, 2.0, 1), (2, 3.0, 1, None, None), (3, None, None, 5.0, 1)]


def test_pivot_unaliased_aggregate_suffix_and_subquery_source():
    names, rows = qq("SELECT * FROM (SELECT k, s, v FROM T WHERE k < 3) t PIVOT (MAX(v), MIN(v) FOR s IN ('a'))")
    assert names == ["k", "a_max(v)", "a_min(v)"]
    assert sorted(rows) == [(1, 1.0, 1.0), (2, 3.0, 3.0)]


def test_pivot_multi_column_values():
    names, rows = qq("SELECT * FROM T PIVOT (MAX(v) FOR (k, s) IN ((1, 'a') AS x, (2, 'a')))")
    assert names == ["x", "[2,a]"] and rows == [(1.0, 3.0)]


def test_pivot_then_where_and_order():
    names, rows = qq("SELECT k, a FROM T PIVOT (SUM(v) FOR s IN ('a')) p WHERE p.a IS NOT NULL ORDER BY k DESC")
    assert rows == [(2, 3.0), (1, 1.0)]


def test_pivot_rejects_non_aggregate():
    with pytest.raises(Exception, match="aggregate"):
        qq("SELECT * FROM T PIVOT (v FOR s IN ('a'))")


# ---- NATURAL JOIN / USING ---------------------------------------------------------------------------------------

def test_natural_join_lists_common_columns_once():
    names, rows = qq("SELECT * FROM T NATURAL JOIN T2")
    assert names == ["k", "s", "v", "name"]
    assert sorted(rows) == [(1, "a", 1.0, "one"), (1, "bb", 2.0, "one"), (3, "bb", 5.0, "three")]


def test_natural_full_join_merges_keys_with_coalesce():
    names, rows = qq("SELECT * FROM T2 NATURAL FULL OUTER JOIN T")
    assert names == ["k", "name", "s", "v"]
    assert sorted(rows, key=repr) == sorted([(1, "one", "a", 1.0), (1, "one", "bb", 2.0), (3, "three", "bb", 5.0),
                                             (4, "four", None, None), (2, None, "a", 3.0), (2, None, None, 4.0)],
                                            key=repr)


def test_using_join_keeps_sides_reachable_qualified():
    names, rows = qq("SELECT T.k, T2.k, k, name FROM T LEFT JOIN T2 USING (k) ORDER BY v")
    assert rows == [(1, 1, 1, "one"), (1, 1, 1, "one"), (2, None, 2, None), (2, None, 2, None),
                    (3, 3, 3, "three")]
    names, rows = qq("SELECT * FROM T RIGHT JOIN T2 USING (k) ORDER BY k, v")
    assert names == ["k", "s", "v", "name"]
    assert rows == [(1, "a", 1.0, "one"), (1, "bb", 2.0, "one"), (3, "bb", 5.0, "three"), (4, None, None, "four")]


def test_natural_join_without_common_columns_is_cross():
    out = run_sql("SELECT * FROM (SELECT k AS a FROM T2) x NATURAL JOIN (SELECT name FROM T2) y", _cat(),
                  EvalContext())
    assert out.length == 9


# ---- DISTRIBUTE BY / SORT BY / CLUSTER BY -----------------------------------------------------------------------

def test_sort_by_on_one_partition_orders_everything():
    assert qq("SELECT k, v FROM T SORT BY v DESC")[1] == [(3, 5.0), (2, 4.0), (2, 3.0), (1, 2.0), (1, 1.0)]
    assert qq("SELECT k, v FROM T DISTRIBUTE BY k SORT BY k DESC, v")[1] == \
        [(3, 5.0), (2, 3.0), (2, 4.0), (1, 1.0), (1, 2.0)]
    assert qq("SELECT k, v AS x FROM T CLUSTER BY x")[1] == [(1, 1.0), (1, 2.0), (2, 3.0), (2, 4.0), (3, 5.0)]
    assert sorted(qq("SELECT k FROM T DISTRIBUTE BY k")[1]) == [(1,), (1,), (2,), (2,), (3,)]


def test_order_by_with_sort_by_is_an_error():
    with pytest.raises(SqlError):
        parse_query("SELECT k FROM T ORDER BY k SORT BY k")


# ---- TABLESAMPLE --------------------------------------------------------------------------------------------------

def test_tablesample_rows_and_fractions():
    assert qq("SELECT * FROM T TABLESAMPLE (2 ROWS)")[1] == [(1, "a", 1.0), (1, "bb", 2.0)]
    assert qq("SELECT COUNT(*) FROM T TABLESAMPLE (100 PERCENT)")[1] == [(5,)]
    assert qq("SELECT COUNT(*) FROM T TABLESAMPLE (0 PERCENT)")[1] == [(0,)]
    assert qq("SELECT COUNT(*) FROM T TABLESAMPLE (BUCKET 3 OUT OF 3) x")[1] == [(5,)]
    with pytest.raises(SqlError):
        parse_query("SELECT * FROM T TABLESAMPLE (150 PERCENT)")


def test_tablesample_fraction_is_deterministic_and_near_the_rate():
    rows = [{"k": i, "s": None, "v": float(i)} for i in range(20000)]
    cat = Catalog()
    cat.register("T", Table.from_pylist(rows, S))
    a = run_sql("SELECT k FROM T TABLESAMPLE (25 PERCENT)", cat, EvalContext()).to_pylist()
    b = run_sql("SELECT k FROM T TABLESAMPLE (BUCKET 1 OUT OF 4)", cat, EvalContext()).to_pylist()
    assert a == b                                        # same fraction, same seed: same rows, every run
    assert 0.23 < len(a) / 20000 < 0.27


# ---- hints ------------------------------------------------------------------------------------------------------

def test_hints_and_comments_are_accepted():
    names, rows = qq("SELECT /*+ BROADCAST(b) */ a.k, b.name FROM T a JOIN T2 b ON a.k = b.k ORDER BY a.v")
    assert rows == [(1, "one"), (1, "one"), (3, "three")]
    assert qq("SELECT /*+ COALESCE(3), REPARTITION(2) */ /* a comment */ COUNT(*) FROM T")[1] == [(5,)]
    assert qq("SELECT /*+ MAPJOIN(T2) SHUFFLE_HASH(T) */ COUNT(*) FROM T JOIN T2 ON T.k = T2.k")[1] == [(3,)]
    j = parse_query("SELECT /*+ BROADCASTJOIN(x) */ * FROM T JOIN T2 x ON T.k = x.k").body.from_
    assert j.broadcast == {"x"}


# ---- distributed (2 gloo ranks) ---------------------------------------------------------------------------------

DIST_QUERIES = [
    "SELECT * FROM T PIVOT (SUM(v) AS sv, COUNT(*) AS c FOR s IN ('a', 'bb', NULL))",
    "SELECT * FROM T NATURAL JOIN T2",
    "SELECT * FROM T NATURAL LEFT JOIN T2",
    "SELECT /*+ BROADCAST(b) */ a.k, a.v, b.name FROM T a JOIN T2 b ON a.k = b.k",
    "SELECT /*+ BROADCAST(a) */ a.k, a.v, b.name FROM T a JOIN T2 b ON a.k = b.k",
    "SELECT k, v FROM T DISTRIBUTE BY k",
    "SELECT k, SUM(v) AS sv FROM T GROUP BY k CLUSTER BY k",
]


def _big_rows(n=300):
    return [{"k": i % 17, "s": ["a", "bb", None][i % 3], "v": float(i % 23)} for i in range(n)]


def _big_rows2():
    return [{"k": k, "name": f"n{k}"} for k in range(0, 17, 2)]


def _canon(rows):
    return sorted((tuple((k, round(v, 6) if isinstance(v, float) else v) for k, v in sorted(r.items()))
                   for r in rows), key=repr)


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dxa import parallel as P
        P.init(dist.group.WORLD, "cpu")
        cat = Catalog()
        t = Table.from_pylist(_big_rows()[rank::world], S)
        t.dist = P.PARTITIONED
        t2 = Table.from_pylist(_big_rows2()[rank::world], S2)
        t2.dist = P.PARTITIONED
        cat.register("T", t)
        cat.register("T2", t2)
        res = []
        for sql in DIST_QUERIES:
            out = run_sql(sql, cat, EvalContext())
            local_sorted = None
            if "CLUSTER BY" in sql:
                ks = [r["k"] for r in out.to_pylist()]
                local_sorted = ks == sorted(ks)
                owners = set(int(x) for x in P.owner_of(
                    __import__("dxa.ops.hashing", fromlist=["hash_columns"]).hash_columns([out.column("k")])
                ).tolist()) if out.length else set()
                local_sorted = local_sorted and owners <= {rank}
            if P.dist_of(out) != P.REPLICATED:
                out = P.allgather_table(out)
            res.append((out.names, out.to_pylist(), local_sorted))
        q.put((rank, res, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_clauses_two_ranks_match_one():
    from dxa import parallel as P
    P.shutdown()
    ctx = mp.get_context("spawn")
    q_ = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q_)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, r, err = q_.get(timeout=240)
        assert err is None, err
        res[rank] = r
    for p in procs:
        p.join(timeout=60)
    cat = _cat(rows=_big_rows(), rows2=_big_rows2())
    for i, sql in enumerate(DIST_QUERIES):
        want = run_sql(sql, cat, EvalContext())
        for r in (0, 1):
            names, rows, local_sorted = res[r][i]
            assert names == want.names, (sql, names)
            assert _canon(rows) == _canon(want.to_pylist()), sql
            if local_sorted is not None:
                assert local_sorted, (sql, r)          # each rank holds only its own keys, sorted


# ---- GPU differential -------------------------------------------------------------------------------------------

GPU_QUERIES = [
    "SELECT * FROM T PIVOT (SUM(v) AS sv, COUNT(*) AS c FOR s IN ('a', 'bb', NULL))",
    "SELECT * FROM T NATURAL FULL OUTER JOIN T2",
    "SELECT k, v FROM T DISTRIBUTE BY k SORT BY k DESC, v",
    "SELECT COUNT(*), SUM(v) FROM T TABLESAMPLE (30 PERCENT)",
    "SELECT /*+ BROADCAST(b) */ a.k, b.name FROM T a JOIN T2 b USING (k)",
]


@pytest.mark.gpu
@pytest.mark.parametrize("sql", GPU_QUERIES)
def test_clauses_gpu_match_cpu(gpu, sql):
    cg, cc = _cat(gpu, _big_rows(5000), _big_rows2()), _cat("cpu", _big_rows(5000), _big_rows2())
    g = run_sql(sql, cg, EvalContext(device=gpu))
    c = run_sql(sql, cc, EvalContext())
    assert g.names == c.names
    if "SORT BY" in sql:
        assert _rows(g) == _rows(c)
    else:
        assert _canon(g.to_pylist()) == _canon(c.to_pylist())
