"""Exact Spark DecimalType(p, s) (dxa/engine/decimal.py, dxa/ops/csrc/decimal.hip).

The reference's input schemas are Spark ``DataType.fromJson`` documents (datax-host/.../input/SchemaFile.scala:25) and
SimulatedData emits ``decimal`` fields (DataX.SimulatedData.DataGenService/DataGen.cs:162,195).  Expected values come
from Spark 2.4's documented decimal rules (DecimalPrecision, Decimal.changePrecision with ROUND_HALF_UP, NULL on
overflow, BigDecimal.toString rendering) and from Python's ``decimal`` module over the same inputs; pyspark is not
importable here, so parity beyond those documents is unpinned."""
import decimal
import json
import os

import pytest
import torch

from dxa.engine.column import Table
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql
from dxa.engine.types import StructField, StructType

Dec = decimal.Decimal

S = StructType((StructField("k", "long"),))


def _q(expr, device="cpu"):
    cat = Catalog()
    cat.register("T", Table.from_pylist([{"k": 1}], S, device))
    out = run_sql(f"SELECT {expr} AS x FROM T", cat, EvalContext(device=torch.device(device)))
    c = out.columns[0]
    return str(c.dtype), c.to_pylist()[0]


PROBES = [
    # the round-3 verdict's probe expressions
    ("CAST(0.1 AS DECIMAL(10,2)) + CAST(0.2 AS DECIMAL(10,2))", "decimal(11,2)", Dec("0.30")),
    ("to_json(named_struct('d', CAST(12.3 AS DECIMAL(10,2))))", "string", '{"d":12.30}'),
    ("CAST(2.345 AS DECIMAL(10,2))", "decimal(10,2)", Dec("2.35")),
    ("CAST(12345 AS DECIMAL(4,0))", "decimal(4,0)", None),
    ("CAST(123456789012345678.12 AS DECIMAL(38,2))", "decimal(38,2)", Dec("123456789012345678.12")),
    # literals are decimals of their own digits; integers widen to decimal(10,0) / decimal(20,0)
    ("0.1 + 0.2", "decimal(2,1)", Dec("0.3")),
    ("k * 1.5", "decimal(23,1)", Dec("1.5")),
    ("CAST(k AS DECIMAL(10,2)) / 3", "decimal(14,6)", Dec("0.333333")),       # 3 → decimal(1,0) (fromLiteral)
    ("CAST(k AS DECIMAL(10,2)) / k", "decimal(31,23)", Dec("1.00000000000000000000000")),  # long → (20,0)
    ("-CAST(k AS DECIMAL(38,10)) * 2.5", "decimal(38,8)", Dec("-2.50000000")),
    ("CAST(-2.5 AS DECIMAL(3,1)) * CAST(-2.5 AS DECIMAL(3,1))", "decimal(7,2)", Dec("6.25")),
    ("CAST(7.5 AS DECIMAL(3,1)) % 2", "decimal(2,1)", Dec("1.5")),
    ("CAST(1 AS DECIMAL(38,0)) / 0", None, None),
    ("CAST(CAST(k AS DECIMAL(38,2)) + 123456789012345678901234567.5 AS STRING)", "string",
     "123456789012345678901234568.50"),
    ("CAST(CAST(0.0000001 AS DECIMAL(8,7)) AS STRING)", "string", "1E-7"),
    ("CAST(' 12.345 ' AS DECIMAL(5,2))", "decimal(5,2)", Dec("12.35")),
    ("CAST('1e2' AS DECIMAL(5,1))", "decimal(5,1)", Dec("100.0")),
    ("CAST('abc' AS DECIMAL(5,1))", "decimal(5,1)", None),
    ("CAST(2.5 AS DECIMAL(3,1)) > 2.49", "boolean", True),
    ("CAST(2.5 AS DECIMAL(3,1)) = 2.5", "boolean", True),
    ("CAST(k AS DECIMAL(38,5)) < 0.5", "boolean", False),
    ("CAST(-7.99 AS DECIMAL(4,2)) + 0", "decimal(5,2)", Dec("-7.99")),
    ("CAST(CAST(-7.99 AS DECIMAL(4,2)) AS INT)", "int", -7),
    ("CAST(CAST(2.5 AS DECIMAL(3,1)) AS DOUBLE) * 2", "double", 5.0),
    ("CAST(2.5 AS DECIMAL(3,1)) * 2.0D", "double", 5.0),
    ("IF(k > 0, CAST(k AS DECIMAL(5,1)), 0.25)", "decimal(6,2)", Dec("1.00")),
    ("abs(CAST(-3.25 AS DECIMAL(4,2)))", "decimal(4,2)", Dec("3.25")),
    ("sqrt(CAST(6.25 AS DECIMAL(4,2)))", "double", 2.5),
    ("CAST(99999999999999999999999999999999999999 AS DECIMAL(38,0)) + 1", "decimal(38,0)", None),
]


def _device_params():
    return ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("device", _device_params())
def test_probe_expressions(device):
    bad = []
    for expr, t, v in PROBES:
        got_t, got = _q(expr, device)
        if (t is not None and got_t != t) or got != v:
            bad.append((expr, got_t, got, t, v))
    assert not bad, bad


def test_column_arithmetic_matches_python_decimal():
    import random
    rnd = random.Random(4)
    rows = []
    for i in range(400):
        a = Dec(rnd.randrange(-10**9, 10**9)).scaleb(-2)
        b = Dec(rnd.randrange(-10**6, 10**6)).scaleb(-3)
        w = Dec(rnd.randrange(-10**30, 10**30)).scaleb(-5)
        rows.append({"a": str(a), "b": str(b), "w": str(w)})
    st = StructType((StructField("a", "string"), StructField("b", "string"), StructField("w", "string")))
    cat = Catalog()
    cat.register("T", Table.from_pylist(rows, st, "cpu"))
    out = run_sql("SELECT CAST(a AS DECIMAL(11,2)) + CAST(b AS DECIMAL(9,3)) AS s, "
                  "CAST(a AS DECIMAL(11,2)) * CAST(b AS DECIMAL(9,3)) AS m, "
                  "CAST(w AS DECIMAL(38,5)) - CAST(a AS DECIMAL(11,2)) AS d, "
                  "CAST(w AS DECIMAL(38,5)) < CAST(a AS DECIMAL(11,2)) AS lt FROM T", cat,
                  EvalContext(device=torch.device("cpu")))
    got = out.to_pylist()
    assert str(out.columns[0].dtype) == "decimal(13,3)" and str(out.columns[1].dtype) == "decimal(21,5)"
    assert str(out.columns[2].dtype) == "decimal(38,5)"
    for r, g in zip(rows, got):
        a, b, w = Dec(r["a"]), Dec(r["b"]), Dec(r["w"])
        assert g["s"] == a + b and g["m"] == a * b and g["d"] == w - a and g["lt"] == (w < a)


@pytest.mark.parametrize("device", _device_params())
def test_json_parse_exact(device):
    from dxa.ops import jsonparse as JP
    schema = StructType((StructField("p", "decimal(10,2)"), StructField("w", "decimal(38,6)"),
                         StructField("d", "double")))
    schema = StructType(tuple(StructField(f.name, _t(f.dtype)) for f in schema.fields))
    recs = [b'{"p": 12.345, "w": 123456789012345678901234.5678905, "d": 0.1}',
            b'{"p": -0.005, "w": -1e-7, "d": 1}',
            b'{"p": 123456789.99, "w": 1E+5, "d": 2.5}',          # 11 digits at scale 2 > precision 10 → null
            b'{"p": "12.5", "w": 0, "d": null}',                   # strings are not decimals (Spark 2.4 JSON)
            b'{"p": 99999999.995, "w": 12.0000005}']               # rounds up past precision → null
    buf, offs = JP.frame_records(recs, device)
    root, ok = JP.parse(buf, offs, JP.ParsePlan(schema))
    p = root.children[0].to_pylist()
    w = root.children[1].to_pylist()
    d = root.children[2].to_pylist()
    assert p == [Dec("12.35"), Dec("-0.01"), None, None, None]
    assert w == [Dec("123456789012345678901234.567891"), Dec("-0.000000"), Dec("100000.000000"),
                 Dec("0.000000"), Dec("12.000001")]
    assert d[:3] == [0.1, 1.0, 2.5]


def _t(s):
    from dxa.engine.types import from_json_obj
    return from_json_obj(s)


@pytest.mark.parametrize("device", _device_params())
def test_serializers_render_scale(device):
    from dxa.engine.serialize import table_to_json_lines
    dt = _t("decimal(10,2)")
    cat = Catalog()
    cat.register("T", Table.from_pylist([{"k": 1}, {"k": -20}, {"k": 0}], S, device))
    out = run_sql("SELECT k, CAST(k AS DECIMAL(10,2)) / 8 AS q, CAST(k AS DECIMAL(38,3)) AS w FROM T", cat,
                  EvalContext(device=torch.device(device)))
    lines = [json.loads(x, parse_float=Dec) for x in table_to_json_lines(out)]
    txt = table_to_json_lines(out)
    assert '"q":0.125000' in txt[0], txt[0]                  # decimal(10,2) / decimal(1,0) → decimal(14,6)
    assert [r["w"] for r in lines] == [Dec("1.000"), Dec("-20.000"), Dec("0.000")]
    assert '"w":-20.000' in txt[1] and '"w":0.000' in txt[2]
    del dt


def _decimal_flow(workdir, device, n_events=3000, batches=3):
    """A SimulatedData stream with a decimal(10,2) price field through a GROUP BY flow (Processor end to end)."""
    from dxa.config.settings import SettingDictionary
    from dxa.engine.processor import Processor, RawBatch
    from dxa.engine.types import schema_to_json
    from dxa.io import sinks
    from dxa.ops import jsonparse as JP
    from dxa.simulate.simulated_data import DataGen
    fields = [{"name": "deviceId", "type": "int", "minRange": 1, "maxRange": 40},
              {"name": "price", "type": "decimal", "minRange": 0, "maxRange": 1000},
              {"name": "qty", "type": "long", "minRange": 1, "maxRange": 9}]
    schema = StructType((StructField("deviceId", "long"), StructField("price", _t("decimal(10,2)")),
                         StructField("qty", "long")))
    paths = {k: os.path.join(workdir, k) for k in ("schema.json", "projection.txt", "transform.txt")}
    with open(paths["schema.json"], "w") as f:
        f.write(schema_to_json(schema))
    with open(paths["projection.txt"], "w") as f:
        f.write("Raw.*\n")
    with open(paths["transform.txt"], "w") as f:
        f.write("--DataXQuery--\nSales = SELECT deviceId, SUM(price) AS total, AVG(price) AS mean, MAX(price) AS hi, "
                "MIN(price) AS lo, SUM(price * qty) AS revenue, COUNT(*) AS n FROM DataXProcessedInput "
                "GROUP BY deviceId\n")
    settings = SettingDictionary({
        "datax.job.name": "decimalflow",
        "datax.job.input.default.blobschemafile": paths["schema.json"],
        "datax.job.input.default.streaming.intervalinseconds": "1",
        "datax.job.process.projection": paths["projection.txt"],
        "datax.job.process.transform": paths["transform.txt"],
        "datax.job.output.Sales.memory.enabled": "true",
    })
    gen = DataGen(seed=11)
    ds = {"fields": fields, "numEventsPerBatch": n_events}
    sinks.MEMORY_SINKS.clear()
    proc = Processor(settings, torch.device(device))
    all_events, results = [], []
    for b in range(batches):
        evs = [gen.random_event(ds).encode() for _ in range(n_events)]
        all_events.append(evs)
        buf, offs = JP.frame_records(evs, device)
        proc.process_batch(RawBatch(buf, offs, n_events), 1_600_000_000_000_000 + b * 1_000_000, 1_000_000)
        proc.drain()
        results.append([json.loads(x, parse_float=Dec) if isinstance(x, str) else x
                        for x in sinks.MEMORY_SINKS.get("Sales", [])])
        sinks.MEMORY_SINKS.clear()
    return all_events, results


def _expected(events):
    q2 = Dec("0.01")
    groups = {}
    for e in events:
        d = json.loads(e, parse_float=Dec)
        p = Dec(d["price"]).quantize(q2, rounding=decimal.ROUND_HALF_UP)
        g = groups.setdefault(d["deviceId"], [])
        g.append((p, d["qty"]))
    out = {}
    for k, v in groups.items():
        ps = [p for p, _ in v]
        tot = sum(ps)
        mean = (tot / len(ps)).quantize(Dec("0.000001"), rounding=decimal.ROUND_HALF_UP)
        out[k] = {"deviceId": k, "total": tot, "mean": mean, "hi": max(ps), "lo": min(ps),
                  "revenue": sum(p * q for p, q in v), "n": len(v)}
    return out


@pytest.mark.parametrize("device", _device_params())
def test_simulated_decimal_groupby_flow(tmp_path, device):
    events, results = _decimal_flow(str(tmp_path), device)
    for evs, rows in zip(events, results):
        exp = _expected(evs)
        assert len(rows) == len(exp)
        for r in rows:
            e = exp[r["deviceId"]]
            for k in ("total", "mean", "hi", "lo", "revenue", "n"):
                assert r[k] == e[k], (k, r, e)
        # rendering: the scale's digits are all printed (sum: decimal(20,2); avg: decimal(14,6))
        assert all(len(str(r["total"]).split(".")[1]) == 2 and len(str(r["mean"]).split(".")[1]) == 6
                   for r in rows)


@pytest.mark.gpu
def test_decimal_literal_next_to_double_still_fuses():
    """``x > 44.99`` (a decimal literal beside a double column) compares in double, and the JIT keeps it fused."""
    from dxa.engine import jit
    n = 1 << 17
    st = StructType((StructField("x", "double"), StructField("k", "long")))
    cat = Catalog()
    from dxa.engine.column import PrimColumn
    x = torch.linspace(40, 50, n, dtype=torch.float64, device="cuda")
    cat.register("T", Table(["x", "k"], [PrimColumn("double", x),
                                         PrimColumn("long", torch.arange(n, device="cuda"))], n, "cuda"))
    before = dict(jit.STATS)
    out = run_sql("SELECT k FROM T WHERE x > 44.99 AND x * 1.5 < 73.5", cat, EvalContext(device=torch.device("cuda")))
    assert jit.STATS["fused"] > before["fused"]
    ref = ((x > 44.99) & (x * 1.5 < 73.5)).sum().item()
    assert out.length == ref
    del st


# ---- distributed: decimals through the exchange (narrow: one int64 leaf; wide: (lo, hi) leaves) -------------------

DIST_S = StructType((StructField("g", "long"), StructField("a", "string"), StructField("w", "string")))
DIST_QUERIES = [
    "SELECT g, SUM(CAST(a AS DECIMAL(10,2))) AS s, AVG(CAST(a AS DECIMAL(10,2))) AS m, "
    "MAX(CAST(w AS DECIMAL(38,4))) AS hi, MIN(CAST(w AS DECIMAL(38,4))) AS lo, SUM(CAST(w AS DECIMAL(38,4))) AS sw "
    "FROM T GROUP BY g",
    "SELECT CAST(w AS DECIMAL(38,4)) AS d, COUNT(*) AS c FROM T GROUP BY CAST(w AS DECIMAL(38,4))",
    "SELECT x.g, x.d, y.d AS d2 FROM (SELECT g, CAST(a AS DECIMAL(10,2)) AS d FROM T) x "
    "JOIN (SELECT g, CAST(w AS DECIMAL(38,4)) AS d FROM T) y ON x.d = y.d",
]


def _dist_rows():
    import random
    rnd = random.Random(9)
    rows = []
    for i in range(600):
        a = Dec(rnd.randrange(-10**6, 10**6)).scaleb(-2)
        w = Dec(rnd.choice([rnd.randrange(-10**30, 10**30), int(a * 100)])).scaleb(-2 if rnd.random() < .5 else -4)
        rows.append({"g": rnd.randrange(15), "a": str(a), "w": str(w) if rnd.random() > .05 else None})
    return rows


def _canon(rows):
    return sorted(repr(sorted(r.items())) for r in rows)


def _dist_worker(rank, world, port, q):
    import traceback
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dxa import parallel as P
        P.init(dist.group.WORLD, "cpu")
        cat = Catalog()
        t = Table.from_pylist(_dist_rows()[rank::world], DIST_S)
        t.dist = P.PARTITIONED
        cat.register("T", t)
        res = []
        for sql in DIST_QUERIES:
            out = run_sql(sql, cat, EvalContext())
            if P.dist_of(out) != P.REPLICATED:
                out = P.allgather_table(out)
            res.append([str(c.dtype) for c in out.columns] and (out.names, out.to_pylist()))
        q.put((rank, res, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def test_decimals_two_ranks_match_one():
    import socket
    import torch.multiprocessing as mp
    from dxa import parallel as P
    P.shutdown()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q_ = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q_)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, r, err = q_.get(timeout=240)
        assert err is None, err
        res[rank] = r
    for p in procs:
        p.join(timeout=60)
    cat = Catalog()
    cat.register("T", Table.from_pylist(_dist_rows(), DIST_S))
    for i, sql in enumerate(DIST_QUERIES):
        want = run_sql(sql, cat, EvalContext())
        assert want.length > 0
        for r in (0, 1):
            names, rows = res[r][i]
            assert names == want.names
            assert _canon(rows) == _canon(want.to_pylist()), sql


@pytest.mark.parametrize("device", _device_params())
def test_order_by_and_window_over_decimals(device):
    rows = [{"a": v} for v in ["3.5", "-1.25", None, "1e20", "-1e20", "0.001", "3.5", "-0.0001"]]
    st = StructType((StructField("a", "string"),))
    cat = Catalog()
    cat.register("T", Table.from_pylist(rows, st, device))
    ctx = EvalContext(device=torch.device(device))
    out = run_sql("SELECT CAST(a AS DECIMAL(38,4)) AS w, CAST(a AS DECIMAL(8,4)) AS n FROM T "
                  "ORDER BY w DESC NULLS LAST", cat, ctx).to_pylist()
    assert [r["w"] for r in out] == [Dec("1e20"), Dec("3.5"), Dec("3.5"), Dec("0.001"), Dec("-0.0001"),
                                     Dec("-1.25"), Dec("-1e20"), None]
    out = run_sql("SELECT n, ROW_NUMBER() OVER (ORDER BY n) AS r, SUM(n) OVER (ORDER BY n ROWS BETWEEN "
                  "UNBOUNDED PRECEDING AND CURRENT ROW) AS s FROM (SELECT CAST(a AS DECIMAL(8,4)) AS n FROM T) "
                  "WHERE n IS NOT NULL", cat, ctx).to_pylist()
    assert [r["n"] for r in sorted(out, key=lambda r: r["r"])] == sorted(r["n"] for r in out)
