"""Spark's hash() (Murmur3Hash over the arguments, seed 42): pinned values Spark returns, the float / decimal
rules (HashExpression: floatToIntBits, unscaled decimals), and the device kernel (spark_hash.hip) against the host."""
import pytest
import torch

from dxa.engine.column import Table, column_from_pylist
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql
from dxa.engine.sqlfuncs import spark_hash_value


def _s32(h):
    return h - (1 << 32) if h >= (1 << 31) else h


def test_pinned_spark_values():
    # values Spark 2.4 / 3.x return for SELECT hash(...)
    assert _s32(spark_hash_value(1, "int", 42)) == -559580957
    assert _s32(spark_hash_value(1, "long", 42)) == -1712319331
    assert _s32(spark_hash_value("Spark", "string", 42)) == 228093765
    assert _s32(spark_hash_value(None, "int", 42)) == 42


def test_float_and_decimal_rules():
    import struct
    from dxa.engine.sqlfuncs import _hash_int, _hash_long
    # float hashes its 32-bit pattern (hashInt), not the double's
    assert spark_hash_value(1.5, "float", 42) == _hash_int(struct.unpack("<I", struct.pack("<f", 1.5))[0], 42)
    assert spark_hash_value(-0.0, "float", 42) == spark_hash_value(0.0, "float", 42)
    assert spark_hash_value(float("nan"), "double", 42) == _hash_long(0x7FF8000000000000, 42)
    # decimal(p, s): hashLong of the unscaled value AT THE COLUMN'S SCALE for p <= 18 (12.34 as decimal(10,2) →
    # 1234; 7 as decimal(10,2) → 700), the BigInteger's bytes above that
    from decimal import Decimal
    from dxa.engine.decimal import DecimalType
    from dxa.engine.sqlfuncs import _hash_bytes
    assert spark_hash_value(1234, DecimalType(10, 2), 42) == _hash_long(1234, 42)
    assert spark_hash_value(Decimal("7"), DecimalType(10, 2), 42) == _hash_long(700, 42)
    assert spark_hash_value(Decimal("1.25"), DecimalType(10, 2), 42) == 1910520950       # hashLong(125, 42)
    assert spark_hash_value([125, 0], DecimalType(20, 2), 42) == _hash_bytes(bytes([125]), 42)
    assert spark_hash_value([-1, -1], DecimalType(20, 2), 42) == _hash_bytes(bytes([0xFF]), 42)   # -1


def test_decimal_hash_in_sql():
    from dxa.engine.column import Table
    from dxa.engine.expr import EvalContext
    from dxa.engine.query import Catalog, run_sql
    from dxa.engine.types import StructField, StructType
    cat = Catalog()
    cat.register("T", Table.from_pylist([{"k": 1}], StructType((StructField("k", "long"),))))
    out = run_sql("SELECT hash(CAST(1.25 AS DECIMAL(10,2))) AS h, hash(CAST(k AS DECIMAL(10,2))) AS h2 FROM T", cat,
                  EvalContext()).to_pylist()
    assert out == [{"h": 1910520950, "h2": _hl(100)}]


def _hl(v):
    from dxa.engine.sqlfuncs import _hash_long
    r = _hash_long(v, 42)
    return r - (1 << 32) if r >= (1 << 31) else r


@pytest.mark.gpu
def test_hash_device_matches_host(gpu):
    import random
    rnd = random.Random(5)
    n = 5000
    data = {
        "i": ([rnd.choice([None, rnd.randint(-2**31, 2**31 - 1)]) for _ in range(n)], "int"),
        "l": ([rnd.choice([None, rnd.randint(-2**63, 2**63 - 1)]) for _ in range(n)], "long"),
        "d": ([rnd.choice([None, 0.0, -0.0, float("nan"), rnd.uniform(-1e9, 1e9)]) for _ in range(n)], "double"),
        "f": ([rnd.choice([None, -0.0, 1.5, rnd.uniform(-1e3, 1e3)]) for _ in range(n)], "float"),
        "b": ([rnd.choice([None, True, False]) for _ in range(n)], "boolean"),
        "s": ([rnd.choice([None, "", "a", "Spark", "ünï", "x" * rnd.randint(0, 40)]) for _ in range(n)], "string"),
        "t": ([rnd.choice([None, rnd.randint(0, 2**50)]) for _ in range(n)], "timestamp"),
    }
    sql = "SELECT hash(i) AS a, hash(l, s) AS b, hash(d, f, b) AS c, hash(s, t, i, 'k', 7) AS e FROM T"
    out = {}
    for dev in (gpu, torch.device("cpu")):
        cols = [column_from_pylist(v, t, dev) for v, t in data.values()]
        cat = Catalog()
        cat.register("T", Table(list(data), cols, n, dev))
        out[dev.type] = [c.to_pylist() for c in run_sql(sql, cat, EvalContext(device=dev)).columns]
    assert out["cuda"] == out["cpu"]
