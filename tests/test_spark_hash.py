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
    # decimal: the unscaled value (12.34 → 1234)
    assert spark_hash_value(12.34, "decimal", 42) == _hash_long(1234, 42)
    assert spark_hash_value(7.0, "decimal", 42) == _hash_long(7, 42)


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
