"""The device serializer's cached render plans (ops/serialize._plan_of): a batch whose outputs have the shape of an
earlier batch's reuses that plan's node array, program and text, with only the buffer pointers patched — the blob
must equal what the builder walk (``_build_plan``) produces for the same columns.  CPU tensors: the plan is host-side
bookkeeping, the pointers are just addresses."""
import numpy as np
import torch

from dxa.engine.decimal import parse_decimal_type
from dxa.engine.column import ConstColumn, PrimColumn, StrColumn, Table
from dxa.ops import serialize as S


class _M:
    def __init__(self, t):
        self.table, self.n = t, t.length


def _table(n, seed):
    g = torch.Generator().manual_seed(seed)
    valid = torch.rand(n, generator=g) > 0.2
    s = StrColumn(torch.randint(65, 90, (n * 4,), dtype=torch.uint8, generator=g),
                  torch.arange(n, dtype=torch.int32) * 4, torch.full((n,), 4, dtype=torch.int32), valid)
    cols = [PrimColumn("long", torch.arange(n, dtype=torch.int64)),
            PrimColumn("int", torch.arange(n, dtype=torch.int32), valid),
            s,
            PrimColumn("double", torch.rand(n, dtype=torch.float64, generator=g)),
            PrimColumn("boolean", torch.rand(n, generator=g) > 0.5),
            PrimColumn("timestamp", torch.arange(n, dtype=torch.int64) * 1000),
            ConstColumn("iot", "string", n, "cpu")]
    return Table(["a", "b", "c", "d", "e", "f", "g"], cols, n, "cpu")


def _fresh(members):
    plan, keep = S._build_plan(members)
    return bytes(plan[0]), plan[1:], keep


def test_cached_plan_equals_builder_walk():
    S._PLANS.clear()
    first = [_M(_table(50, 1)), _M(_table(30, 2))]
    plan1, _ = S._plan_of(first)                   # miss: builds and caches
    assert len(S._PLANS) == 1
    second = [_M(_table(70, 3)), _M(_table(20, 4))]
    plan2, keep = S._plan_of(second)               # hit: template + this batch's pointers
    blob2 = plan2[0].numpy().tobytes() if isinstance(plan2[0], torch.Tensor) else bytes(plan2[0])
    want, rest, _ = _fresh(second)
    assert tuple(plan2[1:]) == tuple(rest)
    nb = S.ctypes.sizeof(S.DevNode) * rest[0]
    assert blob2[nb:] == want[nb:]                 # program and text pool
    mine = np.frombuffer(blob2[:nb], dtype=np.uint64).reshape(rest[0], -1)
    ref = np.frombuffer(want[:nb], dtype=np.uint64).reshape(rest[0], -1)
    assert (mine[:, :-S._PTR_COLS] == ref[:, :-S._PTR_COLS]).all()          # kinds, names, constants
    assert ((mine[:, -S._PTR_COLS:] == 0) == (ref[:, -S._PTR_COLS:] == 0)).all()
    # buffers used as they are (no dtype conversion) are the same addresses; converted ones point at kept tensors
    cols = [c for m in second for c in m.table.columns]
    for i, c in enumerate(cols):
        if isinstance(c, StrColumn):
            assert mine[i, -3] == c.arena.data_ptr() == ref[i, -3]
        elif isinstance(c, PrimColumn) and c.dtype in ("long", "double", "timestamp"):
            assert mine[i, -5] == c.data.data_ptr() == ref[i, -5]
    kept = {t.data_ptr() for t in keep}
    assert all(int(p) in kept for p in mine[:, -S._PTR_COLS:].ravel() if p)


def test_shape_change_misses_and_unsupported_columns_walk():
    S._PLANS.clear()
    a = [_M(_table(10, 1))]
    S._plan_of(a)
    t = _table(10, 1)
    b = [_M(Table(t.names[:-1] + ["h"], t.columns[:-1] + [ConstColumn("other", "string", 10, "cpu")], 10, "cpu"))]
    plan, _ = S._plan_of(b)                        # constant text differs: a second plan
    assert len(S._PLANS) == 2
    want, _, _ = _fresh(b)
    nb = S.ctypes.sizeof(S.DevNode) * plan[1]
    assert bytes(plan[0])[nb:] == want[nb:]
    assert S._flat_signature([_M(Table(["x"], [PrimColumn(parse_decimal_type("decimal(10,2)"), torch.zeros(3, dtype=torch.int64))],
                                             3, "cpu"))]) is None


def _const_texts(blob, nnodes, tw):
    """Each node's constant text, read back through its const_off / const_len."""
    nb = S.ctypes.sizeof(S.DevNode) * nnodes
    raw = blob if isinstance(blob, bytes) else bytes(blob.numpy()) if isinstance(blob, torch.Tensor) else bytes(blob)
    ints = np.frombuffer(raw[:nb], dtype=np.int32).reshape(nnodes, -1)
    text = raw[len(raw) - tw * 8:]
    return [text[o:o + n] for o, n in zip(ints[:, 6], ints[:, 7])]


def test_changing_constant_reuses_plan_with_patched_text():
    """An alert row's batch time is a constant that changes every batch: the plan is reused and the new value's text
    is appended to the pool, so the rendered constants are the builder's."""
    S._PLANS.clear()

    def alert(ts):
        cols = [ConstColumn(ts, "timestamp", 1, "cpu"), ConstColumn("HotAlert", "string", 1, "cpu"),
                ConstColumn(0, "long", 1, "cpu"), PrimColumn("double", torch.tensor([1.5], dtype=torch.float64))]
        return [_M(Table(["EventTime", "MetricName", "Metric", "v"], cols, 1, "cpu")), _M(_table(5, 9))]

    S._plan_of(alert(1792358528000000))
    for ts in (1792358529000000, 1792358530123000):
        plan, _ = S._plan_of(alert(ts))
        assert len(S._PLANS) == 1
        want, rest, _ = _fresh(alert(ts))
        assert _const_texts(plan[0], plan[1], plan[3]) == _const_texts(want, rest[0], rest[2])
