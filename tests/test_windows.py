"""Time-window semantics (TimeWindowHandler.scala / CommonProcessorFactory.scala:156-236) and the paned incremental
aggregation: a GROUP BY over a window view must equal the same query over the materialized union."""
import json

import pytest
import torch

from dxa.engine.column import PrimColumn, Table, strings_from_pylist
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql
from dxa.engine.serialize import table_to_json_lines
from dxa.engine.windows import PanedTable, TimeWindowConf, WindowStore

S = 1_000_000


def batch(rng, t_us, n, spread_us, dev="cpu"):
    ts = torch.tensor([t_us - int(rng.integers(0, spread_us)) for _ in range(n)], dtype=torch.int64)
    dev_id = torch.tensor(rng.integers(0, 7, n), dtype=torch.int64)
    temp = torch.tensor(rng.normal(20, 5, n), dtype=torch.float64)
    valid = torch.tensor(rng.random(n) > 0.1)
    kinds = strings_from_pylist([["a", "b", "c"][int(i) % 3] for i in rng.integers(0, 3, n)], dev)
    return Table(["ts", "deviceId", "kind", "temp"],
                 [PrimColumn("timestamp", ts), PrimColumn("long", dev_id), kinds, PrimColumn("double", temp, valid)],
                 n, dev)


QUERIES = [
    "SELECT deviceId, kind, COUNT(*) AS c, SUM(temp) AS s, MIN(temp) AS mn, MAX(temp) AS mx, AVG(temp) AS av "
    "FROM W GROUP BY deviceId, kind",
    "SELECT kind, COUNT(temp) AS c, STDDEV(temp) AS sd FROM W WHERE deviceId > 2 GROUP BY kind HAVING COUNT(*) > 3",
    "SELECT COUNT(*) AS c, MAX(ts) AS last FROM W",
    "SELECT deviceId % 2 AS parity, SUM(deviceId) AS s FROM W GROUP BY deviceId % 2",
]


def _canon(t):
    rows = [json.loads(r) for r in table_to_json_lines(t)]
    out = []
    for r in rows:
        out.append(tuple(sorted((k, round(v, 6) if isinstance(v, float) else v) for k, v in r.items())))
    return sorted(out)


@pytest.mark.parametrize("quirk,block,win,nb", [(True, 16, 5, 12), (False, 16, 5, 12), (False, 2, 5, 12),
                                                (True, 3, 5, 12), (False, 4, 23, 60), (True, 5, 31, 70)])
def test_paned_aggregate_matches_materialized(quirk, block, win, nb, monkeypatch):
    """Paned answers (per-pane partials and pre-combined complete blocks) equal the materialized window, batch after
    batch, through block completions and evictions."""
    import numpy as np
    import dxa.engine.query as Q
    monkeypatch.setattr(Q, "BLOCK", block)
    rng = np.random.default_rng(7)
    conf = TimeWindowConf({"W": win * S}, True, "ts", 2 * S, win * S, quirk)
    store = WindowStore(conf)
    ctx = EvalContext(now_us=0)
    for b in range(nb):
        T = (100 + b) * S
        views, _ = store.process(batch(rng, T, 200, 3 * S), T, S)
        assert isinstance(views["W"], PanedTable)
        for q in QUERIES:
            cat = Catalog()
            cat.register("W", views["W"])
            paned = run_sql(q, cat, ctx)
            mat = Table(views["W"].names, views["W"].columns, views["W"].length)
            cat2 = Catalog()
            cat2.register("W", mat)
            ref = run_sql(q, cat2, ctx)
            assert _canon(paned) == _canon(ref), (b, q)
    # fully-inside panes were answered from cached partials (and pre-combined blocks when blocks are small)
    assert any(p.partials for p in store.past.values())
    if block <= 3 or win > 2 * block:
        assert store.blocks


def test_window_ranges_and_eviction():
    conf = TimeWindowConf({"W2": 2 * S, "W4": 4 * S}, True, "ts", 0, 4 * S, False)
    store = WindowStore(conf)
    for b in range(8):
        T = (10 + b) * S
        ts = torch.tensor([T - S + 1, T + 5], dtype=torch.int64)    # one row in the last second, one future row
        t = Table(["ts"], [PrimColumn("timestamp", ts)], 2)
        views, kept = store.process(t, T, S)
        assert kept == 1                                              # rows with ts >= E are retained
        # future rows of earlier batches land inside later windows
        assert views["W2"].length == min(2, b)
        # retained batches are evicted by *batch* time (t <= T - (W + M)), so the oldest row drops out early
        assert views["W4"].length == min(3, b)
        assert views["DataXProcessedInput_Batch"].length == 2
    assert len(store.past) <= 5


@pytest.mark.gpu
@pytest.mark.parametrize("spread,nb,win,block", [(S - 1, 40, 9, 16), (S - 1, 40, 11, 3), (3 * S, 24, 5, 2)])
def test_dense_ring_matches_materialized(spread, nb, win, block, monkeypatch):
    """The dense window path (window_dense.py / window_ring.hip: persistent group dictionary + per-pane accumulator
    ring) answers the decomposable window statements on the GPU; its rows equal the materialized window's batch
    after batch — through ring-slot reuse after evictions, clipped panes (re-aggregated into scratch slots) when the
    event times straddle the window edges, NULL arguments and a WHERE; with small ``block`` sizes through block
    slots pre-combined, reused and dropped as the window slides."""
    import numpy as np
    from dxa.engine import window_dense
    monkeypatch.setattr(window_dense, "BLOCK", block)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    conf = TimeWindowConf({"W": win * S}, True, "ts", 2 * S, win * S, False)
    store = WindowStore(conf)
    ctx = EvalContext(now_us=0, device=dev)
    qs = [QUERIES[0], "SELECT kind, deviceId, MAX(ts) AS last, MIN(deviceId) AS lo, COUNT(temp) AS ct, "
                      "SUM(deviceId) AS sd FROM W WHERE temp > 18 GROUP BY kind, deviceId",
          "SELECT deviceId % 2 AS parity, SUM(deviceId) AS s FROM W GROUP BY deviceId % 2 HAVING COUNT(*) > 2"]
    for b in range(nb):
        T = (100 + b) * S
        views, _ = store.process(batch(rng, T, 300, spread).to(dev), T, S)
        for q in qs:
            cat = Catalog()
            cat.register("W", views["W"])
            paned = run_sql(q, cat, ctx)
            mat = Table(views["W"].names, views["W"].columns, views["W"].length, dev)
            cat2 = Catalog()
            cat2.register("W", mat)
            ref = run_sql(q, cat2, ctx)
            assert _canon(paned) == _canon(ref), (b, q)
    dense = store.__dict__.get("_dense", {})
    assert len(dense) == len(qs) and not any(d.disabled for d in dense.values())
    # the ring only ever holds retained panes
    for d in dense.values():
        assert len(d.slot_of) <= len(store.past) + 1
    if block < win:
        assert any(d.blocks for d in dense.values())


@pytest.mark.gpu
def test_dense_deferred_completion_and_collision_fallback(monkeypatch):
    """A deferred windowed statement (ctx.defer_dense: the status read waits for first use, query._deferred_select)
    equals the materialized window; when the status reports a collision the DeferredTable re-runs the statement on
    the paned path against the catalog it was planned with, and the dense state is disabled from then on."""
    import numpy as np
    from dxa.engine import window_dense
    from dxa.engine.column import DeferredTable
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    store = WindowStore(TimeWindowConf({"W": 6 * S}, True, "ts", 2 * S, 6 * S, False))
    q = QUERIES[0]
    finish = window_dense.DenseWindow._finish
    for b in range(14):
        T = (100 + b) * S
        views, _ = store.process(batch(rng, T, 300, S - 1).to(dev), T, S)
        if b == 10:                                  # this batch's status reads as a dictionary collision
            monkeypatch.setattr(window_dense.DenseWindow, "_finish", lambda self, st, *a: finish(self, [0, 1, 0, 0], *a))
        ctx = EvalContext(now_us=0, device=dev)
        ctx.defer_dense = True
        cat = Catalog()
        cat.register("W", views["W"])
        got = run_sql(q, cat, ctx)
        if 4 <= b < 10:
            assert isinstance(got, DeferredTable) and ctx.pending
        mat = Table(views["W"].names, views["W"].columns, views["W"].length, dev)
        cat2 = Catalog()
        cat2.register("W", mat)
        assert _canon(got) == _canon(run_sql(q, cat2, EvalContext(now_us=0, device=dev))), b
        if b == 10:
            monkeypatch.setattr(window_dense.DenseWindow, "_finish", finish)
    assert all(d.disabled for d in store.__dict__["_dense"].values())


def test_pieces_from_bound_arrays_match_the_pane_loop():
    """PanedTable.pieces from the store's maintained pane-bound arrays equals the per-pane loop: empty panes,
    inverted bounds, panes with untimed rows, open and closed ranges."""
    import random
    import numpy as np
    from dxa.engine.column import Table, column_from_pylist
    from dxa.engine.windows import Pane, PanedTable, WindowStore, _pane_meta
    rnd = random.Random(0)
    st = WindowStore.__new__(WindowStore)
    st.past = {}
    panes = []
    for k in range(60):
        n = rnd.choice([0, 3])
        lo = rnd.randint(0, 100)
        p = Pane(k, Table(["a"], [column_from_pylist(list(range(n)), "long")], n), lo, lo + rnd.randint(-5, 30),
                 rnd.random() < 0.8)
        if k:
            st.past[k] = p
        panes.append(p)
    m = st._meta
    st._batch_meta = (panes, *(np.concatenate(([v], a)) for v, a in zip(_pane_meta(panes[0]), m[1:])))
    for lo, hi in [(None, None), (10, 60), (50, None), (None, 40), (200, 300), (30, 31)]:
        fast = PanedTable(st, panes, lo, hi, ["a"], "cpu").pieces()
        saved, st._batch_meta = st._batch_meta, None
        slow = PanedTable(st, panes, lo, hi, ["a"], "cpu").pieces()
        st._batch_meta = saved
        assert [(p.key, f) for p, f in fast] == [(p.key, f) for p, f in slow], (lo, hi)


def test_pieces_bound_arrays_track_process_across_expiry():
    """The store's pane-bound arrays stay aligned with its panes as batches arrive and expire (WindowStore.process):
    every view's pieces equal the per-pane loop over a copy of its pane list."""
    import torch
    from dxa.engine.column import PrimColumn, Table, column_from_pylist
    from dxa.engine.windows import PanedTable, TimeWindowConf, WindowStore
    st = WindowStore(TimeWindowConf({"W_5s": 5_000_000}, True, "ts", 0, 5_000_000, False))
    t0 = 1_700_000_000_000_000
    for i in range(12):
        bt = t0 + i * 1_000_000
        ts = torch.arange(1000, dtype=torch.int64) * 1000 + bt - (400_000 if i % 3 == 0 else 0)   # some late rows
        tab = Table(["ts", "v"], [PrimColumn("timestamp", ts), column_from_pylist(list(range(1000)), "long")], 1000)
        views, _ = st.process(tab, bt, 1_000_000)
        for v in views.values():
            if isinstance(v, PanedTable):
                slow = PanedTable(st, list(v.panes), v.lo, v.hi, v.names, "cpu").pieces()
                assert [(p.key, f) for p, f in v.pieces()] == [(p.key, f) for p, f in slow]
