"""One-launch event-time statistics of a window pane (dxa/ops/csrc/reduce_stats.hip) against tensor reductions,
repeated to check the self-resetting completion ticket."""
import pytest
import torch

from dxa.engine.windows import _ts_stats


def _ref(ts, ok, E):
    big = torch.iinfo(torch.int64).max
    return [int(torch.where(ok, ts, torch.full_like(ts, big)).min()), int(torch.where(ok, ts, torch.full_like(ts, -big)).max()),
            int(ok.sum()), int((ok & (ts >= E)).sum())]


def test_cpu_path():
    ts = torch.tensor([5, 3, 9, 1], dtype=torch.int64)
    ok = torch.tensor([True, True, False, True])
    assert _ts_stats(ts, ok, 3) == [1, 5, 3, 2]


@pytest.mark.gpu
def test_gpu_matches_reference():
    g = torch.Generator().manual_seed(1)
    for n in (1, 63, 1000, 1_000_003, 5_000_000):
        ts = torch.randint(-10**15, 10**15, (n,), generator=g, dtype=torch.int64)
        ok = torch.rand(n, generator=g) > 0.1
        E = int(ts[0])
        for _ in range(2):
            assert _ts_stats(ts.cuda(), ok.cuda(), E) == _ref(ts, ok, E), n


def test_concat_panes_reuses_last_run_and_matches_concat():
    """_concat_panes over a sliding list of partial tables (oldest dropped, newest appended, a fresh clipped part in
    front) equals concat_tables of the same list, batch after batch, while reusing the previous result."""
    import types
    from dxa.engine.column import Table, column_from_pylist, concat_tables, strings_from_pylist
    from dxa.engine.query import _concat_panes

    def part(k):
        n = 3 + k % 4
        return Table(["k", "s", "v"], [column_from_pylist([k * 10 + i for i in range(n)], "long"),
                                      strings_from_pylist([f"s{k}-{i}" if i % 3 else None for i in range(n)], "cpu"),
                                      column_from_pylist([None if i == 1 else float(k + i) for i in range(n)],
                                                         "double")], n)
    store = types.SimpleNamespace()
    panes = [part(k) for k in range(12)]
    for b in range(8):
        clipped = part(100 + b)                                # recomputed every batch
        parts = [clipped] + panes[b:b + 8]
        got = _concat_panes(parts, store, "fp")
        want = concat_tables(parts)
        assert got.length == want.length
        for x, y in zip(got.columns, want.columns):
            assert x.to_pylist() == y.to_pylist()
        if b:
            # the previous batch's panes[b:b+7] were reused as one view of its result
            assert store.concat_cache["fp"][0][1] is panes[b]
