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
