"""Window-pane string compaction: the lengths of a parsed batch's string leaves as one view (strings.lens_concat)
and the multi-column compaction whose gather derives each row's destination from the byte scan
(strings.compact_many), against the per-column reference."""
import pytest
import torch

from dxa.engine.column import StrColumn, strings_from_pylist
from dxa.ops.strings import compact, compact_many, lens_concat


def test_lens_concat_views_consecutive_rows_cpu():
    m = torch.arange(12, dtype=torch.int32).reshape(3, 4)
    v = lens_concat([m[0], m[1], m[2]])
    assert v.data_ptr() == m.data_ptr() and torch.equal(v, m.reshape(-1))
    w = lens_concat([m[1], m[2]])                     # a suffix block: still a view
    assert w.data_ptr() == m[1].data_ptr() and torch.equal(w, m[1:].reshape(-1))
    x = lens_concat([m[2], m[0]])                     # out of order: a copy
    assert x.data_ptr() not in (m.data_ptr(), m[2].data_ptr()) and torch.equal(x, torch.cat([m[2], m[0]]))
    y = lens_concat([m[0, :2], m[1, :2]])             # partial rows are not consecutive: a copy
    assert torch.equal(y, torch.tensor([0, 1, 4, 5], dtype=torch.int32))


@pytest.mark.gpu
def test_compact_many_matches_compact(gpu):
    vals = [["a", "bb", None, "", "dddd" * 40], ["x" * 200, "y", "zz", None, "w"], ["p", "", "q", "r", "s"]]
    src = [strings_from_pylist(v, gpu) for v in vals]
    # rows that view a shared arena out of order, as a parsed batch's columns do
    cols = [StrColumn(c.arena, c.starts.flip(0), c.lens.flip(0), None if c.valid is None else c.valid.flip(0))
            for c in src]
    lens = torch.stack([c.lens for c in cols]).contiguous()
    cols = [StrColumn(c.arena, c.starts, lens[k], c.valid) for k, c in enumerate(cols)]
    got = compact_many(cols)
    for c, g in zip(cols, got):
        assert g.to_pylist() == compact(c).to_pylist() == c.to_pylist()
        assert g.arena.data_ptr() == got[0].arena.data_ptr()
    # starts are disjoint and in order in the shared arena
    starts = torch.cat([g.starts for g in got]).cpu()
    ln = torch.cat([g.lens for g in got]).cpu().to(torch.int64)
    assert torch.equal(starts[1:], (starts + ln)[:-1])
