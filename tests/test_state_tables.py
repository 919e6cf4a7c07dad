"""State tables reloaded from Parquet carry a host bound on their string bytes (``StrColumn.max_len``), so the
per-batch ``UNION ALL`` with the state concatenates without reading a device scan (strings.concat_multi)."""
import pytest
import torch

from dxa.engine.column import Table, column_from_pylist, concat_tables, strings_from_pylist
from dxa.engine.state import StateTable
from dxa.engine.types import parse_ddl_schema


def _roundtrip(tmp_path, device):
    loc = str(tmp_path / "st")
    schema = parse_ddl_schema("k long, name string")
    st = StateTable("S", schema, loc, device)
    names = ["a", "bbbbbbbbbb", None, "ccc"]
    t = Table(["k", "name"], [column_from_pylist([1, 2, 3, 4], "long", device),
                              strings_from_pylist(names, device)], 4, device)
    st.overwrite(t, tag=1)
    st.flush(1)
    st.persist(1)
    st.release()
    return StateTable("S", schema, loc, device), names


def test_reloaded_state_strings_are_length_bounded(tmp_path):
    again, names = _roundtrip(tmp_path, "cpu")
    col = again.active.columns[1]
    assert col.to_pylist() == names
    assert col.max_len == 10


@pytest.mark.gpu
def test_union_with_reloaded_state_needs_no_scan(tmp_path, gpu):
    """The concatenation of a reloaded state and a bounded batch output sizes its arena from the bounds alone
    (no `.item()`); the result is still exact and stays bounded."""
    again, names = _roundtrip(tmp_path, gpu)
    batch = strings_from_pylist(["dddd", "e"], gpu)
    batch.max_len = 48
    other = Table(["k", "name"], [column_from_pylist([5, 6], "long", gpu), batch], 2, gpu)
    orig = torch.Tensor.item

    def no_item(self):
        raise AssertionError("concat read a device scalar")
    torch.Tensor.item = no_item
    try:
        out = concat_tables([again.active, other])
    finally:
        torch.Tensor.item = orig
    assert out.columns[1].to_pylist() == names + ["dddd", "e"]
    assert out.columns[1].max_len == 48
