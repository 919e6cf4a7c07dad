"""Deferred completion of windowed statements (query._deferred_select): the DeferredTable proxy, and the level-ordered
sequential schedule that lets independent statements run before a windowed statement's readers."""
from dxa.engine.column import DeferredTable, Table, column_from_pylist


def test_deferred_table_completes_on_first_use():
    calls = []

    def finish():
        calls.append(1)
        t = Table(["a", "b"], [column_from_pylist([1, 2, 3], "long"), column_from_pylist([4, 5, 6], "long")], 3)
        t.dist = "hashed"
        return t
    d = DeferredTable(finish)
    d.tag = "set while pending"
    assert not calls
    assert len(d) == 3 and calls == [1]
    assert type(d) is Table and d.dist == "hashed" and d.tag == "set while pending"
    assert d.column("b").to_pylist() == [4, 5, 6] and d.names == ["a", "b"]
    assert calls == [1]


def test_deferred_table_chains():
    inner = DeferredTable(lambda: Table(["x"], [column_from_pylist([7], "long")], 1))
    outer = DeferredTable(lambda: inner)
    assert outer.columns[0].to_pylist() == [7] and type(outer) is Table
