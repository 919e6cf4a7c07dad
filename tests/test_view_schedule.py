"""The concurrent-view schedule (Processor._view_schedule): levels from read-after-write and write-after-read
dependencies, accumulator statements alone, sequential order when concurrency is off."""
import pytest

from dxa.engine.processor import Processor
from dxa.models import iot


def _proc(tmp_path, variant):
    return Processor(iot.flow_settings(workdir=str(tmp_path), variant=variant, sink="memory", ref_rows=100), "cpu")


def _names(p, steps):
    cmds = p.transform.commands
    return [[cmds[k].name for k in s] for s in steps]


def test_sequential_by_default(tmp_path):
    p = _proc(tmp_path, "groupby")
    assert not p._concurrent_views() and p.window_store is None    # default: statement order
    steps = p._view_schedule(p._live_statements())
    assert all(len(s) == 1 for s in steps)
    assert [k for s in steps for k in s] == sorted(k for s in steps for k in s)


def test_sequential_level_order_with_a_window(tmp_path):
    """With a time window, sequential views run level by level (one per step): a windowed statement's readers
    come after the statements that do not read it, so its deferred completion finds its kernels done."""
    p = _proc(tmp_path, "full")
    assert not p._concurrent_views() and p.window_store is not None
    live = p._live_statements()
    steps = p._view_schedule(live)
    assert all(len(s) == 1 for s in steps)
    names = [n for s in _names(p, steps) for n in s]
    from dxa.sql.transform import COMMAND_COMMAND
    assert sorted(k for s in steps for k in s) == [k for k, c in enumerate(p.transform.commands)
                                                   if c.command_type == COMMAND_COMMAND or k in live]
    pos = {n: i for i, n in enumerate(names)}
    assert pos["DeviceWindow"] < pos["DeviceNamed"] < pos["UnhealthyDevices"]
    assert pos["DeviceWindow"] < pos["DeviceState"]
    # a statement that reads only the input runs before DeviceWindow's first reader
    indep = [n for n in names if n and n.startswith("sa1_")]
    assert indep and all(pos[n] < pos["DeviceNamed"] for n in indep)
    # within a level the windowed statement comes first and its readers last: DeviceWindow before the rules'
    # filters, the alerts before DeviceWindow's readers
    assert all(pos["DeviceWindow"] < pos[n] for n in indep)
    assert pos["HotAlert"] < pos["DeviceNamed"] and pos["LowBatteryAlert"] < pos["DeviceNamed"]


def test_levels_and_accumulator(tmp_path, monkeypatch):
    p = _proc(tmp_path, "full")
    monkeypatch.setattr(Processor, "_concurrent_views", lambda self: True)
    live = p._live_statements()
    names = _names(p, p._view_schedule(live))
    flat = [n for s in names for n in s if n]
    assert sorted(flat) == sorted(p.transform.commands[k].name for k in live)
    assert all(n for s in names if len(s) > 1 for n in s)      # commands never share a step
    pos = {n: i for i, s in enumerate(names) for n in s}
    # DeviceWindow feeds DeviceNamed and DeviceState; DeviceNamed feeds UnhealthyDevices
    assert pos["DeviceWindow"] < pos["DeviceNamed"] < pos["UnhealthyDevices"]
    assert pos["DeviceWindow"] < pos["DeviceState"]
    assert ["DeviceState"] in names                   # the accumulator runs alone
    assert any(len(s) > 1 for s in names)             # something runs concurrently
    level0 = next(s for s in names if s[0])
    assert "DeviceWindow" in level0


def test_write_after_read(tmp_path, monkeypatch):
    """A statement reading an accumulator's previous state runs before the accumulator's statement even when it
    sits at a deeper level."""
    from dxa.sql.transform import parse_transform
    p = _proc(tmp_path, "full")
    monkeypatch.setattr(Processor, "_concurrent_views", lambda self: True)
    p.transform = parse_transform([
        "--DataXQuery--", "A = SELECT deviceDetails.deviceId AS deviceId FROM DataXProcessedInput;",
        "--DataXQuery--", "B = SELECT deviceId FROM A;",
        "--DataXQuery--", "Old = SELECT COUNT(*) AS c FROM DeviceState JOIN B ON DeviceState.deviceId = B.deviceId;",
        "--DataXQuery--", "DeviceState = SELECT * FROM DeviceState;",
    ])
    names = _names(p, p._view_schedule(None))
    pos = {n: i for i, s in enumerate(names) for n in s}
    assert pos["A"] < pos["B"] < pos["Old"] < pos["DeviceState"]


def test_filter_readers_of_produced_views(tmp_path):
    """Statements with a plain WHERE over a view the batch produces are found by that view's name
    (query.filter_readers): the processor queues their masks when the view is registered."""
    from dxa.engine.expr import EvalContext
    from dxa.engine.query import filter_readers
    p = _proc(tmp_path, "full")
    cmds = p.transform.commands
    order = [k for s in p._view_schedule(p._live_statements()) for k in s if cmds[k].name]
    got = filter_readers([(k, p._query(cmds[k])) for k in order], EvalContext())
    assert [cmds[k].name for k, _, _ in got.get("devicenamed", [])] == ["UnhealthyDevices"]
    # the windowed GROUP BY is not a filter of its input (the dense / paned path applies its WHERE per pane)
    assert all(cmds[k].name != "DeviceWindow" for v in got.values() for k, _, _ in v)
