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
    p = _proc(tmp_path, "full")
    assert not p._concurrent_views()                  # default: statement order
    steps = p._view_schedule(p._live_statements())
    assert all(len(s) == 1 for s in steps)
    assert [k for s in steps for k in s] == sorted(k for s in steps for k in s)


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
