"""Stage tracing: named ranges around every micro-batch stage.

* ``DXA_TRACE=1`` emits ROCm-tracer ranges (roctx, through ``torch.cuda.nvtx`` on ROCm builds) so
  ``rocprofv3 --marker-trace`` / ``--kernel-trace`` timelines show parse / project / window / each SQL statement /
  output staging per batch (SURVEY §5 "roctx ranges per batch stage").
* Stage wall times are always recorded and exported with the batch metrics as ``Latency-Stage-<name>`` (seconds), so
  they reach the metric store and the dashboard like the reference's ``Latency-Process``.
* ``logger()`` returns a logger whose name carries the rank suffix (the reference's ``-P<partition>-T<attempt>``
  executor logger suffix, SparkEnvVariables.scala:14-17).
"""
from __future__ import annotations

import collections
import logging
import os
import time
from contextlib import contextmanager
from typing import Dict, Optional

_TRACE = os.environ.get("DXA_TRACE") == "1"
_nvtx = None
if _TRACE:
    try:
        import torch
        if torch.cuda.is_available():
            _nvtx = torch.cuda.nvtx
    except Exception:  # noqa: BLE001 — tracing is best effort
        _nvtx = None


_record_function = None


def enable_profiler_ranges():
    """Also open a ``torch.profiler.record_function`` range per stage (``bench.py --torch-profile``)."""
    global _record_function
    import torch
    _record_function = torch.profiler.record_function


@contextmanager
def stage(name: str, times: Optional[Dict[str, float]] = None):
    """Time (and, with DXA_TRACE=1, mark) one stage; ``times[name]`` receives the wall seconds."""
    if _nvtx is not None:
        _nvtx.range_push(name)
    rf = _record_function(name) if _record_function is not None else None
    if rf is not None:
        rf.__enter__()
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if times is not None:
            times[name] = time.perf_counter() - t0
        if rf is not None:
            rf.__exit__(None, None, None)
        if _nvtx is not None:
            _nvtx.range_pop()


# host-time sections inside a statement (DXA_HOST_TIMERS=1; bench.py --profile-stages prints them per step)
HOST_ACC: Dict[str, float] = collections.defaultdict(float)
_HOST_TIMERS = os.environ.get("DXA_HOST_TIMERS") == "1"


class _Section:
    __slots__ = ("name", "t0")

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.t0 = time.perf_counter()

    def __exit__(self, *exc):
        HOST_ACC[self.name] += time.perf_counter() - self.t0


class _NoSection:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NO_SECTION = _NoSection()


def host_section(name: str):
    """Accumulate this block's host wall time under ``name`` (no-op unless DXA_HOST_TIMERS=1)."""
    return _Section(name) if _HOST_TIMERS else _NO_SECTION


def time_host_syncs() -> None:
    """DXA_HOST_TIMERS=1: also accumulate the host time spent blocked in ``.item()`` / ``.tolist()`` /
    ``Event.synchronize`` / ``Stream.synchronize`` (device waits) under ``sync:<name>``."""
    if not _HOST_TIMERS:
        return
    import torch

    def wrap(owner, attr, key):
        fn = getattr(owner, attr)

        def timed(*a, **k):
            t0 = time.perf_counter()
            try:
                return fn(*a, **k)
            finally:
                HOST_ACC[key] += time.perf_counter() - t0
        setattr(owner, attr, timed)
    wrap(torch.Tensor, "item", "sync:item")
    wrap(torch.Tensor, "tolist", "sync:tolist")
    wrap(torch.cuda.Event, "synchronize", "sync:event")
    wrap(torch.cuda.Stream, "synchronize", "sync:stream")


def stage_metrics(times: Dict[str, float]) -> Dict[str, float]:
    return {f"Latency-Stage-{k}": float(v) for k, v in times.items()}


def logger(name: str) -> logging.Logger:
    rank = os.environ.get("RANK")
    return logging.getLogger(f"{name}-R{rank}" if rank is not None else name)
