"""Batch scheduling: turn a batching flow's ``batchList`` (one-time and recurring entries) into one job per time slot,
then (re)start them; plus the timed background scheduler that triggers it.

Behaviour follows the reference:
  * ConfigHelper.cs:40-280 — partition increment from the path template, interval/delay/window translation
    (a window of N units is ``N units - 1 min + 59.059 s``), time normalisation per interval type, the
    schedule / recurring-validity predicates;
  * S600_GenerateJobConfigBatch.cs:60-240 — the slot loop ``processing = start; processing <= end; += interval``,
    the slot window ``[ps_e - window, ps_e]`` with ``ps_e = slot + interval - 1 ms`` (rendered at second precision),
    job names ``<flow>[-OneTime]-<digits of the scheduled time>``, ``lastProcessedTime`` advanced for recurring
    entries and one-time entries disabled after scheduling;
  * FlowOperation.cs:88-104 (``flow/schedulebatch``) and DataX.Flow.Scheduler/TimedScheduler.cs (hourly wake-up).
"""
from __future__ import annotations

import datetime as _dt
import logging
import os
import re
import threading
from typing import Any, Dict, List, Optional

log = logging.getLogger("dxa.scheduler")

ONE_TIME, RECURRING = "oneTime", "recurring"
_TEMPLATE = re.compile(r"\{([yMdHhmsS\-/.,: ]+)\}*", re.I)


def _unit_minutes(unit: str) -> int:
    return {"min": 1, "hour": 60}.get(unit, 60 * 24)


def translate_interval(value, unit: str) -> _dt.timedelta:
    return _dt.timedelta(minutes=_unit_minutes(unit) * int(value))


translate_delay = translate_interval


def translate_window(value, unit: str) -> _dt.timedelta:
    return _dt.timedelta(minutes=_unit_minutes(unit) * int(value) - 1, seconds=59, milliseconds=59)


def normalize_time(t: _dt.datetime, interval_type: str, delay: _dt.timedelta = _dt.timedelta()) -> _dt.datetime:
    t = t - delay
    if interval_type == "min":
        return t.replace(second=0, microsecond=0)
    if interval_type == "hour":
        return t.replace(minute=0, second=0, microsecond=0)
    return t.replace(hour=0, minute=0, second=0, microsecond=0)


def should_schedule(disabled: bool, one_time: bool, start: Optional[_dt.datetime], end: Optional[_dt.datetime]):
    return not (disabled or start is None or (one_time and end is None))


def is_valid_recurring(now: _dt.datetime, start: _dt.datetime, end: Optional[_dt.datetime]) -> bool:
    return not (now < start or (end is not None and end < now))


def partition_increment(path: str) -> int:
    """Minutes between blob time partitions implied by the ``{…}`` template of ``path``."""
    m = _TEMPLATE.search(path or "")
    if m:
        v = m.group(1).strip()
        if "h" in v.lower():
            return 60
        if "d" in v.lower():
            return 60 * 24
        if "M" in v:
            return 60 * 24 * 30
        if "y" in v.lower():
            return 60 * 24 * 30 * 12
    return 1


def blob_partition_format(mode: str, fmt: str) -> str:
    if mode != "batching":
        return "%1$tY/%1$tm/%1$td/%1$tH/${quarterBucket}/${minuteBucket}"
    conv = {"s": "%1$tS", "m": "%1$tM", "h": "%1$tH", "H": "%1$tH", "d": "%1$td", "M": "%1$tm", "y": "%1$ty"}
    for part in re.split(r"[,/: \-]", fmt):
        if part:
            fmt = fmt.replace(part, conv.get(part[0], ""))
    return fmt


def _parse_time(v) -> Optional[_dt.datetime]:
    if v in (None, ""):
        return None
    if isinstance(v, (int, float)):
        return _dt.datetime.fromtimestamp(v, _dt.timezone.utc).replace(tzinfo=None)
    s = str(v).strip().replace("Z", "").replace("z", "")
    t = _dt.datetime.fromisoformat(s)
    if t.tzinfo is not None:
        t = t.astimezone(_dt.timezone.utc).replace(tzinfo=None)
    return t


def _fmt(t: _dt.datetime) -> str:
    return t.replace(microsecond=0).isoformat() + "Z"


def batch_slots(flow_name: str, entry: Dict[str, Any], now: _dt.datetime) -> Dict[str, Any]:
    """Slots for one ``batchList`` entry: ``{"slots": [...], "lastProcessedTime": …, "disable": bool}``."""
    one_time = entry.get("type") == ONE_TIME
    p = entry.get("properties") or {}
    start, end = _parse_time(p.get("startTime")), _parse_time(p.get("endTime"))
    out: Dict[str, Any] = {"slots": [], "lastProcessedTime": None, "disable": False}
    if not should_schedule(bool(entry.get("disabled")), one_time, start, end):
        return out
    interval = translate_interval(p.get("interval", 1), p.get("intervalType", "day"))
    delay = translate_delay(p.get("delay", 0), p.get("delayType", "day"))
    window = translate_window(p.get("window", 1), p.get("windowType", "day"))
    if not one_time and not is_valid_recurring(now, start, end):
        out["disable"] = True
        return out
    if one_time:
        prefix, lo, hi = "-OneTime", start, end
    else:
        prefix = ""
        last = p.get("lastProcessedTime")
        lo = start if last in (None, "") else _dt.datetime.fromtimestamp(int(last), _dt.timezone.utc).replace(
            tzinfo=None) + interval
        hi = now
    t, last_slot = lo, None
    while t <= hi:
        last_slot = t
        scheduled = normalize_time(t, p.get("intervalType", "day"))
        processing = normalize_time(t, p.get("intervalType", "day"), delay)
        ps_e = processing + interval - _dt.timedelta(milliseconds=1)
        pe_e = ps_e - window
        digits = re.sub(r"[^0-9]", "", _fmt(scheduled))
        out["slots"].append({"name": f"{flow_name}{prefix}-{digits}", "processStartTime": _fmt(pe_e),
                             "processEndTime": _fmt(ps_e), "processingTime": _fmt(scheduled),
                             "isOneTime": one_time,
                             "folder": ("OneTime/" if one_time else "Recurring/") + digits})
        t += interval
    if one_time:
        out["disable"] = True
    elif last_slot is not None:
        out["lastProcessedTime"] = str(int(last_slot.replace(tzinfo=_dt.timezone.utc).timestamp()))
    return out


def plan_batches(flow: Dict[str, Any], now: Optional[_dt.datetime] = None) -> List[Dict[str, Any]]:
    """All slots of a flow; mutates the flow's ``batchList`` (lastProcessedTime / disabled) like the reference."""
    now = now or _dt.datetime.utcnow()
    gui = flow.get("gui", flow)
    slots = []
    for entry in gui.get("batchList") or []:
        r = batch_slots(flow["name"], entry, now)
        slots += r["slots"]
        if r["lastProcessedTime"] is not None:
            entry.setdefault("properties", {})["lastProcessedTime"] = r["lastProcessedTime"]
        if r["disable"]:
            entry["disabled"] = True
    return slots


def schedule_batches(st, body=None, now: Optional[_dt.datetime] = None) -> Dict[str, Any]:
    """``flow/schedulebatch``: for every batching flow, generate its config, create one job per slot, start them."""
    from ..flow import configgen
    started: Dict[str, List[str]] = {}
    for flow in st.store.get_all("flows"):
        if (flow.get("gui", {}).get("input", {}).get("mode") or "").lower() != "batching":
            continue
        slots = plan_batches(flow, now)
        res = configgen.generate(flow, os.path.join(st.root, "runtime"), metrics_endpoint=st.metrics_endpoint)
        saved = res.flow
        saved["gui"]["batchList"] = flow["gui"].get("batchList")
        base = res.jobs[0]
        names = []
        for s in slots:
            job = {**base, "name": s["name"], "flow": flow["name"], "app": "batch", "isOneTime": s["isOneTime"],
                   "args": {"processStartTime": s["processStartTime"], "processEndTime": s["processEndTime"]},
                   "state": "Idle"}
            st.jobs.upsert(job)
            st.jobs.restart(s["name"])
            names.append(s["name"])
        saved["jobNames"] = sorted(set((flow.get("jobNames") or []) + names) - {base["name"]})
        st.store.upsert("flows", flow["name"], saved)
        started[flow["name"]] = names
    return started


class TimedScheduler(threading.Thread):
    """Calls ``schedule_batches`` every ``period_s`` (the reference wakes hourly)."""

    def __init__(self, st, period_s: float = 3600.0):
        super().__init__(daemon=True, name="dxa-scheduler")
        self.st = st
        self.period_s = period_s
        self._stop = threading.Event()

    def run(self):
        while not self._stop.is_set():
            try:
                schedule_batches(self.st)
            except Exception:  # noqa: BLE001
                log.exception("batch scheduling failed")
            self._stop.wait(self.period_s)

    def stop(self):
        self._stop.set()
