"""Spark SQL built-ins beyond the core set in ``expr.py``: math, date formatting / arithmetic, array functions
(``split`` and friends), hashing / encoding, JSON extraction.

Device-first where it matters for event-rate work: math is tensor arithmetic, ``split`` produces slot views into
the source arena with two small kernels (strings.hip), ``date_format`` renders fixed-width patterns with one
kernel and no host synchronisation, ``from_json`` runs the batch JSON parser over the column's bytes.  The
rarely-hot string digests and encodings are host-assisted (per-row Python), as the engine's other host string
functions are.
"""
from __future__ import annotations

import base64 as _b64
import datetime as _dt
import hashlib
import json
import math
import re
import zlib
from typing import List, Optional

import torch

from ..sql import ast as A
from . import functions as F
from .decimal import true_div as _true_div
from .types import INTEGRAL, SIMPLE_NAME, ArrayType, MapType, StructField, StructType, wrap_int_tensor
from .column import (ArrayColumn, Column, ConstColumn, PrimColumn, StrColumn, StructColumn, column_from_pylist,
                     materialize, strings_from_pylist)
from .expr import (EvalError, _args, _host_string_fn, _slot_present, bool_col, cast_column, evaluate,
                   register_function)

_EPOCH = _dt.datetime(1970, 1, 1)


# ---------------------------------------------------------------------------------------------------------------
# math
# ---------------------------------------------------------------------------------------------------------------

def _num(c: Column, n, dev) -> PrimColumn:
    c = materialize(c) if isinstance(c, ConstColumn) else c
    if not isinstance(c, PrimColumn):
        c = cast_column(c, "double")
    return c


def _and(*valids):
    out = None
    for v in valids:
        if v is not None:
            out = v if out is None else out & v
    return out


def _binary_double(fn):
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        a, b = _args(e, scope, ctx, subst)
        if isinstance(a, ConstColumn) and isinstance(b, ConstColumn):
            if a.value is None or b.value is None:
                return ConstColumn(None, "double", n, dev)
            r = fn(torch.tensor([float(a.value)], dtype=torch.float64), torch.tensor([float(b.value)],
                                                                                     dtype=torch.float64))
            return ConstColumn(float(r[0]), "double", n, dev)
        a, b = _num(a, n, dev), _num(b, n, dev)
        return PrimColumn("double", fn(a.data.to(torch.float64), b.data.to(torch.float64)), _and(a.valid, b.valid))
    return f


def _unary_double(fn):
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        (a,) = _args(e, scope, ctx, subst)
        if isinstance(a, ConstColumn):
            return ConstColumn(None if a.value is None else float(fn(torch.tensor([float(a.value)],
                                                                                    dtype=torch.float64))[0]),
                               "double", n, dev)
        a = _num(a, n, dev)
        return PrimColumn("double", fn(a.data.to(torch.float64)), a.valid)
    return f


def _f_log(e, scope, ctx, subst):
    if len(e.args) == 1:
        return _unary_double(torch.log)(e, scope, ctx, subst)
    return _binary_double(lambda b, x: torch.log(x) / torch.log(b))(e, scope, ctx, subst)


def _f_mod(positive: bool):
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        a, b = (_num(c, n, dev) for c in _args(e, scope, ctx, subst))
        integral = a.dtype in INTEGRAL and b.dtype in INTEGRAL
        x = a.data if integral else a.data.to(torch.float64)
        y = b.data if integral else b.data.to(torch.float64)
        zero = y == 0
        ys = torch.where(zero, torch.ones_like(y), y)
        r = torch.fmod(x, ys)                                   # sign of the dividend (Java %)
        if positive:
            r = torch.where(r < 0, torch.fmod(r + ys, ys), r)
        valid = _and(a.valid, b.valid, ~zero)                   # x % 0 is null in Spark
        return PrimColumn(a.dtype if integral else "double", r, valid)
    return f


def _f_const(v):
    def f(e, scope, ctx, subst):
        return ConstColumn(v, "double", scope.length, scope.device)
    return f


def _f_rand(normal: bool):
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        g = None
        if e.args:
            s = evaluate(e.args[0], scope, ctx, subst)
            g = torch.Generator(device=dev)
            g.manual_seed(int(s.value or 0))
        d = torch.randn(n, dtype=torch.float64, device=dev, generator=g) if normal else \
            torch.rand(n, dtype=torch.float64, device=dev, generator=g)
        return PrimColumn("double", d)
    return f


def _f_isnan(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    (a,) = _args(e, scope, ctx, subst)
    if isinstance(a, ConstColumn):
        v = a.value
        return ConstColumn(isinstance(v, float) and math.isnan(v), "boolean", n, dev)
    a = _num(a, n, dev)
    return bool_col(torch.isnan(a.data.to(torch.float64)) & a.valid_mask(), None)


def _f_nanvl(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    a, b = (_num(c, n, dev) for c in _args(e, scope, ctx, subst))
    x, y = a.data.to(torch.float64), b.data.to(torch.float64)
    nan = torch.isnan(x)
    return PrimColumn("double", torch.where(nan, y, x), torch.where(nan, b.valid_mask(), a.valid_mask())
                      if (a.valid is not None or b.valid is not None) else None)


def _f_cast_to(to):
    def f(e, scope, ctx, subst):
        (a,) = _args(e, scope, ctx, subst)
        return cast_column(a, to)
    return f


# ---------------------------------------------------------------------------------------------------------------
# dates
# ---------------------------------------------------------------------------------------------------------------

def _ts(c: Column) -> Column:
    if c.dtype == "timestamp":
        return c
    return cast_column(c, "timestamp")


def _days(c: Column) -> Column:
    """date / timestamp / string → days since epoch (PrimColumn 'date')."""
    if c.dtype == "date":
        return c
    return cast_column(_ts(c), "date")


def _f_date_add(sign: int):
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        a, k = _args(e, scope, ctx, subst)
        d = _days(a)
        if isinstance(d, ConstColumn) and isinstance(k, ConstColumn):
            return ConstColumn(None if d.value is None or k.value is None else d.value + sign * int(k.value),
                               "date", n, dev)
        d, k = materialize(d), _num(k, n, dev)
        return PrimColumn("date", d.data + sign * k.data.to(torch.int64), _and(d.valid, k.valid))
    return f


def _f_datediff(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    a, b = (materialize(_days(c)) for c in _args(e, scope, ctx, subst))
    return PrimColumn("int", a.data - b.data, _and(a.valid, b.valid))


def _f_add_months(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    a, k = _args(e, scope, ctx, subst)
    d = materialize(_days(a))
    k = _num(k, n, dev)
    y, m, dd = F.civil_from_days(d.data)
    tot = y * 12 + (m - 1) + k.data.to(torch.int64)
    ny, nm = F.floor_div(tot, 12), tot % 12 + 1
    last = _month_len(ny, nm)
    return PrimColumn("date", F.days_from_civil(ny, nm, torch.minimum(dd, last)), _and(d.valid, k.valid))


def _month_len(y, m):
    nxt_y = torch.where(m == 12, y + 1, y)
    nxt_m = torch.where(m == 12, torch.ones_like(m), m + 1)
    return F.days_from_civil(nxt_y, nxt_m, torch.ones_like(m)) - F.days_from_civil(y, m, torch.ones_like(m))


def _f_last_day(e, scope, ctx, subst):
    (a,) = _args(e, scope, ctx, subst)
    d = materialize(_days(a))
    y, m, _ = F.civil_from_days(d.data)
    return PrimColumn("date", F.days_from_civil(y, m, _month_len(y, m)), d.valid)


def _f_months_between(e, scope, ctx, subst):
    args = _args(e, scope, ctx, subst)
    a, b = (materialize(_ts(c)) for c in args[:2])

    def parts(us):
        days = F.floor_div(us, F.US_PER_DAY)
        y, m, d = F.civil_from_days(days)
        sec = _true_div((us - days * F.US_PER_DAY).to(torch.float64), 1e6)
        return y, m, d, sec, _month_len(y, m)
    ya, ma, da, sa, la = parts(a.data)
    yb, mb, db, sb, lb = parts(b.data)
    months = ((ya - yb) * 12 + (ma - mb)).to(torch.float64)
    same = (da == db) | ((da == la) & (db == lb))
    frac = ((da - db).to(torch.float64) * 86400 + (sa - sb)) / (31 * 86400)
    r = torch.where(same, months, months + frac)
    r = torch.round(r * 1e8) / 1e8
    return PrimColumn("double", r, _and(a.valid, b.valid))


def _f_weekofyear(e, scope, ctx, subst):
    (a,) = _args(e, scope, ctx, subst)
    d = materialize(_days(a))
    # ISO week: the Thursday of this week decides the year
    wd = (d.data + 3) % 7                                         # 0 = Monday
    thu = d.data - wd + 3
    y, _, _ = F.civil_from_days(thu)
    jan1 = F.days_from_civil(y, torch.ones_like(y), torch.ones_like(y))
    return PrimColumn("int", F.floor_div(thu - jan1, 7) + 1, d.valid)


def _f_make_date(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    y, m, d = (_num(c, n, dev) for c in _args(e, scope, ctx, subst))
    yy, mm, ddd = (c.data.to(torch.int64) for c in (y, m, d))
    ok = (mm >= 1) & (mm <= 12) & (ddd >= 1)
    mm_s = torch.where(ok, mm, torch.ones_like(mm))
    ok = ok & (ddd <= _month_len(yy, mm_s))
    return PrimColumn("date", F.days_from_civil(yy, mm_s, torch.where(ok, ddd, torch.ones_like(ddd))),
                      _and(y.valid, m.valid, d.valid, ok))


_TOKEN = re.compile(r"'([^']|'')*'|([A-Za-z])\2*|.", re.S)
# fixed-width device codes (strings.hip ts_format_kernel)
_FIXED = {"yyyy": (1, 4), "yy": (2, 2), "MM": (3, 2), "dd": (4, 2), "HH": (5, 2), "hh": (6, 2), "mm": (7, 2),
          "ss": (8, 2), "SSS": (9, 3), "SSSSSS": (10, 6), "a": (11, 2), "MMM": (12, 3), "EEE": (13, 3),
          "DDD": (14, 3)}


def _tokens(fmt: str):
    out = []
    for m in _TOKEN.finditer(fmt):
        t = m.group(0)
        if t.startswith("'"):
            out.append(("lit", t[1:-1].replace("''", "'") if t != "''" else "'"))
        elif t[0].isalpha():
            out.append(("pat", t))
        else:
            out.append(("lit", t))
    return out


def compile_pattern(fmt: str):
    """(ops, literal bytes, width) for a fixed-width Java date pattern, or None (variable-width tokens)."""
    ops, lits = [], bytearray()
    width = 0
    for kind, t in _tokens(fmt):
        if kind == "lit":
            b = t.encode("utf-8")
            if not b:
                continue
            if len(b) > 255 or len(lits) + len(b) > 65535:
                return None
            ops.append(0 | (len(lits) << 8) | (len(b) << 24))
            lits += b
            width += len(b)
            continue
        if t not in _FIXED:
            return None
        code, w = _FIXED[t]
        ops.append(code)
        width += w
    return ops, bytes(lits), width


def _java_format(us: int, fmt: str) -> str:
    t = _EPOCH + _dt.timedelta(microseconds=us)
    out = []
    for kind, tok in _tokens(fmt):
        if kind == "lit":
            out.append(tok)
            continue
        c, k = tok[0], len(tok)
        if c == "y":
            out.append(f"{t.year % 100:02d}" if k == 2 else f"{t.year:0{max(k, 4) if k != 1 else 1}d}")
        elif c == "M":
            out.append(t.strftime("%B") if k >= 4 else t.strftime("%b") if k == 3 else f"{t.month:0{k}d}")
        elif c == "d":
            out.append(f"{t.day:0{k}d}")
        elif c == "D":
            out.append(f"{t.timetuple().tm_yday:0{k}d}")
        elif c == "H":
            out.append(f"{t.hour:0{k}d}")
        elif c == "h":
            out.append(f"{(t.hour % 12) or 12:0{k}d}")
        elif c == "m":
            out.append(f"{t.minute:0{k}d}")
        elif c == "s":
            out.append(f"{t.second:0{k}d}")
        elif c == "S":
            out.append(f"{t.microsecond:06d}"[:k].ljust(k, "0"))
        elif c == "a":
            out.append("AM" if t.hour < 12 else "PM")
        elif c == "E":
            out.append(t.strftime("%A") if k >= 4 else t.strftime("%a"))
        elif c in "XxZ":
            out.append("Z" if c == "X" else "+0000")
        elif c == "z":
            out.append("UTC")
        elif c == "u":                                 # day number of week, 1 = Monday … 7 = Sunday
            out.append(f"{t.isoweekday():0{k}d}")
        elif c == "F":                                 # day of week in month (the n-th such weekday)
            out.append(f"{(t.day - 1) // 7 + 1:0{k}d}")
        elif c == "k":                                 # hour 1-24
            out.append(f"{t.hour or 24:0{k}d}")
        elif c == "K":                                 # hour 0-11
            out.append(f"{t.hour % 12:0{k}d}")
        elif c == "L":                                 # stand-alone month
            out.append(t.strftime("%B") if k >= 4 else t.strftime("%b") if k == 3 else f"{t.month:0{k}d}")
        elif c == "G":
            out.append("AD")
        elif c in "wW":
            out.append(f"{_us_week(t.date(), c == 'W'):0{k}d}")
        else:
            raise EvalError(f"unsupported date pattern letter {c!r}")
    return "".join(out)


def _us_week(d: "_dt.date", in_month: bool) -> int:
    """SimpleDateFormat 'w' / 'W' in the US locale Spark 2.4's formatter uses: weeks start on Sunday and the week
    holding the 1st (of the year / month) is week 1; late-December days in the week that holds the next January 1st
    are week 1 of that year."""
    sun = d - _dt.timedelta(days=(d.weekday() + 1) % 7)
    if not in_month and (sun + _dt.timedelta(days=6)).year > d.year:
        return 1
    first = _dt.date(d.year, d.month if in_month else 1, 1)
    first_sun = first - _dt.timedelta(days=(first.weekday() + 1) % 7)
    return (sun - first_sun).days // 7 + 1


def format_timestamps(ts: Column, fmt: str) -> Column:
    """Timestamp column → strings in a Java ``SimpleDateFormat`` pattern (UTC)."""
    n, dev = ts.length, ts.device
    if isinstance(ts, ConstColumn):
        return ConstColumn(None if ts.value is None else _java_format(int(ts.value), fmt), "string", n, dev)
    comp = compile_pattern(fmt) if dev.type == "cuda" else None
    if comp is not None and n:
        from ..ops import native as N
        ops, lits, width = comp
        opt = torch.tensor(ops or [0], dtype=torch.int32).to(dev, non_blocking=True)
        lt = torch.frombuffer(bytearray(lits + b"\0"), dtype=torch.uint8).to(dev, non_blocking=True)
        arena = torch.empty(n * width + 16, dtype=torch.uint8, device=dev)
        arena[n * width:].zero_()
        data = ts.data.to(torch.int64).contiguous()
        N.call("dxa_ts_format", N.ptr(data), n, N.ptr(opt), len(ops), N.ptr(lt), width, N.ptr(arena),
               N.stream_handle(dev))
        starts = torch.arange(n, dtype=torch.int64, device=dev) * width
        col = StrColumn(arena, starts, torch.full((n,), width, dtype=torch.int32, device=dev), ts.valid)
        col._keep = (opt, lt)
        return col
    vals = ts.data.cpu().tolist()
    ok = ts.valid.cpu().tolist() if ts.valid is not None else [True] * n
    return strings_from_pylist([_java_format(int(v), fmt) if k else None for v, k in zip(vals, ok)], dev)


def _fmt_arg(e, scope, ctx, subst, k, default):
    if len(e.args) <= k:
        return default
    f = evaluate(e.args[k], scope, ctx, subst)
    if not isinstance(f, ConstColumn):
        raise EvalError("date pattern must be a constant")
    return str(f.value)


def _f_date_format(e, scope, ctx, subst):
    a = evaluate(e.args[0], scope, ctx, subst)
    return format_timestamps(_ts(a) if a.dtype != "date" else cast_column(a, "timestamp"),
                             _fmt_arg(e, scope, ctx, subst, 1, "yyyy-MM-dd HH:mm:ss"))


def _f_from_unixtime(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    a = _num(evaluate(e.args[0], scope, ctx, subst), n, dev)
    sec = a.data.to(torch.int64) if a.data.dtype != torch.float64 else a.data.floor().to(torch.int64)
    return format_timestamps(PrimColumn("timestamp", sec * 1_000_000, a.valid),
                             _fmt_arg(e, scope, ctx, subst, 1, "yyyy-MM-dd HH:mm:ss"))


# java.time.ZoneId.SHORT_IDS, which java.util.TimeZone.getTimeZone (Spark 2.4's DateTimeUtils.getTimeZone) honours;
# EST / MST / HST are fixed offsets there
_JAVA_SHORT_IDS = {
    "ACT": "Australia/Darwin", "AET": "Australia/Sydney", "AGT": "America/Argentina/Buenos_Aires",
    "ART": "Africa/Cairo", "AST": "America/Anchorage", "BET": "America/Sao_Paulo", "BST": "Asia/Dhaka",
    "CAT": "Africa/Harare", "CNT": "America/St_Johns", "CST": "America/Chicago", "CTT": "Asia/Shanghai",
    "EAT": "Africa/Addis_Ababa", "ECT": "Europe/Paris", "IET": "America/Indiana/Indianapolis",
    "IST": "Asia/Kolkata", "JST": "Asia/Tokyo", "MIT": "Pacific/Apia", "NET": "Asia/Yerevan",
    "NST": "Pacific/Auckland", "PLT": "Asia/Karachi", "PNT": "America/Phoenix", "PRT": "America/Puerto_Rico",
    "PST": "America/Los_Angeles", "SST": "Pacific/Guadalcanal", "VST": "Asia/Ho_Chi_Minh"}
_JAVA_FIXED = {"EST": -5 * 60, "MST": -7 * 60, "HST": -10 * 60}
_GMT_OFFSET = re.compile(r"^(?:GMT|UTC)([+-])(\d{1,2})(?::?(\d{2}))?$")


def java_time_zone(tz: str):
    """tzinfo for a zone id as java.util.TimeZone.getTimeZone reads it: region ids, the legacy three-letter ids
    (``PST``, ``CTT``, … via ZoneId.SHORT_IDS; ``EST`` / ``MST`` / ``HST`` fixed), ``GMT+8`` / ``GMT-08:00``
    custom offsets, and — like Java — GMT for an id it does not know."""
    from zoneinfo import ZoneInfo
    t = str(tz).strip()
    if t in _JAVA_FIXED:
        return _dt.timezone(_dt.timedelta(minutes=_JAVA_FIXED[t]))
    if t in _JAVA_SHORT_IDS:
        return ZoneInfo(_JAVA_SHORT_IDS[t])
    m = _GMT_OFFSET.match(t)
    if m:
        mins = int(m.group(2)) * 60 + int(m.group(3) or 0)
        return _dt.timezone(_dt.timedelta(minutes=-mins if m.group(1) == "-" else mins))
    try:
        return ZoneInfo(t)
    except Exception:  # noqa: BLE001 — unknown ids are GMT in Java
        return _dt.timezone.utc


def _tz_shift(to_utc: bool):
    """to_utc_timestamp(ts, tz): ts is wall-clock time in tz → UTC.  from_utc_timestamp(ts, tz): UTC → wall clock
    in tz.  Host-assisted (zone rules from the system tz database)."""
    def f(e, scope, ctx, subst):
        a = materialize(_ts(evaluate(e.args[0], scope, ctx, subst)))
        tz = _fmt_arg(e, scope, ctx, subst, 1, "UTC")
        z = java_time_zone(tz)
        out = []
        for v in a.data.cpu().tolist():
            t = _EPOCH + _dt.timedelta(microseconds=int(v))
            if to_utc:
                off = t.replace(tzinfo=z).utcoffset()
            else:
                off = t.replace(tzinfo=_dt.timezone.utc).astimezone(z).utcoffset()
            us = int(off.total_seconds() * 1_000_000) if off is not None else 0
            out.append(int(v) - us if to_utc else int(v) + us)
        return PrimColumn("timestamp", _h2d(out, torch.int64, a.device), a.valid)
    return f


# ---------------------------------------------------------------------------------------------------------------
# arrays
# ---------------------------------------------------------------------------------------------------------------

_META = set(".$|()[]{}^?*+\\")


def _literal_delim(pat: str) -> Optional[bytes]:
    """A regex that only matches one fixed string (``','``, ``'\\|'``, ``'::'``) → that string."""
    out, i = [], 0
    while i < len(pat):
        c = pat[i]
        if c == "\\" and i + 1 < len(pat) and not pat[i + 1].isalnum():
            out.append(pat[i + 1])
            i += 2
            continue
        if c in _META:
            return None
        out.append(c)
        i += 1
    s = "".join(out)
    return s.encode("utf-8") if s else None


def array_from_pylist(lists, elem_type, device) -> ArrayColumn:
    n = len(lists)
    k = max((len(l) for l in lists if l is not None), default=0)
    els = [column_from_pylist([l[j] if l is not None and j < len(l) else None for l in lists], elem_type, device)
           for j in range(max(k, 1))]
    valid = None if all(l is not None for l in lists) else torch.tensor([l is not None for l in lists],
                                                                       dtype=torch.bool, device=device)
    if all(len(l) == k for l in lists if l is not None) and k:
        return ArrayColumn(els, n, valid, False, device)
    # rows of different lengths: a presence mask keeps real null elements (drop_nulls would lose them)
    present = torch.tensor([[l is not None and j < len(l) for j in range(max(k, 1))] for l in lists],
                           dtype=torch.bool, device=device).reshape(n, max(k, 1))
    return ArrayColumn(els, n, valid, False, device, present=present)


def split_strings(col: Column, pattern: str, limit: int = -1) -> ArrayColumn:
    n, dev = col.length, col.device
    if not isinstance(col, StrColumn):
        col = cast_column(col, "string")
    if isinstance(col, ConstColumn):
        col = materialize(col)
    d = _literal_delim(pattern)
    if col.starts.is_cuda and d is not None and limit <= 0 and n:
        from ..ops import native as N
        st = N.stream_handle(dev)
        dt = torch.frombuffer(bytearray(d), dtype=torch.uint8).to(dev, non_blocking=True)
        cnt = torch.empty(n, dtype=torch.int32, device=dev)
        N.call("dxa_str_split_count", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n, N.ptr(dt), len(d),
               N.ptr(cnt), st)
        K = int(cnt.max().item())                                       # slot count: the one host read
        ostarts = torch.empty((K, n), dtype=torch.int64, device=dev)
        olens = torch.empty((K, n), dtype=torch.int32, device=dev)
        N.call("dxa_str_split_write", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n, N.ptr(dt), len(d),
               K, N.ptr(ostarts), N.ptr(olens), st)
        row_ok = col.valid
        els = []
        for j in range(K):
            present = olens[j] >= 0
            v = present if row_ok is None else (present & row_ok)
            els.append(StrColumn(col.arena, ostarts[j], torch.clamp(olens[j], min=0), v))
        out = ArrayColumn(els, n, row_ok, True, dev)
        out._keep = dt
        return out
    rx = re.compile(pattern)
    vals = col.to_pylist()
    lists = []
    for v in vals:
        if v is None:
            lists.append(None)
            continue
        parts = rx.split(v, maxsplit=max(0, limit - 1)) if limit > 0 else rx.split(v)
        lists.append(parts)
    return array_from_pylist(lists, "string", dev)


def _f_split(e, scope, ctx, subst):
    a = evaluate(e.args[0], scope, ctx, subst)
    p = evaluate(e.args[1], scope, ctx, subst)
    lim = int(evaluate(e.args[2], scope, ctx, subst).value) if len(e.args) > 2 else -1
    if not isinstance(p, ConstColumn):
        raise EvalError("split() pattern must be a constant")
    if isinstance(a, ConstColumn):
        a = a.materialize()
    return split_strings(a, str(p.value), lim)


def _f_array_contains(e, scope, ctx, subst):
    from .expr import _compare
    n, dev = scope.length, scope.device
    arr, v = _args(e, scope, ctx, subst)
    if not isinstance(arr, ArrayColumn):
        raise EvalError("array_contains() expects an array")
    acc = torch.zeros(n, dtype=torch.bool, device=dev)
    for el in arr.elements:
        eq = _compare("=", el, v, n, dev)
        if isinstance(eq, ConstColumn):          # a literal array against a literal value
            eq = eq.materialize()
        acc = acc | (eq.data.bool() & eq.valid_mask() & _slot_present(arr, el))
    return bool_col(acc, arr.valid)


def _nan_key(x):
    return (isinstance(x, float) and x != x, x if not (isinstance(x, float) and x != x) else 0.0)


def _host_array_fn(fn, elem_type_of=None, scalar_type=None):
    """Array function evaluated per row on the host: fn(list, *args) → list (array result) or value."""
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        args = _args(e, scope, ctx, subst)
        arr = args[0]
        if not isinstance(arr, ArrayColumn):
            raise EvalError(f"{e.name}() expects an array")
        lists = arr.to_pylist()
        extra = [a.to_pylist() if not isinstance(a, ConstColumn) else [a.value] * n for a in args[1:]]
        out = [None if l is None else fn(l, *[x[i] for x in extra]) for i, l in enumerate(lists)]
        et = str(arr.elements[0].dtype) if arr.elements else "string"
        if scalar_type is not None:
            return column_from_pylist(out, scalar_type if scalar_type != "elem" else et, dev)
        return array_from_pylist(out, elem_type_of or et, dev)
    return f


def _f_slice(l, start, length):
    # Spark 2.4 Slice: a negative start counts from the end; a start index before the first element (or past the
    # last) gives an empty array, not a clipped one
    start, length = int(start), int(length)
    if start == 0:
        raise EvalError("slice: SQL array indices start at 1")
    if length < 0:
        raise EvalError("slice: length must be greater than or equal to 0")
    s = start - 1 if start > 0 else len(l) + start
    if s < 0 or s >= len(l):
        return []
    return l[s:s + length]


def _f_sequence(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    args = _args(e, scope, ctx, subst)
    cols = [a.to_pylist() if not isinstance(a, ConstColumn) else [a.value] * n for a in args]
    out = []
    for i in range(n):
        a, b = cols[0][i], cols[1][i]
        st = cols[2][i] if len(cols) > 2 else (1 if b >= a else -1)
        out.append(None if a is None or b is None else list(range(int(a), int(b) + (1 if st > 0 else -1), int(st))))
    return array_from_pylist(out, "long", dev)


def _f_map_part(which):
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        (m,) = _args(e, scope, ctx, subst)
        if not (isinstance(m, StructColumn) and m.is_map):
            raise EvalError(f"{e.name}() expects a map")
        if which == "keys":
            els = [ConstColumn(k, "string", n, dev).materialize().with_valid(c.valid_mask() if c.valid is not None
                                                                          else None)
                   for k, c in zip(m.names, m.children)]
            return ArrayColumn(els, n, m.valid, True, dev)
        return ArrayColumn(list(m.children), n, m.valid, True, dev)
    return f


# ---------------------------------------------------------------------------------------------------------------
# hashing / encoding
# ---------------------------------------------------------------------------------------------------------------

def _sha2(s, bits=256):
    bits = int(bits)
    h = {224: hashlib.sha224, 256: hashlib.sha256, 0: hashlib.sha256, 384: hashlib.sha384,
         512: hashlib.sha512}.get(bits)
    return None if h is None else h(_bytes_of(s)).hexdigest()


def _java_regex(p):
    from ..ops.regex_dfa import java_to_python
    return re.compile(java_to_python(str(p)), re.ASCII)


def _host_regexp_extract(s, p, g=1):
    m = _java_regex(p).search(str(s))
    return (m.group(int(g)) or "") if m else ""


def _host_regexp_replace(s, p, r):
    """Java Matcher.replaceAll: after an empty match the next search starts one character later (Python's re.sub
    would retry the same position for a non-empty match, which Java does not)."""
    from ..ops.regex_vm import replacement_tokens
    rx = _java_regex(p)
    toks = replacement_tokens(str(r), rx.groups)
    s = str(s)

    def expand(m):
        out = bytearray()
        for t in toks:
            if t >= 0:
                out.append(t)
            else:
                out += (m.group(-1 - t) or "").encode("utf-8")
        return out.decode("utf-8")
    out, pos, last = [], 0, 0
    while pos <= len(s):
        m = rx.search(s, pos)
        if m is None:
            break
        out.append(s[last:m.start()])
        out.append(expand(m))
        last = m.end()
        pos = m.end() if m.end() > m.start() else m.end() + 1
    out.append(s[last:])
    return "".join(out)


def _f_regexp(kind):
    """regexp_extract / regexp_replace: the backtracking program on the device (ops/regex_vm.py) for device string
    columns with a constant pattern; rows over the kernel's budget and everything else go to the host regex (Java
    syntax read the Java way)."""
    host = _host_regexp_extract if kind == "extract" else _host_regexp_replace

    def f(e, scope, ctx, subst):
        args = _args(e, scope, ctx, subst)
        a = args[0] if args else None
        consts = all(isinstance(x, ConstColumn) and x.value is not None for x in args[1:])
        if _gpu_str(a) and consts and len(args) >= 2:
            from ..ops import regex_vm, strings as S
            try:
                prog = regex_vm.compile_vm(str(args[1].value))
                if kind == "extract":
                    g = int(args[2].value) if len(args) > 2 else 1
                    if not 0 <= g <= min(prog.ngroups, regex_vm.MAX_GROUPS):
                        raise regex_vm.Unsupported("group index")
                    out, bad = S.regex_extract(a, prog, g)
                else:
                    toks = regex_vm.replacement_tokens(str(args[2].value) if len(args) > 2 else "", prog.ngroups)
                    out, bad = S.regex_replace(a, prog, toks)
                if not bool(bad.any()):
                    return out
            except regex_vm.Unsupported:
                pass
        return _host_string_fn(host)(e, scope, ctx, subst)
    return f


def _sha2_kind(args):
    b = args[1] if len(args) > 1 else None
    if b is None or not isinstance(b, ConstColumn) or b.value is None:
        return None
    return {0: 2, 256: 2, 224: 3}.get(int(b.value))          # 384 / 512: host


def _f_digest(kind, host, out_type="string"):
    """md5 / sha1 / sha2 / crc32 / hex / base64: device kernels (ops/csrc/digest.hip) for device string columns,
    the host function otherwise (constants, numeric hex, sha2 384/512)."""
    def f(e, scope, ctx, subst):
        args = _args(e, scope, ctx, subst)
        a = args[0] if args else None
        k = kind(args) if callable(kind) else kind
        if k is not None and _gpu_str(a):
            from ..ops import strings as S
            if k == "crc32":
                return PrimColumn("long", S.crc32(a), a.valid)
            if k in ("hex", "base64"):
                return S.encode(a, 0 if k == "hex" else 1)
            return S.digest(a, k)
        return _host_string_fn(host, out_type)(e, scope, ctx, subst)
    return f


def _hex(v):
    if isinstance(v, (int, bool)) and not isinstance(v, bool):
        return format(v & 0xFFFFFFFFFFFFFFFF, "X") if v < 0 else format(v, "X")
    return _bytes_of(v).hex().upper()


def _bytes_of(v) -> bytes:
    """A string's UTF-8 bytes, or a binary value's own bytes (encode / unhex / unbase64 results)."""
    return bytes(v) if isinstance(v, (bytes, bytearray)) else str(v).encode()


def _initcap(s):
    return " ".join(w[:1].upper() + w[1:].lower() for w in str(s).split(" "))


def _translate(s, frm, to):
    s, frm, to = str(s), str(frm), str(to)
    table = {}
    for i, c in enumerate(frm):
        if c not in table:
            table[c] = to[i] if i < len(to) else None
    return "".join(table.get(c, c) or "" if c in table else c for c in s)


# Spark's hash(): Murmur3_x86_32, seed 42 chained through the arguments (HashExpression / Murmur3Hash), with its
# byte-at-a-time tail for strings (Murmur3_x86_32.hashUnsafeBytes).
_M32 = 0xFFFFFFFF


def _rotl(x, r):
    return ((x << r) | (x >> (32 - r))) & _M32


def _mix_k1(k1):
    k1 = (k1 * 0xCC9E2D51) & _M32
    return (_rotl(k1, 15) * 0x1B873593) & _M32


def _mix_h1(h1, k1):
    h1 ^= k1
    return (_rotl(h1, 13) * 5 + 0xE6546B64) & _M32


def _fmix(h1, length):
    h1 ^= length
    h1 ^= h1 >> 16
    h1 = (h1 * 0x85EBCA6B) & _M32
    h1 ^= h1 >> 13
    h1 = (h1 * 0xC2B2AE35) & _M32
    return h1 ^ (h1 >> 16)


def _hash_int(v, seed):
    return _fmix(_mix_h1(seed, _mix_k1(v & _M32)), 4)


def _hash_long(v, seed):
    v &= 0xFFFFFFFFFFFFFFFF
    h1 = _mix_h1(seed, _mix_k1(v & _M32))
    return _fmix(_mix_h1(h1, _mix_k1(v >> 32)), 8)


def _hash_bytes(b: bytes, seed):
    h1 = seed
    aligned = len(b) - len(b) % 4
    for i in range(0, aligned, 4):
        h1 = _mix_h1(h1, _mix_k1(int.from_bytes(b[i:i + 4], "little")))
    for i in range(aligned, len(b)):
        x = b[i] - 256 if b[i] >= 128 else b[i]                     # Java byte: signed
        h1 = _mix_h1(h1, _mix_k1(x & _M32))
    return _fmix(h1, len(b))


def spark_hash_value(v, dtype, seed):
    """One argument of Spark's hash() (Murmur3Hash, HashExpression): int/date/boolean → hashInt, long/timestamp →
    hashLong, float → hashInt(floatToIntBits), double → hashLong(doubleToLongBits) (-0.0 as 0.0, NaN canonical),
    decimal(p, s) → hashLong(unscaled) for p ≤ 18 else the unscaled BigInteger's two's-complement bytes (the
    column's precision decides, not the value's)."""
    import math
    import struct
    if v is None:
        return seed
    if dtype in ("byte", "short", "int", "date") or isinstance(v, bool):
        return _hash_int(int(v), seed)
    if dtype in ("long", "timestamp"):
        return _hash_long(int(v), seed)
    if dtype == "float":
        f = struct.unpack("<f", struct.pack("<f", float(v)))[0]
        bits = 0x7FC00000 if math.isnan(f) else struct.unpack("<I", struct.pack("<f", 0.0 if f == 0 else f))[0]
        return _hash_int(bits, seed)
    if dtype == "double":
        d = 0.0 if v == 0 else float(v)                                   # -0.0 hashes as 0.0
        bits = 0x7FF8000000000000 if math.isnan(d) else struct.unpack("<Q", struct.pack("<d", d))[0]
        return _hash_long(bits, seed)
    from .decimal import is_decimal
    if is_decimal(dtype):
        # the column's unscaled integer: storage int (narrow), [lo, hi] words (wide), or a Python Decimal (literals)
        if isinstance(v, list):
            lo, hi = int(v[0]), int(v[1])
            unscaled = (hi << 64) | (lo & ((1 << 64) - 1))
        elif isinstance(v, int):
            unscaled = v
        else:
            from decimal import Decimal
            unscaled = int(Decimal(str(v)).scaleb(dtype.scale))
        if dtype.precision <= 18:                                   # DecimalType.MAX_LONG_DIGITS
            return _hash_long(unscaled, seed)
        nbytes = (unscaled.bit_length() + 8) // 8                  # BigInteger.toByteArray: minimal two's complement
        return _hash_bytes(unscaled.to_bytes(nbytes, "big", signed=True), seed)
    if isinstance(v, (dict, list)):
        v = json.dumps(v, separators=(",", ":"))
    return _hash_bytes(str(v).encode("utf-8"), seed)


def _is_dec(t):
    from .decimal import is_decimal
    return is_decimal(t)


_HASH_KIND = {"byte": 0, "short": 0, "int": 0, "date": 0, "long": 1, "timestamp": 1, "double": 2, "float": 3, "boolean": 4}


def _hash_device(args, n, dev):
    """hash() on the device (spark_hash.hip): one launch per argument folding into an int32 per-row state; None
    when an argument type needs the host path (decimal, nested)."""
    from ..ops import native as N
    from .column import StrColumn, materialize
    cols = []
    for a in args:
        a = materialize(a) if isinstance(a, ConstColumn) else a
        if isinstance(a, StrColumn):
            cols.append(("s", a))
        elif isinstance(a, PrimColumn) and str(a.dtype) in _HASH_KIND:
            cols.append(("p", a))
        elif isinstance(a, PrimColumn) and _is_dec(a.dtype) and a.dtype.narrow:
            cols.append(("p", PrimColumn("long", a.data, a.valid)))    # hashLong(unscaled): the storage word
        else:
            return None
    h = torch.full((n,), 42, dtype=torch.int32, device=dev)
    st = N.stream_handle(dev)
    for kind, a in cols:
        v = None if a.valid is None else N.u8(a.valid.contiguous())
        if kind == "s":
            N.call("dxa_spark_hash_str", N.ptr(a.arena), N.ptr(a.starts), N.ptr(a.lens.contiguous()),
                   N.ptr(v) if v is not None else None, n, N.ptr(h), st)
        else:
            d = a.data.contiguous()
            d = d.view(torch.uint8) if d.dtype == torch.bool else d
            N.call("dxa_spark_hash_fixed", N.ptr(d), _HASH_KIND[str(a.dtype)], N.ptr(v) if v is not None else None,
                   n, N.ptr(h), st)
    return PrimColumn("int", h.to(torch.int64))


def _f_hash(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    args = _args(e, scope, ctx, subst)
    if dev.type == "cuda":
        out = _hash_device(args, n, dev)
        if out is not None:
            return out
    from .column import ts_to_datetime  # noqa: F401  (storage values below, not datetimes)
    cols = []
    for a in args:
        if isinstance(a, ConstColumn):
            cols.append(([a.value] * n, a.dtype if _is_dec(a.dtype) else str(a.dtype)))
        elif isinstance(a, PrimColumn):
            vals = a.data.cpu().tolist()
            ok = a.valid.cpu().tolist() if a.valid is not None else None
            cols.append(([v if (ok is None or ok[i]) else None for i, v in enumerate(vals)],
                         a.dtype if _is_dec(a.dtype) else str(a.dtype)))
        else:
            cols.append((a.to_pylist(), str(a.dtype)))
    out = []
    for i in range(n):
        h = 42
        for vals, dt in cols:
            h = spark_hash_value(vals[i], dt, h)
        out.append(h - (1 << 32) if h >= (1 << 31) else h)
    return column_from_pylist(out, "int", dev)


# ---------------------------------------------------------------------------------------------------------------
# JSON
# ---------------------------------------------------------------------------------------------------------------

_PATH = re.compile(r"\.([^.\[]+)|\[(\d+)\]|\['([^']+)'\]")


def _json_path(doc, path: str):
    if not path.startswith("$"):
        return None
    cur = doc
    for m in _PATH.finditer(path[1:]):
        key = m.group(1) or m.group(3)
        if key is not None:
            if key == "*" or not isinstance(cur, dict) or key not in cur:
                return None
            cur = cur[key]
        else:
            i = int(m.group(2))
            if not isinstance(cur, list) or i >= len(cur):
                return None
            cur = cur[i]
    return cur


def _get_json_object(s, path):
    try:
        v = _json_path(json.loads(s), str(path))
    except (ValueError, TypeError):
        return None
    if v is None:
        return None
    if isinstance(v, str):
        return v
    if isinstance(v, bool):
        return "true" if v else "false"
    return json.dumps(v, separators=(",", ":"))


_SIMPLE_PATH = re.compile(r"^\$((?:\.[A-Za-z_][A-Za-z0-9_]*)+)$")


def _f_get_json_object(e, scope, ctx, subst):
    """get_json_object(json, '$.a.b'): on the GPU a dotted path becomes a one-leaf schema for the batch JSON
    parser (the leaf read as a string: string values unquoted, anything else as its JSON text, as Spark returns
    it); array-index paths and host columns take the per-row host path."""
    a = evaluate(e.args[0], scope, ctx, subst)
    p = evaluate(e.args[1], scope, ctx, subst)
    m = _SIMPLE_PATH.match(str(p.value)) if isinstance(p, ConstColumn) and p.value is not None else None
    if m is None or isinstance(a, ConstColumn) or not a.device.type == "cuda":
        return _host_string_fn(_get_json_object)(e, scope, ctx, subst)
    from ..ops.jsonparse import ParsePlan, parse
    from .types import StructField, StructType
    keys = m.group(1)[1:].split(".")
    t = "string"
    for k in reversed(keys):
        t = StructType((StructField(k, t),))
    if not isinstance(a, StrColumn):
        a = cast_column(a, "string")
    c = a.compact()                                 # the parser un-escapes in place: parse a private copy
    n, dev = c.length, c.device
    ends = c.starts + c.lens.to(torch.int64)
    offs = torch.cat([c.starts, ends[-1:] if n else torch.zeros(1, dtype=torch.int64, device=dev)])
    raw, ok = parse(c.arena, offs, ParsePlan(t), ends)
    col, valid = raw, ok if a.valid is None else (ok & a.valid)
    for k in keys:
        if col.valid is not None:
            valid = valid & col.valid
        col = col.child(k)
    if col.valid is not None:
        valid = valid & col.valid
    out = StrColumn(col.arena, col.starts, col.lens, valid)
    out._keep = c
    return out


def _f_from_json(e, scope, ctx, subst):
    """from_json(str, schema): the batch JSON parser (device kernel on the GPU) over a private copy of the column's
    bytes (the parser un-escapes in place)."""
    from ..ops.jsonparse import ParsePlan, parse
    from .types import StructType, parse_ddl_schema, schema_from_json
    n, dev = scope.length, scope.device
    a = evaluate(e.args[0], scope, ctx, subst)
    sch = evaluate(e.args[1], scope, ctx, subst)
    if not isinstance(sch, ConstColumn):
        raise EvalError("from_json() schema must be a constant")
    text = str(sch.value).strip()
    schema = schema_from_json(text) if text.startswith("{") else parse_ddl_schema(text)
    if not isinstance(schema, StructType):
        raise EvalError("from_json() supports struct schemas")
    if isinstance(a, ConstColumn):
        a = a.materialize()
    if not isinstance(a, StrColumn):
        a = cast_column(a, "string")
    c = a.compact()
    plan = ParsePlan(schema)
    ends = c.starts + c.lens.to(torch.int64)
    offs = torch.cat([c.starts, ends[-1:] if n else torch.zeros(1, dtype=torch.int64, device=dev)])
    raw, ok = parse(c.arena, offs, plan, ends)
    valid = ok if a.valid is None else (ok & a.valid)
    out = raw.with_valid(valid)
    out._keep = c
    return out


# ---------------------------------------------------------------------------------------------------------------

def _f_window(e, scope, ctx, subst):
    """window(ts, 'duration'[, 'slide'[, 'start offset']]) → struct<start, end> of the tumbling window holding ts
    (Spark's event-time window function).  Sliding windows (slide < duration) assign a row to several windows;
    DataX flows express those with TIMEWINDOW, which this engine evaluates incrementally."""
    from ..sql.parser import parse_duration_micros
    n, dev = scope.length, scope.device
    a = materialize(_ts(evaluate(e.args[0], scope, ctx, subst)))

    def dur(k, default=None):
        if len(e.args) <= k:
            return default
        c = evaluate(e.args[k], scope, ctx, subst)
        if not isinstance(c, ConstColumn):
            raise EvalError("window() durations must be constants")
        return c.value if isinstance(c.value, int) and c.dtype == "interval" else parse_duration_micros(str(c.value))
    size = dur(1)
    slide = dur(2, size)
    off = dur(3, 0)
    if not size or size <= 0:
        raise EvalError("window() duration must be positive")
    if slide != size:
        raise EvalError("sliding window() is expanded by the SELECT it appears in (query._sliding_windows)")
    start = F.floor_div(a.data - off, size) * size + off
    return StructColumn(["start", "end"], [PrimColumn("timestamp", start, a.valid),
                                           PrimColumn("timestamp", start + size, a.valid)], n, a.valid, False, None,
                        dev)


def window_params(e, scope, ctx):
    """(duration, slide, start offset) in microseconds of a ``window(ts, dur[, slide[, start]])`` call."""
    from ..sql.parser import parse_duration_micros

    def dur(k, default=None):
        if len(e.args) <= k:
            return default
        c = evaluate(e.args[k], scope, ctx)
        if not isinstance(c, ConstColumn):
            raise EvalError("window() durations must be constants")
        return c.value if isinstance(c.value, int) and c.dtype == "interval" else parse_duration_micros(str(c.value))
    size = dur(1)
    slide = dur(2, size)
    off = dur(3, 0)
    if not size or size <= 0 or not slide or slide <= 0:
        raise EvalError("window() duration and slide must be positive")
    if slide > size:
        raise EvalError("window() slide must not exceed the duration")
    return size, slide, off


def sliding_windows(e, scope, ctx):
    """Rows of a sliding ``window(ts, dur, slide[, start])`` expansion (Spark's TimeWindowing: every window
    [s, s + dur) with s ≡ start (mod slide) that holds ts; rows with a null ts produce none) →
    (input row of every output row, struct<start, end> column), in input-row order with windows latest-start
    first, as Spark's expansion emits them."""
    size, slide, off = window_params(e, scope, ctx)
    a = materialize(_ts(evaluate(e.args[0], scope, ctx)))
    n, dev = scope.length, scope.device
    k = -(-size // slide)
    ok = a.valid_mask()
    last = a.data - torch.remainder(a.data - off, slide)
    picks = []
    for j in range(k):
        st = last - j * slide
        m = ok & (a.data < st + size)
        picks.append(torch.nonzero(m).flatten() * k + j)
    code = torch.sort(torch.cat(picks)).values
    rows, j = code // k, code % k
    start = last[rows] - j * slide
    m = int(rows.shape[0])
    return rows, StructColumn(["start", "end"], [PrimColumn("timestamp", start), PrimColumn("timestamp", start + size)],
                              m, None, False, None, dev)


# ---------------------------------------------------------------------------------------------------------------
# character functions on the GPU (strings.hip): substring / trim / left / right are views into the same arena
# ---------------------------------------------------------------------------------------------------------------

def spark_substr(s: str, pos: int, length: Optional[int] = None) -> str:
    """UTF8String.substringSQL: 1-based pos, 0 treated as 1, negative from the end; end computed before the start
    is clamped."""
    n = len(s)
    start = pos - 1 if pos > 0 else (n + pos if pos < 0 else 0)
    end = n if length is None else start + length
    start = max(start, 0)
    if start >= end:
        return ""
    return s[start:end]


def _gpu_str(c) -> bool:
    return isinstance(c, StrColumn) and c.starts.is_cuda


def _int_arg(c, n, dev):
    """(per-row int64 tensor or None, constant, validity)."""
    if isinstance(c, ConstColumn):
        return None, (None if c.value is None else int(c.value)), None
    c = _num(c, n, dev)
    return c.data.to(torch.int64).contiguous(), 0, c.valid


def _view(col: StrColumn, starts, lens, valid) -> StrColumn:
    out = StrColumn(col.arena, starts, lens, valid)
    return out


def _f_substr(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    args = _args(e, scope, ctx, subst)
    a = args[0]
    if isinstance(a, ConstColumn) or not _gpu_str(a if isinstance(a, StrColumn) else None):
        def host(s, p, ln=None):
            return spark_substr(str(s), int(p), None if ln is None else int(ln))
        return _host_string_fn(host)(e, scope, ctx, subst)
    from ..ops import native as N
    pos_t, pos_c, pos_v = _int_arg(args[1], n, dev)
    if len(args) > 2:
        len_t, len_c, len_v = _int_arg(args[2], n, dev)
    else:
        len_t, len_c, len_v = None, 2**63 - 1, None
    if (pos_t is None and pos_c is None) or (len_t is None and len_c is None):
        return ConstColumn(None, "string", n, dev)
    os_ = torch.empty(n, dtype=torch.int64, device=dev)
    ol = torch.empty(n, dtype=torch.int32, device=dev)
    N.call("dxa_str_substr", N.ptr(a.arena), N.ptr(a.starts), N.ptr(a.lens), n, N.ptr(pos_t), pos_c or 0,
           N.ptr(len_t), len_c if len_c is not None else 0, N.ptr(os_), N.ptr(ol), N.stream_handle(dev))
    return _view(a, os_, ol, _and(a.valid, pos_v, len_v))


def _f_left_right(right: bool):
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        a, k = _args(e, scope, ctx, subst)
        if not isinstance(a, StrColumn) or not _gpu_str(a) or not isinstance(k, ConstColumn):
            fn = (lambda s, kk: str(s)[-int(kk):] if int(kk) > 0 else "") if right else \
                (lambda s, kk: str(s)[:max(0, int(kk))])
            return _host_string_fn(fn)(e, scope, ctx, subst)
        kk = int(k.value)
        from ..ops import native as N
        os_ = torch.empty(n, dtype=torch.int64, device=dev)
        ol = torch.empty(n, dtype=torch.int32, device=dev)
        if kk <= 0:
            return _view(a, a.starts, torch.zeros_like(a.lens), a.valid)
        pos, ln = (-kk, kk) if right else (1, kk)
        N.call("dxa_str_substr", N.ptr(a.arena), N.ptr(a.starts), N.ptr(a.lens), n, None, pos, None, ln,
               N.ptr(os_), N.ptr(ol), N.stream_handle(dev))
        return _view(a, os_, ol, a.valid)
    return f


def _f_trim(mode: int, py):
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        args = _args(e, scope, ctx, subst)
        a = args[0]
        if len(args) != 1 or not isinstance(a, StrColumn) or not _gpu_str(a):
            return _host_string_fn(py)(e, scope, ctx, subst)
        from ..ops import native as N
        os_ = torch.empty(n, dtype=torch.int64, device=dev)
        ol = torch.empty(n, dtype=torch.int32, device=dev)
        N.call("dxa_str_trim", N.ptr(a.arena), N.ptr(a.starts), N.ptr(a.lens), n, mode, N.ptr(os_), N.ptr(ol),
               N.stream_handle(dev))
        return _view(a, os_, ol, a.valid)
    return f


def _trim_py(chars_mode):
    def fn(s, t=" "):
        s, t = str(s), str(t)
        return s.strip(t) if chars_mode == 3 else s.lstrip(t) if chars_mode == 1 else s.rstrip(t)
    return fn


def _f_char_length(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    (a,) = _args(e, scope, ctx, subst)
    if isinstance(a, ConstColumn):
        return ConstColumn(None if a.value is None else len(str(a.value)), "int", n, dev)
    if not isinstance(a, StrColumn):
        a = cast_column(a, "string")
    if not _gpu_str(a):
        return column_from_pylist([None if v is None else len(v) for v in a.to_pylist()], "int", dev)
    from ..ops import native as N
    out = torch.empty(n, dtype=torch.int64, device=dev)
    N.call("dxa_str_numchars", N.ptr(a.arena), N.ptr(a.starts), N.ptr(a.lens), n, N.ptr(out), N.stream_handle(dev))
    return PrimColumn("int", out, a.valid)


def _locate_gpu(a: StrColumn, needle: str, start: int, n, dev):
    from ..ops import native as N
    b = needle.encode("utf-8")
    dt = torch.frombuffer(bytearray(b + b"\0"), dtype=torch.uint8).to(dev, non_blocking=True)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    N.call("dxa_str_locate", N.ptr(a.arena), N.ptr(a.starts), N.ptr(a.lens), n, N.ptr(dt), len(b), int(start),
           N.ptr(out), N.stream_handle(dev))
    r = PrimColumn("int", out, a.valid)
    r._keep = dt
    return r


def _spark_locate(sub, s, pos=1):
    pos = int(pos)
    if pos < 1:
        return 0
    sub, s = str(sub), str(s)
    if sub == "":
        return 1
    i = s.find(sub, pos - 1) if pos - 1 <= len(s) else -1
    return i + 1


def _f_instr(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    a, sub = _args(e, scope, ctx, subst)
    if isinstance(a, StrColumn) and _gpu_str(a) and isinstance(sub, ConstColumn) and sub.value is not None:
        return _locate_gpu(a, str(sub.value), 1, n, dev)
    return _host_string_fn(lambda s, x: _spark_locate(x, s, 1), "int")(e, scope, ctx, subst)


def _f_locate(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    args = _args(e, scope, ctx, subst)
    sub, a = args[0], args[1]
    pos = args[2] if len(args) > 2 else ConstColumn(1, "int", n, dev)
    if isinstance(a, StrColumn) and _gpu_str(a) and isinstance(sub, ConstColumn) and sub.value is not None and \
            isinstance(pos, ConstColumn) and pos.value is not None:
        return _locate_gpu(a, str(sub.value), int(pos.value), n, dev)
    lists = [x.to_pylist() if not isinstance(x, ConstColumn) else [x.value] * n for x in (sub, a, pos)]
    out = [None if any(v is None for v in vals) else _spark_locate(*vals) for vals in zip(*lists)]
    return column_from_pylist(out, "int", dev)


def _f_replace(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    args = _args(e, scope, ctx, subst)
    a = args[0]
    srch = args[1]
    rep = args[2] if len(args) > 2 else ConstColumn("", "string", n, dev)
    if not (isinstance(a, StrColumn) and _gpu_str(a) and isinstance(srch, ConstColumn) and
            isinstance(rep, ConstColumn) and srch.value is not None and rep.value is not None):
        return _host_string_fn(lambda s, x, y="": str(s).replace(str(x), str(y)) if str(x) else str(s))(
            e, scope, ctx, subst)
    sb, rb = str(srch.value).encode("utf-8"), str(rep.value).encode("utf-8")
    if not sb:
        return a
    from ..ops import native as N
    from ..ops.strings import _alloc_arena, _offsets
    st = N.stream_handle(dev)
    dt = torch.frombuffer(bytearray(sb + b"\0"), dtype=torch.uint8).to(dev, non_blocking=True)
    rt = torch.frombuffer(bytearray(rb + b"\0"), dtype=torch.uint8).to(dev, non_blocking=True)
    lens = torch.empty(n, dtype=torch.int64, device=dev)
    N.call("dxa_str_replace_len", N.ptr(a.arena), N.ptr(a.starts), N.ptr(a.lens), n, N.ptr(dt), len(sb), len(rb),
           N.ptr(lens), st)
    off, total = _offsets(lens)
    dst = _alloc_arena(total, dev)
    N.call("dxa_str_replace_write", N.ptr(a.arena), N.ptr(a.starts), N.ptr(a.lens), n, N.ptr(dt), len(sb),
           N.ptr(rt), len(rb), N.ptr(off), N.ptr(dst), st)
    out = StrColumn(dst, off, lens.to(torch.int32), a.valid)
    out._keep = (dt, rt)
    return out


def _register():
    reg = register_function
    reg("pow", _binary_double(torch.pow))
    reg("power", _binary_double(torch.pow))
    reg("atan2", _binary_double(torch.atan2))
    reg("hypot", _binary_double(torch.hypot))
    reg("log", _f_log)
    reg("log1p", _unary_double(torch.log1p))
    reg("expm1", _unary_double(torch.expm1))
    reg("cbrt", _unary_double(lambda x: torch.sign(x) * torch.abs(x).pow(1.0 / 3.0)))
    reg("degrees", _unary_double(torch.rad2deg))
    reg("radians", _unary_double(torch.deg2rad))
    for nm in ("sin", "cos", "tan", "asin", "acos", "atan", "sinh", "cosh", "tanh"):
        reg(nm, _unary_double(getattr(torch, nm)))
    reg("cot", _unary_double(lambda x: 1.0 / torch.tan(x)))
    reg("mod", _f_mod(False))
    reg("pmod", _f_mod(True))
    reg("e", _f_const(math.e))
    reg("pi", _f_const(math.pi))
    reg("rand", _f_rand(False))
    reg("random", _f_rand(False))
    reg("randn", _f_rand(True))
    reg("isnan", _f_isnan)
    reg("nanvl", _f_nanvl)
    reg("factorial", _host_string_fn(lambda x: math.factorial(int(x)) if 0 <= int(x) <= 20 else None, "long"))
    reg("bin", _host_string_fn(lambda x: format(int(x) & 0xFFFFFFFFFFFFFFFF, "b") if int(x) < 0
                               else format(int(x), "b")))
    for nm, to in (("string", "string"), ("int", "int"), ("integer", "int"), ("bigint", "long"), ("long", "long"),
                   ("smallint", "short"), ("short", "short"), ("tinyint", "byte"), ("byte", "byte"),
                   ("double", "double"), ("float", "double"), ("boolean", "boolean"), ("date", "date"),
                   ("timestamp", "timestamp")):
        reg(nm, _f_cast_to(to))
    reg("date_add", _f_date_add(1))
    reg("dateadd", _f_date_add(1))
    reg("date_sub", _f_date_add(-1))
    reg("datediff", _f_datediff)
    reg("add_months", _f_add_months)
    reg("last_day", _f_last_day)
    reg("months_between", _f_months_between)
    reg("weekofyear", _f_weekofyear)
    reg("make_date", _f_make_date)
    reg("date_format", _f_date_format)
    reg("from_unixtime", _f_from_unixtime)
    reg("to_utc_timestamp", _tz_shift(True))
    reg("from_utc_timestamp", _tz_shift(False))
    reg("split", _f_split)
    reg("array_contains", _f_array_contains)
    reg("array_join", _host_array_fn(lambda l, sep, nr=None: str(sep).join(
        str(x) if x is not None else str(nr) for x in l if x is not None or nr is not None), scalar_type="string"))
    # Spark orders NaN above every other double
    reg("array_max", _host_array_fn(lambda l: max((x for x in l if x is not None), default=None, key=_nan_key),
                                    scalar_type="elem"))
    reg("array_min", _host_array_fn(lambda l: min((x for x in l if x is not None), default=None, key=_nan_key),
                                    scalar_type="elem"))
    reg("sort_array", _host_array_fn(lambda l, asc=True: (
        [x for x in l if x is None] + sorted((x for x in l if x is not None), key=_nan_key)) if bool(asc) else
        (sorted((x for x in l if x is not None), key=_nan_key, reverse=True) + [x for x in l if x is None])))
    reg("array_sort", _host_array_fn(lambda l: sorted((x for x in l if x is not None), key=_nan_key) +
                                     [x for x in l if x is None]))
    reg("array_distinct", _host_array_fn(lambda l: list(dict.fromkeys(l))))
    reg("array_position", _host_array_fn(lambda l, v: next((i + 1 for i, x in enumerate(l) if x == v), 0),
                                         scalar_type="long"))
    reg("array_remove", _host_array_fn(lambda l, v: [x for x in l if x != v]))
    reg("slice", _host_array_fn(_f_slice))
    reg("sequence", _f_sequence)
    reg("map_keys", _f_map_part("keys"))
    reg("map_values", _f_map_part("values"))
    reg("regexp_extract", _f_regexp("extract"))
    reg("regexp_replace", _f_regexp("replace"))
    reg("sha2", _f_digest(_sha2_kind, _sha2))
    reg("sha", _f_digest(1, lambda s: hashlib.sha1(_bytes_of(s)).hexdigest()))
    reg("sha1", _f_digest(1, lambda s: hashlib.sha1(_bytes_of(s)).hexdigest()))
    reg("md5", _f_digest(0, lambda s: hashlib.md5(_bytes_of(s)).hexdigest()))
    reg("crc32", _f_digest("crc32", lambda s: zlib.crc32(_bytes_of(s)) & 0xFFFFFFFF, "long"))
    reg("base64", _f_digest("base64", lambda s: _b64.b64encode(_bytes_of(s)).decode()))
    reg("unbase64", _host_string_fn(lambda s: _unbase64(s)))
    reg("hex", _f_digest("hex", _hex))
    reg("unhex", _host_string_fn(lambda s: _unhex(s)))
    reg("initcap", _host_string_fn(_initcap))
    reg("repeat", _host_string_fn(lambda s, k: str(s) * max(0, int(k))))
    reg("left", _f_left_right(False))
    reg("right", _f_left_right(True))
    reg("substring", _f_substr)
    reg("substr", _f_substr)
    reg("trim", _f_trim(3, _trim_py(3)))
    reg("ltrim", _f_trim(1, _trim_py(1)))
    reg("rtrim", _f_trim(2, _trim_py(2)))
    reg("length", _f_char_length)
    reg("char_length", _f_char_length)
    reg("character_length", _f_char_length)
    reg("instr", _f_instr)
    reg("locate", _f_locate)
    reg("position", _f_locate)
    reg("replace", _f_replace)
    reg("translate", _host_string_fn(_translate))
    reg("ascii", _host_string_fn(lambda s: ord(str(s)[0]) if str(s) else 0, "int"))
    reg("get_json_object", _f_get_json_object)
    reg("from_json", _f_from_json)
    reg("hash", _f_hash)
    reg("window", _f_window)
    reg("tumble", _f_window)


_register()


# ---------------------------------------------------------------------------------------------------------------
# more Spark built-ins: bit ops, rint, width_bucket, next_day, typeof, spark_partition_id, timestamp_seconds and
# host-assisted text functions (format_number, conv, soundex, levenshtein, substring_index, format_string, …)
# ---------------------------------------------------------------------------------------------------------------

def _f_shift(kind):
    def f(e, scope, ctx, subst):
        n, dev = scope.length, scope.device
        a, k = _args(e, scope, ctx, subst)
        a, k = materialize(_num(a, n, dev)), materialize(_num(k, n, dev))
        x = a.data.to(torch.int64)
        if a.dtype in ("byte", "short", "int"):
            # Spark ShiftLeft / ShiftRight(Unsigned) on an INT (smaller types widen to it): Java's 32-bit shifts,
            # the count taken mod 32, the result an INT
            s = (k.data.to(torch.int64) & 31)
            if kind == "left":
                r = wrap_int_tensor(torch.bitwise_left_shift(x, s), "int")
            elif kind == "right":
                r = torch.bitwise_right_shift(x, s)
            else:
                r = wrap_int_tensor(torch.bitwise_right_shift(x & 0xFFFFFFFF, s), "int")
            return PrimColumn("int", r, _and(a.valid, k.valid))
        s = (k.data.to(torch.int64) & 63)
        if kind == "left":
            r = torch.bitwise_left_shift(x, s)
        elif kind == "right":
            r = torch.bitwise_right_shift(x, s)
        else:                                   # unsigned: logical shift of the 64-bit pattern
            r = torch.where(s == 0, x, torch.bitwise_right_shift(x, s) & ((1 << (64 - s)) - 1))
        return PrimColumn("long", r, _and(a.valid, k.valid))
    return f


def _f_bit_count(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    (a,) = _args(e, scope, ctx, subst)
    a = materialize(_num(a, n, dev))
    x = a.data.to(torch.int64)
    c = torch.zeros_like(x)
    for b in range(64):
        c += (torch.bitwise_right_shift(x, b) & 1)
    return PrimColumn("int", c.to(torch.int32), a.valid)


def _f_rint(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    (a,) = _args(e, scope, ctx, subst)
    a = materialize(_num(a, n, dev))
    return PrimColumn("double", torch.round(a.data.to(torch.float64)), a.valid)    # round half to even


def _f_width_bucket(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    v, lo, hi, k = (materialize(_num(c, n, dev)) for c in _args(e, scope, ctx, subst))
    x, a, b = (c.data.to(torch.float64) for c in (v, lo, hi))
    nb = k.data.to(torch.int64)
    asc = a < b
    frac = torch.where(asc, (x - a) / (b - a), (a - x) / (a - b))
    inner = torch.floor(frac * nb.to(torch.float64)).to(torch.int64) + 1
    r = torch.where(frac < 0, torch.zeros_like(inner), torch.where(frac >= 1, nb + 1, inner))
    ok = _and(_and(v.valid, lo.valid), _and(hi.valid, k.valid))
    good = (nb > 0) & (a != b) & torch.isfinite(x)
    ok = good if ok is None else ok & good
    return PrimColumn("long", r, ok)


_DOW = {"mo": 0, "mon": 0, "monday": 0, "tu": 1, "tue": 1, "tuesday": 1, "we": 2, "wed": 2, "wednesday": 2,
        "th": 3, "thu": 3, "thursday": 3, "fr": 4, "fri": 4, "friday": 4, "sa": 5, "sat": 5, "saturday": 5,
        "su": 6, "sun": 6, "sunday": 6}


def _f_next_day(e, scope, ctx, subst):
    """next_day(date, 'Mon'): the first date later than ``date`` falling on that weekday (null for a bad name)."""
    n, dev = scope.length, scope.device
    a, w = _args(e, scope, ctx, subst)
    if not isinstance(w, ConstColumn):
        raise EvalError("next_day() day-of-week must be a constant")
    tgt = _DOW.get(str(w.value or "").strip().lower())
    d = materialize(_days(a))
    if tgt is None:
        return ConstColumn(None, "date", n, dev)
    cur = torch.remainder(d.data.to(torch.int64) + 3, 7)          # 1970-01-01 was a Thursday (Mon = 0)
    step = torch.remainder(tgt - cur + 6, 7) + 1
    return PrimColumn("date", d.data.to(torch.int64) + step, d.valid)


def _f_typeof(e, scope, ctx, subst):
    (a,) = _args(e, scope, ctx, subst)
    t = dict(SIMPLE_NAME, double="double", string="string", boolean="boolean", timestamp="timestamp",
             date="date").get(str(a.dtype), str(a.dtype))
    return ConstColumn(t, "string", scope.length, scope.device)


def _f_partition_id(e, scope, ctx, subst):
    from .. import parallel as P
    return ConstColumn(P.rank() if P.active() else 0, "int", scope.length, scope.device)


def _f_timestamp_seconds(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    (a,) = _args(e, scope, ctx, subst)
    a = materialize(_num(a, n, dev))
    x = a.data
    us = torch.round(x.to(torch.float64) * 1e6).to(torch.int64) if x.is_floating_point() else x.to(torch.int64) * \
        1_000_000
    return PrimColumn("timestamp", us, a.valid)


def _format_number(x, d):
    """java.text.DecimalFormat("#,##0.00…", HALF_EVEN) over the value's shortest digits (Spark FormatNumber)."""
    if isinstance(d, str):
        raise ValueError("format patterns are not supported")
    d = int(d)
    if d < 0:
        return None
    from decimal import ROUND_HALF_EVEN, Decimal
    if isinstance(x, float) and (x != x or x in (float("inf"), float("-inf"))):
        return "\ufffd" if x != x else ("-\u221e" if x < 0 else "\u221e")      # Java 8 DecimalFormatSymbols
    v = Decimal(x) if isinstance(x, int) and not isinstance(x, bool) else Decimal(repr(float(x)))
    q = v.quantize(Decimal(1).scaleb(-d), rounding=ROUND_HALF_EVEN)
    return f"{q:,.{d}f}"


_DIGITS = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ"


def _conv(s, fb, tb):
    """conv(num, from_base, to_base): Spark 2.4 NumberConverter.convert — the space-trimmed digits up to the first
    invalid one as an unsigned 64-bit value (saturating at 2^64 - 1), negated for a leading '-' unless to_base < 0,
    which prints a signed value instead."""
    fb, tb = int(fb), int(tb)
    if not (2 <= fb <= 36 and 2 <= abs(tb) <= 36):
        return None
    t = str(s).strip(" ")
    if not t:
        return None
    neg = t.startswith("-")
    t = t[1:] if neg else t
    if len(t.encode("utf-8")) > 64:
        return None
    M = (1 << 64) - 1
    v = 0
    for ch in t:
        k = _DIGITS.find(ch.upper()) if ch.isascii() else -1
        if k < 0 or k >= fb:
            break
        v = v * fb + k
        if v > M:
            v = M
            break
    if neg and tb > 0:
        v = M if v >= 1 << 63 else (-v) & M
    if tb < 0 and v >= 1 << 63:
        v = (-v) & M
        neg = True
    b = abs(tb)
    digits = ""
    while True:
        digits = _DIGITS[v % b] + digits
        v //= b
        if not v:
            break
    return ("-" if neg and tb < 0 else "") + digits


def _soundex(s):
    s = str(s)
    if not s or not ("a" <= s[0] <= "z" or "A" <= s[0] <= "Z"):      # UTF8String.soundex: ASCII letters only
        return s
    codes = {**dict.fromkeys("BFPV", "1"), **dict.fromkeys("CGJKQSXZ", "2"), **dict.fromkeys("DT", "3"), "L": "4",
             **dict.fromkeys("MN", "5"), "R": "6"}
    up = "".join(c.upper() if c.isascii() else "\0" for c in s)
    out, last = up[0], codes.get(up[0], "")
    for ch in up[1:]:
        c = codes.get(ch, "")
        if c and c != last:
            out += c
            if len(out) == 4:
                break
        if ch not in "HW":
            last = c
    return out.ljust(4, "0")


def _levenshtein(a, b):
    a, b = str(a), str(b)
    prev = list(range(len(b) + 1))
    for i, ca in enumerate(a, 1):
        cur = [i]
        for j, cb in enumerate(b, 1):
            cur.append(min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ca != cb)))
        prev = cur
    return prev[-1]


def _substring_index(s, delim, count):
    s, delim, count = str(s), str(delim), int(count)
    if not delim or count == 0:
        return ""
    parts = s.split(delim)
    return delim.join(parts[:count]) if count > 0 else delim.join(parts[count:])


def _java_printf(fmt, *args):
    """format_string / printf: Java Formatter specs mapped onto Python's % formatting (%s %d %f %e %x %o %c %b %%,
    flags and widths)."""
    import re as _re
    out, it = [], iter(args)

    def conv(m):
        spec, flags, width, prec, c = m.group(0), m.group(1) or "", m.group(2) or "", m.group(3) or "", m.group(4)
        if c == "%":
            return "%"
        if c == "n":
            return "\n"
        v = next(it, None)
        if c in "bB":
            return str(v is not None and v is not False).lower()
        if v is None:
            return "null"
        pf = flags.replace(",", "")
        body = f"%{pf}{width}{prec}{'s' if c in 'sS' else c.lower() if c in 'xXeEgG' else c}"
        r = body % (int(v) if c in "dxXoc" else float(v) if c in "feEgG" else v)
        if "," in flags and c in "df":
            r = f"{(int(v) if c == 'd' else float(v)):,{prec}{'d' if c == 'd' else 'f'}}".rjust(int(width or 0))
        return r.upper() if c in "SXEG" else r
    return _re.sub(r"%([-#+ 0,(]*)(\d+)?(\.\d+)?([a-zA-Z%])", conv, str(fmt))


def _unhex(s):
    """Spark Hex.unhex: an odd length pads a leading '0'; any non-hex character → NULL (BINARY shown as text)."""
    t = str(s)
    if len(t) % 2:
        t = "0" + t
    try:
        if not all(c in "0123456789abcdefABCDEF" for c in t):
            return None
        return bytes.fromhex(t).decode("utf-8", errors="replace")
    except ValueError:
        return None


_B64 = {c: i for i, c in enumerate("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/")}
_B64.update({"-": 62, "_": 63})


def _unbase64(s):
    """commons-codec Base64.decodeBase64 (Spark UnBase64): lenient — characters outside the (standard or URL-safe)
    alphabet are skipped, '=' ends the data, a trailing 2- / 3-symbol group gives 1 / 2 bytes."""
    acc, m, out = 0, 0, bytearray()
    for c in str(s):
        if c == "=":
            break
        v = _B64.get(c)
        if v is None:
            continue
        acc = (acc << 6) | v
        m += 1
        if m == 4:
            out += bytes(((acc >> 16) & 255, (acc >> 8) & 255, acc & 255))
            acc, m = 0, 0
    if m >= 2:
        out.append((acc >> (4 if m == 2 else 10)) & 255)
        if m == 3:
            out.append((acc >> 2) & 255)
    return bytes(out).decode("utf-8", errors="replace")


def _split_part(s, d, k):
    """split_part(str, delim, n): the n-th field (from the end when n < 0); out of range → ''; an empty delimiter
    makes the whole string the only field; n = 0 is an error."""
    s, d, k = str(s), str(d), int(k)
    if k == 0:
        raise EvalError("split_part: the field index must not be 0")
    parts = s.split(d) if d else [s]
    if abs(k) > len(parts):
        return ""
    return parts[k - 1] if k > 0 else parts[k]


def _overlay(s, rep, pos, ln=None):
    """overlay(input, replace, pos[, len]): Spark's Overlay — input[:pos-1] + replace + input[pos-1+len:], len
    defaulting to the replacement's length."""
    s, rep, pos = str(s), str(rep), int(pos)
    ln = len(rep) if ln is None or int(ln) < 0 else int(ln)
    start = max(pos - 1, 0)
    return s[:start] + rep + s[start + ln:]


def _arrays_overlap(l, m):
    if m is None:
        return None
    a = {x for x in l if x is not None}
    if any(x in a for x in m if x is not None):
        return True
    return None if (l and m and (None in l or None in m)) else False


def _dedup(xs):
    out, seen, null = [], set(), False
    for x in xs:
        if x is None:
            if not null:
                out.append(None)
                null = True
        elif x not in seen:
            seen.add(x)
            out.append(x)
    return out


def _f_flatten(e, scope, ctx, subst):
    (arr,) = _args(e, scope, ctx, subst)
    if not isinstance(arr, ArrayColumn) or not arr.elements or not isinstance(arr.elements[0], ArrayColumn):
        raise EvalError("flatten() expects an array of arrays")
    inner = arr.elements[0]
    et = str(inner.elements[0].dtype) if inner.elements else "string"
    out = [None if l is None or any(x is None for x in l) else [y for x in l for y in x] for l in arr.to_pylist()]
    return array_from_pylist(out, et, scope.device)


def _json_ddl(v) -> str:
    """Spark's JsonInferSchema type of one JSON value, as schema_of_json prints it (fields sorted by name)."""
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, int):
        return "bigint"
    if isinstance(v, float):
        return "double"
    if isinstance(v, dict):
        return "struct<" + ",".join(f"{k}:{_json_ddl(x)}" for k, x in sorted(v.items())) + ">"
    if isinstance(v, list):
        kinds = {_json_ddl(x) for x in v if x is not None}
        if not kinds:
            return "array<string>"
        if kinds <= {"bigint", "double"}:
            return "array<double>" if "double" in kinds else "array<bigint>"
        return f"array<{kinds.pop()}>" if len(kinds) == 1 else "array<string>"
    return "string"


def _f_zip_with(e, scope, ctx, subst):
    """zip_with(a, b, (x, y) -> f): element-wise over the longer array's length, the shorter side padded with nulls
    (Spark's ZipWith).  Fixed-length arrays only: a slot-compacted (variable-length) array cannot hold the null
    elements the padding produces."""
    from .expr import _lambda_arg
    a = evaluate(e.args[0], scope, ctx, subst)
    b = evaluate(e.args[1], scope, ctx, subst)
    if not (isinstance(a, ArrayColumn) and isinstance(b, ArrayColumn)):
        raise EvalError("zip_with() expects two arrays")
    if a.drop_nulls or b.drop_nulls:
        raise EvalError("zip_with() over variable-length arrays is not supported")
    lam = _lambda_arg(e, 2)
    if len(lam.params) != 2:
        raise EvalError("zip_with() takes a two-argument lambda")
    n, dev = scope.length, scope.device

    def slot(arr, j):
        if j < len(arr.elements):
            return arr.elements[j]
        t = str(arr.elements[0].dtype) if arr.elements else "string"
        return ConstColumn(None, t, n, dev)
    out = [evaluate(lam.body, scope.with_bindings(list(lam.params), [slot(a, j), slot(b, j)]), ctx, subst)
           for j in range(max(len(a.elements), len(b.elements)))]
    valid = a.valid if b.valid is None else (b.valid if a.valid is None else a.valid & b.valid)
    return ArrayColumn(out, n, valid, False, dev)


def _f_map_from_arrays(e, scope, ctx, subst):
    """map_from_arrays(keys, values) with a constant key array (this engine's maps have constant keys): the map
    whose key i holds element i of ``values``."""
    from .expr import _const_str
    ks = evaluate(e.args[0], scope, ctx, subst)
    vs = evaluate(e.args[1], scope, ctx, subst)
    if not (isinstance(ks, ArrayColumn) and all(isinstance(k, ConstColumn) for k in ks.elements)):
        raise EvalError("map_from_arrays() needs a constant key array")
    if not isinstance(vs, ArrayColumn) or len(vs.elements) != len(ks.elements) or vs.drop_nulls:
        raise EvalError("map_from_arrays() needs a fixed-length value array of the keys' length")
    names = [_const_str(k) for k in ks.elements]
    if len(set(names)) != len(names):
        raise EvalError("map_from_arrays(): duplicate map keys")
    return StructColumn(names, list(vs.elements), scope.length, vs.valid, True, None, scope.device)


def _register_more():
    reg = register_function
    reg("shiftleft", _f_shift("left"))
    reg("shiftright", _f_shift("right"))
    reg("shiftrightunsigned", _f_shift("unsigned"))
    reg("bit_count", _f_bit_count)
    reg("rint", _f_rint)
    reg("width_bucket", _f_width_bucket)
    reg("next_day", _f_next_day)
    reg("typeof", _f_typeof)
    reg("spark_partition_id", _f_partition_id)
    reg("timestamp_seconds", _f_timestamp_seconds)
    reg("input_file_name", lambda e, scope, ctx, subst: ConstColumn("", "string", scope.length, scope.device))
    reg("format_number", _host_string_fn(_format_number))
    reg("conv", _host_string_fn(_conv))
    reg("soundex", _host_string_fn(_soundex))
    reg("levenshtein", _host_string_fn(_levenshtein, "int"))
    reg("substring_index", _host_string_fn(_substring_index))
    reg("char", _host_string_fn(lambda x: chr(int(x) % 256) if int(x) >= 0 else ""))
    reg("chr", _host_string_fn(lambda x: chr(int(x) % 256) if int(x) >= 0 else ""))
    reg("octet_length", _host_string_fn(lambda s: len(str(s).encode("utf-8")), "int"))
    reg("bit_length", _host_string_fn(lambda s: 8 * len(str(s).encode("utf-8")), "int"))
    reg("overlay", _host_string_fn(_overlay))
    reg("arrays_overlap", _host_array_fn(_arrays_overlap, scalar_type="boolean"))
    reg("array_union", _host_array_fn(lambda l, m: None if m is None else _dedup(list(l) + list(m))))
    reg("array_intersect", _host_array_fn(lambda l, m: None if m is None else _dedup([x for x in l if x in m])))
    reg("array_except", _host_array_fn(lambda l, m: None if m is None else _dedup([x for x in l if x not in m])))
    reg("flatten", _f_flatten)
    reg("zip_with", _f_zip_with)
    reg("map_from_arrays", _f_map_from_arrays)
    reg("schema_of_json", _host_string_fn(lambda t: _json_ddl(json.loads(str(t)))))
    reg("format_string", _host_string_fn(_java_printf))
    reg("printf", _host_string_fn(_java_printf))


_register_more()


# ---------------------------------------------------------------------------------------------------------------
# device paths of the string built-ins (dxa/ops/strfuncs.py, csrc/strfuncs.hip)
# ---------------------------------------------------------------------------------------------------------------

def _const_arg(args, i, default=None):
    if i >= len(args):
        return True, default
    a = args[i]
    return (isinstance(a, ConstColumn), a.value if isinstance(a, ConstColumn) else None)


def _dev_str(c):
    """``c`` as a device StrColumn with contiguous int64 starts / int32 lens (or None if it is not one)."""
    if not _gpu_str(c):
        return None
    st = c.starts if (c.starts.dtype == torch.int64 and c.starts.is_contiguous()) else \
        c.starts.to(torch.int64).contiguous()
    ln = c.lens if (c.lens.dtype == torch.int32 and c.lens.is_contiguous()) else c.lens.to(torch.int32).contiguous()
    if st is c.starts and ln is c.lens:
        return c
    return type(c)(c.arena, st, ln, c.valid, c.dtype)


def _device_string_fn(name, device_fn, host_fn, out_type="string"):
    """``device_fn(col, *const_args)`` on a device string column with constant (non-null) extra arguments; a None
    result (rows the kernel does not handle) or any other argument shape → the host function."""
    host = _host_string_fn(host_fn, out_type)

    def f(e, scope, ctx, subst):
        args = _args(e, scope, ctx, subst)
        a = _dev_str(args[0]) if args else None
        if a is not None and all(isinstance(x, ConstColumn) and x.value is not None for x in args[1:]):
            out = device_fn(a, *[x.value for x in args[1:]])
            if out is not None:
                return out
        return host(e, scope, ctx, subst)
    f.__name__ = f"_f_{name}"
    return f


def _lpad_host(s, l, p=" "):
    s, l, p = str(s), int(l), str(p)
    if l <= 0:
        return ""
    if len(s) >= l or not p:
        return s[:l]
    fill = l - len(s)
    return (p * (fill // len(p) + 1))[:fill] + s


def _rpad_host(s, l, p=" "):
    s, l, p = str(s), int(l), str(p)
    if l <= 0:
        return ""
    if len(s) >= l or not p:
        return s[:l]
    fill = l - len(s)
    return s + (p * (fill // len(p) + 1))[:fill]


def _ascii_host(s):
    b = str(s).encode("utf-8")
    return (b[0] - 256 if b[0] >= 128 else b[0]) if b else 0


def _levenshtein_fn(e, scope, ctx, subst):
    args = _args(e, scope, ctx, subst)
    if len(args) == 2 and any(_gpu_str(x) for x in args):
        cols = [materialize(x) if isinstance(x, ConstColumn) and x.value is not None else x for x in args]
        a, b = (_dev_str(c) for c in cols)
        if a is not None and b is not None and a.length == b.length:
            from ..ops import strfuncs as SF
            out = SF.levenshtein(a, b)
            if out is not None:
                return out
    return _host_string_fn(_levenshtein, "int")(e, scope, ctx, subst)


def _octets(mult):
    """octet_length / bit_length: byte counts of the UTF-8 text (the lengths column itself on the device)."""
    host = _host_string_fn(lambda s: mult * len(str(s).encode("utf-8")), "int")

    def f(e, scope, ctx, subst):
        args = _args(e, scope, ctx, subst)
        if len(args) == 1 and isinstance(args[0], StrColumn):
            return PrimColumn("int", args[0].lens.to(torch.int32) * mult, args[0].valid)
        return host(e, scope, ctx, subst)
    return f


_CHR_TABLE = None


def _f_chr(e, scope, ctx, subst):
    """chr(n) / char(n): the character n mod 256 (Latin-1 code point, UTF-8 encoded); '' for n < 0 — a view into
    a 256-entry table arena, no per-row host work."""
    global _CHR_TABLE
    (a,) = _args(e, scope, ctx, subst)
    if isinstance(a, ConstColumn) or not isinstance(a, PrimColumn):
        return _host_string_fn(lambda x: chr(int(x) % 256) if int(x) >= 0 else "")(e, scope, ctx, subst)
    dev = a.device
    if _CHR_TABLE is None or _CHR_TABLE[0].device != dev:
        enc = [chr(c).encode("utf-8") for c in range(256)]
        starts, pos = [], 0
        for b in enc:
            starts.append(pos)
            pos += len(b)
        from ..ops.native import h2d
        _CHR_TABLE = (h2d(b"".join(enc) + b"\0" * 16, torch.uint8, dev), h2d(starts, torch.int64, dev),
                      h2d([len(b) for b in enc], torch.int32, dev))
    arena, st, ln = _CHR_TABLE
    x = a.data.to(torch.int64)
    code = torch.remainder(x, 256)
    neg = x < 0
    return StrColumn(arena, st[code], torch.where(neg, torch.zeros_like(ln[code]), ln[code]), a.valid)


def _register_device_strings():
    from ..ops import strfuncs as SF
    reg = register_function
    reg("octet_length", _octets(1))
    reg("bit_length", _octets(8))
    reg("chr", _f_chr)
    reg("char", _f_chr)
    reg("lpad", _device_string_fn("lpad", lambda c, l, p=" ": SF.pad(c, int(l), str(p), True), _lpad_host))
    reg("rpad", _device_string_fn("rpad", lambda c, l, p=" ": SF.pad(c, int(l), str(p), False), _rpad_host))
    reg("reverse", _device_string_fn("reverse", SF.reverse, lambda s: str(s)[::-1]))
    reg("repeat", _device_string_fn("repeat", lambda c, k: SF.repeat(c, int(k)),
                                    lambda s, k: str(s) * max(0, int(k))))
    reg("translate", _device_string_fn("translate", lambda c, m, r: SF.translate(c, str(m), str(r)), _translate))
    reg("initcap", _device_string_fn("initcap", SF.initcap, _initcap))
    reg("ascii", _device_string_fn("ascii", SF.ascii_code, _ascii_host, "int"))
    reg("substring_index", _device_string_fn("substring_index",
                                             lambda c, d, k: SF.substring_index(c, str(d), int(k)),
                                             _substring_index))
    reg("levenshtein", _levenshtein_fn)
    reg("format_number", _f_format_number)
    reg("conv", _device_string_fn("conv", _conv_device, _conv))
    reg("bin", _f_bin)
    reg("soundex", _device_string_fn("soundex", SF.soundex, _soundex))
    reg("unhex", _device_string_fn("unhex", lambda c: SF.decode(c, 0), _unhex))
    reg("unbase64", _device_string_fn("unbase64", lambda c: SF.decode(c, 1), _unbase64))
    reg("split_part", _device_string_fn("split_part", lambda c, d, k: SF.split_part(c, str(d), int(k))
                                        if int(k) != 0 else None, _split_part))
    reg("factorial", _f_factorial)
    reg("overlay", _f_overlay)


def _conv_device(col, fb, tb):
    from ..ops import strfuncs as SF
    fb, tb = int(fb), int(tb)
    if not (2 <= fb <= 36 and 2 <= abs(tb) <= 36):
        return None                                  # the host path yields the NULLs
    return SF.conv(col, fb, tb)


def _f_format_number(e, scope, ctx, subst):
    args = _args(e, scope, ctx, subst)
    x = args[0] if args else None
    if (len(args) == 2 and isinstance(x, PrimColumn) and x.data.is_cuda and x.dtype in INTEGRAL + ("double", "float")
            and isinstance(args[1], ConstColumn) and isinstance(args[1].value, int)):
        from ..ops import strfuncs as SF
        out = SF.format_number(x, int(args[1].value))
        if out is not None:
            return out
    return _host_string_fn(_format_number)(e, scope, ctx, subst)


def _f_bin(e, scope, ctx, subst):
    (x,) = _args(e, scope, ctx, subst)
    if isinstance(x, PrimColumn) and x.data.is_cuda and x.dtype in INTEGRAL + ("double", "float"):
        from ..ops import strfuncs as SF
        if x.data.dtype == torch.float64:             # Spark casts to bigint (truncation)
            x = cast_column(x, "long")
        return SF.bin_text(x)
    return _host_string_fn(lambda v: format(int(v) & 0xFFFFFFFFFFFFFFFF, "b"))(e, scope, ctx, subst)


_FACT = [math.factorial(i) for i in range(21)]


def _f_factorial(e, scope, ctx, subst):
    (x,) = _args(e, scope, ctx, subst)
    n, dev = scope.length, scope.device
    if isinstance(x, ConstColumn):
        v = None if x.value is None else int(x.value)
        return ConstColumn(_FACT[v] if v is not None and 0 <= v <= 20 else None, "long", n, dev)
    k = x.data.to(torch.int64) if x.data.dtype != torch.float64 else x.data.trunc().to(torch.int64)
    ok = (k >= 0) & (k <= 20)
    table = _h2d(_FACT, torch.int64, dev)
    out = table[torch.where(ok, k, torch.zeros_like(k))]
    return PrimColumn("long", out, ok if x.valid is None else ok & x.valid)


def _f_overlay(e, scope, ctx, subst):
    """overlay(input, replace, pos[, len]) = substring(input, 1, pos - 1) || replace || substring(input, pos + len)
    (Spark's Overlay over substringSQL; len < 0 or absent → the replacement's length) — evaluated through the
    device substring / concat paths."""
    if len(e.args) not in (3, 4):
        raise EvalError("overlay expects 3 or 4 arguments")
    s, r, pos = e.args[:3]
    rlen = A.Call("char_length", [r])
    if len(e.args) == 4:
        ln = e.args[3]
        ln = A.Call("if", [A.BinOp(">=", ln, A.Literal(0, "int")), ln, rlen])
    else:
        ln = rlen
    head = A.Call("substring", [s, A.Literal(1, "int"), A.BinOp("-", pos, A.Literal(1, "int"))])
    tail = A.Call("substring", [s, A.BinOp("+", pos, ln)])
    return evaluate(A.Call("concat", [head, r, tail]), scope, ctx, subst)


_register_device_strings()


def _h2d(data, dtype, device):
    from ..ops.native import h2d
    return h2d(data, dtype, device)


# array built-ins as slot-matrix tensor operations (dxa/engine/arrayfuncs.py registers itself on import, with the
# row-wise functions above as its fallback)
from . import arrayfuncs  # noqa: E402,F401


# ---------------------------------------------------------------------------------------------------------------
# Spark 2.4 built-ins: str_to_map, map_concat, array_repeat, encode / decode, sentences, xpath_*, assert_true
# ---------------------------------------------------------------------------------------------------------------

def _const_str(c):
    from .expr import _const_str as cs
    return cs(c)


def _raw_rows(col) -> list:
    """Row bytes of a string / binary column (None for null), without a UTF-8 decode."""
    col = materialize(col)
    if isinstance(col, ConstColumn):
        v = col.value
        return [None if v is None else (v if isinstance(v, bytes) else str(v).encode("utf-8"))] * col.length
    if not isinstance(col, StrColumn):
        return [None if v is None else str(v).encode("utf-8") for v in col.to_pylist()]
    arena = col.arena.cpu().numpy().tobytes()
    st, ln = col.starts.cpu().tolist(), col.lens.cpu().tolist()
    ok = col.valid.cpu().tolist() if col.valid is not None else [True] * col.length
    return [arena[s:s + l] if o else None for s, l, o in zip(st, ln, ok)]


def _binary_column(values, device):
    sc = strings_from_pylist(values, device)
    return StrColumn(sc.arena, sc.starts, sc.lens, sc.valid, "binary")


# java.nio charset names Spark's Encode / Decode accept (StringUtils: US-ASCII, ISO-8859-1, UTF-8, UTF-16BE,
# UTF-16LE, UTF-16); Java's UTF-16 encoder writes a big-endian byte-order mark
_CHARSETS = {"us-ascii": "ascii", "iso-8859-1": "latin-1", "utf-8": "utf-8", "utf-16be": "utf-16-be",
             "utf-16le": "utf-16-le", "utf-16": "utf-16"}


def _charset(name) -> str:
    cs = _CHARSETS.get(str(name).strip().lower())
    if cs is None:
        raise EvalError(f"unsupported charset {name!r} (US-ASCII, ISO-8859-1, UTF-8, UTF-16BE, UTF-16LE, UTF-16)")
    return cs


def _f_encode(e, scope, ctx, subst):
    s, cs = _args(e, scope, ctx, subst)
    py = _charset(_const_str(cs))
    out = []
    for v in (s.to_pylist() if not isinstance(s, ConstColumn) else [s.value] * scope.length):
        if v is None:
            out.append(None)
        elif py == "utf-16":
            out.append(b"\xfe\xff" + str(v).encode("utf-16-be"))
        else:
            out.append(str(v).encode(py, errors="replace"))
    return _binary_column(out, scope.device)


def _f_decode(e, scope, ctx, subst):
    b, cs = _args(e, scope, ctx, subst)
    py = _charset(_const_str(cs))
    out = []
    for v in _raw_rows(b):
        if v is None:
            out.append(None)
        elif py == "utf-16":
            if v[:2] == b"\xff\xfe":
                out.append(v[2:].decode("utf-16-le", errors="replace"))
            else:
                out.append((v[2:] if v[:2] == b"\xfe\xff" else v).decode("utf-16-be", errors="replace"))
        else:
            out.append(v.decode(py, errors="replace"))
    return column_from_pylist(out, "string", scope.device)


def _f_str_to_map(e, scope, ctx, subst):
    """str_to_map(text[, pairDelim = ',', keyValueDelim = ':']): delimiters are regexes (StringToMap splits
    with String.split); a pair without the key/value delimiter maps to NULL.  This engine's maps have the batch's
    keys as fields (in first-appearance order); a key a row lacks is absent there."""
    n, dev = scope.length, scope.device
    args = _args(e, scope, ctx, subst)
    pd = _const_str(args[1]) if len(args) > 1 else ","
    kd = _const_str(args[2]) if len(args) > 2 else ":"
    texts = args[0].to_pylist() if not isinstance(args[0], ConstColumn) else [args[0].value] * n
    rows, keys = [], {}
    for t in texts:
        if t is None:
            rows.append(None)
            continue
        m = {}
        for pair in re.split(pd, str(t)):
            kv = re.split(kd, pair, maxsplit=1)
            k = kv[0]
            if k not in m:
                m[k] = kv[1] if len(kv) > 1 else None
            keys.setdefault(k, None)
        rows.append(m)
    names = list(keys)
    cols = [column_from_pylist([None if r is None else r.get(k) for r in rows], "string", dev) for k in names]
    valid = None if all(r is not None for r in rows) else torch.tensor([r is not None for r in rows],
                                                                      dtype=torch.bool, device=dev)
    return StructColumn(names, cols, n, valid, True, None, dev)


def _f_map_concat(e, scope, ctx, subst):
    """map_concat(m1, m2, …): the union of the maps' keys; a key in several maps takes the later map's value
    where that map has it.  NULL when any argument is NULL (Spark 2.4 MapConcat)."""
    n, dev = scope.length, scope.device
    ms = [materialize(m) for m in _args(e, scope, ctx, subst)]
    for m in ms:
        if not (isinstance(m, StructColumn) and m.is_map):
            raise EvalError("map_concat() expects maps")
    names, cols = [], {}
    for m in ms:
        for k, c in zip(m.names, m.children):
            c = materialize(c)
            if k not in cols:
                names.append(k)
                cols[k] = c
            else:
                from .expr import _select_by_conditions
                cols[k] = _select_by_conditions([PrimColumn("boolean", c.valid_mask())], [c], cols[k], n, dev)
    valid = None
    for m in ms:
        if m.valid is not None:
            valid = m.valid if valid is None else valid & m.valid
    return StructColumn(names, [cols[k] for k in names], n, valid, True, None, dev)


def _f_array_repeat(e, scope, ctx, subst):
    """array_repeat(element, count): ``count`` copies (a NULL count → NULL, a negative one → empty)."""
    n, dev = scope.length, scope.device
    x, c = _args(e, scope, ctx, subst)
    if isinstance(c, ConstColumn):
        if c.value is None:
            return ConstColumn(None, "null", n, dev)
        k = max(0, int(c.value))
        return ArrayColumn([x] * k, n, None, False, dev) if k else \
            ArrayColumn([], n, None, False, dev, present=torch.zeros((n, 0), dtype=torch.bool, device=dev))
    cnt = materialize(c)
    cd = cnt.data.to(torch.int64).clamp(min=0)
    k = int(cd.max()) if n else 0                                 # slot count: one host read
    j = torch.arange(max(k, 0), device=dev)
    present = j.unsqueeze(0) < cd.unsqueeze(1)
    return ArrayColumn([x] * k, n, cnt.valid, False, dev, present=present)


_SENT_END = re.compile(r"(?<=[.!?])\s+")
_WORD = re.compile(r"[\w']+", re.UNICODE)


def _sentences(text):
    """Sentences → words, as Spark's Sentences does with java.text.BreakIterator (sentence then word instances,
    punctuation dropped)."""
    out = []
    for sent in _SENT_END.split(str(text).strip()):
        words = [w.strip("'") for w in _WORD.findall(sent)]
        words = [w for w in words if w]
        if words:
            out.append(words)
    return out


def _f_sentences(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    a = _args(e, scope, ctx, subst)[0]
    texts = a.to_pylist() if not isinstance(a, ConstColumn) else [a.value] * n
    rows = [None if t is None else _sentences(t) for t in texts]
    k = max((len(r) for r in rows if r is not None), default=0)
    outer = [array_from_pylist([r[j] if r is not None and j < len(r) else [] for r in rows], "string", dev)
             for j in range(k)]
    present = torch.tensor([[r is not None and j < len(r) for j in range(k)] for r in rows],
                           dtype=torch.bool, device=dev).reshape(n, k)
    valid = None if all(r is not None for r in rows) else torch.tensor([r is not None for r in rows],
                                                                      dtype=torch.bool, device=dev)
    return ArrayColumn(outer, n, valid, False, dev, present=present)


def _xpath_eval(xml, path):
    """The XPath subset Spark's xpath_* examples use: location paths from the document (``a/b``, ``/a/b``,
    ``//b``, ``a/b/@attr``, ``a/b/text()``) and ``sum(…)`` / ``count(…)`` over them → ('nodes', [text]) or
    ('number', v).  (Spark runs javax.xml.xpath; full XPath 1.0 is out of scope here.)"""
    import xml.etree.ElementTree as ET
    p = str(path).strip()
    m = re.match(r"^(sum|count)\((.*)\)$", p)
    if m:
        kind, vals = _xpath_eval(xml, m.group(2))
        if m.group(1) == "count":
            return "number", float(len(vals))
        tot = 0.0
        for v in vals:
            try:
                tot += float(v)
            except ValueError:
                return "number", float("nan")
        return "number", tot
    root = ET.fromstring(str(xml))
    attr = text = False
    if p.endswith("/text()"):
        p, text = p[:-7], True
    am = re.match(r"^(.*)/@([\w:-]+)$", p)
    if am:
        p, attr = am.group(1), am.group(2)
    if p.startswith("//"):
        nodes = ([root] if root.tag == p[2:].split("/")[0] and "/" not in p[2:] else []) + root.findall(".//" + p[2:])
    else:
        steps = [s for s in p.lstrip("/").split("/") if s]
        if not steps or steps[0] not in (root.tag, "*"):
            nodes = []
        elif len(steps) == 1:
            nodes = [root]
        else:
            nodes = root.findall("/".join(steps[1:]))
    if attr:
        return "nodes", [n.get(attr) for n in nodes if n.get(attr) is not None]
    if text:
        return "nodes", [n.text for n in nodes if n.text is not None]
    return "nodes", ["".join(n.itertext()) for n in nodes]


def _xpath_scalar(kind):
    def fn(xml, path):
        k, v = _xpath_eval(xml, path)
        if kind == "string":
            return (v[0] if v else "") if k == "nodes" else F.java_double_str(v)
        if kind == "boolean":
            return bool(v) if k == "nodes" else v != 0
        num = v if k == "number" else (float(v[0]) if v else float("nan"))
        if kind in INTEGRAL:
            return 0 if num != num else int(num)
        return num
    return fn


def _f_xpath(e, scope, ctx, subst):
    n, dev = scope.length, scope.device
    x, p = _args(e, scope, ctx, subst)
    xs = x.to_pylist() if not isinstance(x, ConstColumn) else [x.value] * n
    path = _const_str(p)
    rows = [None if v is None else _xpath_eval(v, path)[1] for v in xs]
    return array_from_pylist(rows, "string", dev)


def _f_assert_true(e, scope, ctx, subst):
    """assert_true(cond): NULL when every row's condition holds; otherwise the query fails (Spark's AssertTrue:
    "'<cond>' is not true!")."""
    from .expr import output_name
    (c,) = _args(e, scope, ctx, subst)
    c = materialize(c)
    ok = c.data.bool() & c.valid_mask() if not isinstance(c, ConstColumn) else None
    bad = (not c.value) if isinstance(c, ConstColumn) else bool((~ok).any())
    if bad:
        raise EvalError(f"'{output_name(e.args[0])}' is not true!")
    return ConstColumn(None, "null", scope.length, scope.device)


def _register_spark24_more():
    reg = register_function
    reg("encode", _f_encode)
    reg("decode", _f_decode)
    reg("str_to_map", _f_str_to_map)
    reg("map_concat", _f_map_concat)
    reg("array_repeat", _f_array_repeat)
    reg("sentences", _f_sentences)
    reg("xpath", _f_xpath)
    reg("xpath_string", _host_string_fn(_xpath_scalar("string")))
    reg("xpath_boolean", _host_string_fn(_xpath_scalar("boolean"), "boolean"))
    reg("xpath_int", _host_string_fn(_xpath_scalar("int"), "int"))
    reg("xpath_short", _host_string_fn(_xpath_scalar("short"), "int"))
    reg("xpath_long", _host_string_fn(_xpath_scalar("long"), "long"))
    reg("xpath_double", _host_string_fn(_xpath_scalar("double"), "double"))
    reg("xpath_number", _host_string_fn(_xpath_scalar("double"), "double"))
    reg("xpath_float", _host_string_fn(_xpath_scalar("double"), "double"))
    reg("assert_true", _f_assert_true)


_register_spark24_more()


# ---- round-6 Spark 2.4 built-ins: arrays_zip, shuffle, map_from_entries, space; reverse on arrays --------------

def _f_arrays_zip(e, scope, ctx, subst):
    """arrays_zip(a1, …, ak) → array<struct<n1, …, nk>>: the i-th struct holds every array's i-th element, NULL past a
    shorter array's end; NULL when any argument is NULL.  Field names: a column argument's name, else its position
    ("0", "1", …) — Spark 2.4 ArraysZip."""
    n, dev = scope.length, scope.device
    args = _args(e, scope, ctx, subst)
    if not args:
        return ConstColumn([], ArrayType(StructType(())), n, dev)
    for a in args:
        if not (isinstance(a, ArrayColumn) or (isinstance(a, ConstColumn) and a.value is None)):
            raise EvalError("arrays_zip() expects array arguments")
    names = [x.parts[-1] if isinstance(x, A.Ident) else str(i) for i, x in enumerate(e.args)]
    ftypes = [a.dtype.element if isinstance(a.dtype, ArrayType) else "null" for a in args]
    st = StructType(tuple(StructField(nm, t) for nm, t in zip(names, ftypes)))
    lists = [a.to_pylist() if not isinstance(a, ConstColumn) else [None] * n for a in args]
    out = []
    for i in range(n):
        row = [l[i] for l in lists]
        if any(r is None for r in row):
            out.append(None)
            continue
        k = max((len(r) for r in row), default=0)
        out.append([{nm: (r[j] if j < len(r) else None) for nm, r in zip(names, row)} for j in range(k)])
    return array_from_pylist(out, st, dev)


def _f_shuffle(e, scope, ctx, subst):
    """shuffle(array): a random permutation of each row's elements (non-deterministic, like Spark's Shuffle; the
    optional seed argument makes it repeatable here)."""
    import random as _rnd
    args = _args(e, scope, ctx, subst)
    arr = args[0]
    if isinstance(arr, ConstColumn) and arr.value is None:
        return arr
    if not isinstance(arr, ArrayColumn):
        raise EvalError("shuffle() expects an array")
    seed = args[1].value if len(args) > 1 and isinstance(args[1], ConstColumn) else None
    rng = _rnd.Random(seed)
    out = []
    for l in arr.to_pylist():
        if l is not None:
            l = list(l)
            rng.shuffle(l)
        out.append(l)
    return array_from_pylist(out, arr.dtype.element, scope.device)


def _f_map_from_entries(e, scope, ctx, subst):
    """map_from_entries(array<struct<k, v>>) → map<k, v>; a NULL entry makes the row NULL, a NULL key is an error
    (Spark 2.4 MapFromEntries); a repeated key keeps its last value."""
    (arr,) = _args(e, scope, ctx, subst)
    if isinstance(arr, ConstColumn) and arr.value is None:
        return arr
    if not isinstance(arr, ArrayColumn) or not isinstance(arr.dtype.element, StructType) or \
            len(arr.dtype.element.fields) != 2:
        raise EvalError("map_from_entries() expects an array of two-field structs")
    kf, vf = arr.dtype.element.fields
    out = []
    for l in arr.to_pylist():
        if l is None or any(x is None for x in l):
            out.append(None)
            continue
        m = {}
        for x in l:
            k = x[kf.name]
            if k is None:
                raise EvalError("map_from_entries(): cannot use null as map key")
            m[k] = x[vf.name]
        out.append(m)
    return column_from_pylist(out, MapType(kf.dtype, vf.dtype), scope.device)


def _f_space(e, scope, ctx, subst):
    """space(n): n spaces (none for n <= 0)."""
    n, dev = scope.length, scope.device
    (k,) = _args(e, scope, ctx, subst)
    if isinstance(k, ConstColumn):
        return ConstColumn(None if k.value is None else " " * max(0, int(k.value)), "string", n, dev)
    return strings_from_pylist([None if v is None else " " * max(0, int(v)) for v in k.to_pylist()], dev)


def _array_reverse(arr: ArrayColumn) -> ArrayColumn:
    """reverse(array): the slot order reversed — a row's array is its present slots left to right, so reversing the
    slots (and the presence mask's columns) reverses every row's array, on the device, without a host round trip."""
    pres = None if arr.present is None else torch.flip(arr.present, dims=[1])
    return ArrayColumn(list(reversed(arr.elements)), arr.length, arr.valid, arr.drop_nulls, arr.device, present=pres)


def _register_round6():
    reg = register_function
    reg("arrays_zip", _f_arrays_zip)
    reg("shuffle", _f_shuffle)
    reg("map_from_entries", _f_map_from_entries)
    reg("space", _f_space)
    reg("xpath_short", _host_string_fn(_xpath_scalar("short"), "short"))
    from .expr import _FUNCS
    string_reverse = _FUNCS["reverse"]

    def _f_reverse(e, scope, ctx, subst):
        args = _args(e, scope, ctx, subst)
        if args and isinstance(args[0], ArrayColumn):
            return _array_reverse(args[0])
        return string_reverse(e, scope, ctx, subst)
    reg("reverse", _f_reverse)


_register_round6()
