"""Value-level helpers shared by the expression evaluator: timestamp arithmetic on int64 µs tensors (runs as plain
device tensor math), Java-compatible number formatting (Spark's ``to_json``/``CAST AS STRING`` use
``Double.toString``), and casts.
"""
from __future__ import annotations

import datetime as _dt
import math
from typing import Optional

import torch

US_PER_SEC = 1_000_000
US_PER_MIN = 60 * US_PER_SEC
US_PER_HOUR = 60 * US_PER_MIN
US_PER_DAY = 24 * US_PER_HOUR


def floor_div(a: torch.Tensor, b: int) -> torch.Tensor:
    return torch.div(a, b, rounding_mode="floor")


def civil_from_days(z: torch.Tensor):
    """days since epoch → (year, month, day) tensors (Howard Hinnant's algorithm, vectorised)."""
    z = z + 719468
    era = floor_div(z, 146097)
    doe = z - era * 146097
    yoe = floor_div(doe - floor_div(doe, 1460) + floor_div(doe, 36524) - floor_div(doe, 146096), 365)
    y = yoe + era * 400
    doy = doe - (365 * yoe + floor_div(yoe, 4) - floor_div(yoe, 100))
    mp = floor_div(5 * doy + 2, 153)
    d = doy - floor_div(153 * mp + 2, 5) + 1
    m = torch.where(mp < 10, mp + 3, mp - 9)
    y = torch.where(m <= 2, y + 1, y)
    return y, m, d


def days_from_civil(y: torch.Tensor, m: torch.Tensor, d: torch.Tensor) -> torch.Tensor:
    y = torch.where(m <= 2, y - 1, y)
    era = floor_div(y, 400)
    yoe = y - era * 400
    mp = torch.where(m > 2, m - 3, m + 9)
    doy = floor_div(153 * mp + 2, 5) + d - 1
    doe = yoe * 365 + floor_div(yoe, 4) - floor_div(yoe, 100) + doy
    return era * 146097 + doe - 719468


def ts_part(us: torch.Tensor, part: str) -> torch.Tensor:
    part = part.lower()
    if part == "hour":
        return floor_div(us, US_PER_HOUR) % 24
    if part == "minute":
        return floor_div(us, US_PER_MIN) % 60
    if part == "second":
        return floor_div(us, US_PER_SEC) % 60
    days = floor_div(us, US_PER_DAY)
    if part in ("dayofweek",):   # Spark: 1 = Sunday
        return (days + 4) % 7 + 1
    if part == "weekday":        # 0 = Monday
        return (days + 3) % 7
    y, m, d = civil_from_days(days)
    if part == "year":
        return y
    if part == "month":
        return m
    if part in ("day", "dayofmonth"):
        return d
    if part == "quarter":
        return floor_div(m - 1, 3) + 1
    if part == "dayofyear":
        return days - days_from_civil(y, torch.ones_like(m), torch.ones_like(d)) + 1
    raise ValueError(f"unsupported date part {part}")


def ts_trunc(us: torch.Tensor, unit: str) -> torch.Tensor:
    unit = unit.lower().strip()
    unit = {"yyyy": "year", "yy": "year", "mon": "month", "mm": "month", "dd": "day", "hh": "hour"}.get(unit, unit)
    if unit in ("microsecond",):
        return us
    if unit == "millisecond":
        return floor_div(us, 1000) * 1000
    if unit == "second":
        return floor_div(us, US_PER_SEC) * US_PER_SEC
    if unit == "minute":
        return floor_div(us, US_PER_MIN) * US_PER_MIN
    if unit == "hour":
        return floor_div(us, US_PER_HOUR) * US_PER_HOUR
    days = floor_div(us, US_PER_DAY)
    if unit == "day":
        return days * US_PER_DAY
    if unit == "week":
        # Monday-based weeks
        return (days - (days + 3) % 7) * US_PER_DAY
    y, m, d = civil_from_days(days)
    one = torch.ones_like(d)
    if unit == "month":
        return days_from_civil(y, m, one) * US_PER_DAY
    if unit == "quarter":
        return days_from_civil(y, floor_div(m - 1, 3) * 3 + 1, one) * US_PER_DAY
    if unit == "year":
        return days_from_civil(y, one, one) * US_PER_DAY
    raise ValueError(f"unsupported truncation unit {unit}")


def java_double_str(d: float) -> str:
    """``java.lang.Double.toString`` (shortest round-trip digits, Java's layout rules)."""
    if d != d:
        return "NaN"
    if d == math.inf:
        return "Infinity"
    if d == -math.inf:
        return "-Infinity"
    if d == 0.0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    r = repr(float(d))
    neg = r.startswith("-")
    if neg:
        r = r[1:]
    # digits and decimal exponent from Python's shortest repr
    if "e" in r or "E" in r:
        mant, ex = r.lower().split("e")
        ex = int(ex)
    else:
        mant, ex = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    # position of the decimal point relative to the start of `digits`
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip("0"))
    point = len(ip) - lead_zeros + ex
    digits = digits.rstrip("0") or "0"
    a = abs(d)
    if 1e-3 <= a < 1e7:
        if point <= 0:
            s = "0." + "0" * (-point) + digits
        elif point >= len(digits):
            s = digits + "0" * (point - len(digits)) + ".0"
        else:
            s = digits[:point] + "." + digits[point:]
    else:
        e = point - 1
        frac = digits[1:] or "0"
        s = f"{digits[0]}.{frac}E{e}"
    return ("-" if neg else "") + s


def format_timestamp_us(us: int, iso: bool = True) -> str:
    """Spark ``to_json`` timestamp text (``yyyy-MM-dd'T'HH:mm:ss.SSSXXX`` in UTC) or CAST text
    (``yyyy-MM-dd HH:mm:ss[.fff]``)."""
    t = _dt.datetime(1970, 1, 1) + _dt.timedelta(microseconds=int(us))
    if iso:
        return t.strftime("%Y-%m-%dT%H:%M:%S.") + f"{t.microsecond // 1000:03d}Z"
    s = t.strftime("%Y-%m-%d %H:%M:%S")
    if t.microsecond:
        s += ("." + f"{t.microsecond:06d}").rstrip("0")
    return s


def parse_timestamp_literal(s: str) -> Optional[int]:
    from ..ops.jsonparse import _iso_to_us
    from ..ops.strings import py_string_to_timestamp_us
    v = _iso_to_us(s.strip())
    if v is None:
        v = py_string_to_timestamp_us(s.strip())
    return v
