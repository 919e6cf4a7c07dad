"""Exact Spark ``DecimalType(precision, scale)``.

Reference: the reference's input schemas are Spark ``DataType.fromJson`` documents (DataProcessing/datax-host/src/
main/scala/datax/input/SchemaFile.scala:25) and SimulatedData emits ``decimal`` fields (Services/DataX.SimulatedData/
DataX.SimulatedData.DataGenService/DataGen.cs:162,195); user SQL runs with Spark 2.4's decimal semantics.

Representation (device or CPU tensors, no host objects): the unscaled integer of every value —
  precision ≤ 18  → one int64 per row (``data`` shape [n]);
  precision ≤ 38  → a signed 128-bit integer as two int64 lanes, (lo, hi) in ``data`` shape [n, 2]
                    (lo holds the low 64 bits' bit pattern, hi the signed high word).
Arithmetic on the 128-bit form runs lane-wise in tensor ops (carry from an unsigned compare, 32-bit limbs for
multiplication / division by small constants), so the same code is the device path and the CPU evaluator.

Spark 2.4 rules implemented here (DecimalPrecision / Decimal.changePrecision):
  * CAST to decimal(p, s) rounds HALF_UP to scale s; a value needing more than p digits is NULL;
  * a + b, a − b → decimal(max(s1,s2) + max(p1−s1, p2−s2) + 1, max(s1,s2)); a × b → decimal(p1+p2+1, s1+s2);
    a / b → decimal(p1−s1+s2 + max(6, s1+p2+1), max(6, s1+p2+1)); all bounded to 38 digits (scale reduced to keep
    at least min(s, 6) fraction digits — ``bounded`` with allowPrecisionLoss);
  * SUM(decimal(p,s)) → decimal(min(38, p+10), s); AVG → decimal(min(38, p+4), min(38, s+4));
  * integers take part as decimal(10,0) (int) / decimal(20,0) (long); doubles win over decimals (→ double);
  * rendering (to_json, outputs): plain digits with exactly ``scale`` fraction digits.
"""
from __future__ import annotations

import decimal as _pd
from typing import Optional, Tuple

import torch

MAX_PRECISION = 38
MAX_NARROW = 18
SIGN = -0x8000000000000000          # int64 sign bit
MASK32 = 0xFFFFFFFF
_CTX = _pd.Context(prec=80, rounding=_pd.ROUND_HALF_UP)     # exact for every 38-digit operand and result


class DecimalType(str):
    """``decimal(p,s)`` as a type tag (a ``str`` so type plumbing that passes type names along keeps working)."""

    def __new__(cls, precision: int = 10, scale: int = 0):
        precision, scale = int(precision), int(scale)
        if not (1 <= precision <= MAX_PRECISION) or not (0 <= scale <= precision):
            raise ValueError(f"invalid decimal({precision},{scale})")
        o = str.__new__(cls, f"decimal({precision},{scale})")
        o.precision, o.scale = precision, scale
        return o

    def __reduce__(self):
        return (DecimalType, (self.precision, self.scale))

    @property
    def narrow(self) -> bool:
        return self.precision <= MAX_NARROW


def is_decimal(t) -> bool:
    return isinstance(t, DecimalType)


def parse_decimal_type(text: str) -> DecimalType:
    """'decimal' / 'decimal(10)' / 'decimal(10,2)' (Spark: bare DECIMAL is decimal(10,0))."""
    t = text.strip().lower().replace(" ", "")
    for pre in ("decimal", "numeric", "dec"):
        if t.startswith(pre):
            rest = t[len(pre):]
            break
    else:
        raise ValueError(text)
    if not rest:
        return DecimalType(10, 0)
    if not (rest.startswith("(") and rest.endswith(")")):
        raise ValueError(text)
    parts = rest[1:-1].split(",")
    return DecimalType(int(parts[0]), int(parts[1]) if len(parts) > 1 else 0)


def bounded(p: int, s: int) -> DecimalType:
    """Spark's DecimalType.adjustPrecisionScale (allowPrecisionLoss): over 38 digits, keep the integer digits and
    reduce the scale down to min(s, 6)."""
    if p <= MAX_PRECISION:
        return DecimalType(p, s)
    int_digits = p - s
    min_scale = min(s, 6)
    adj = max(MAX_PRECISION - int_digits, min_scale)
    return DecimalType(MAX_PRECISION, adj)


def of_integral(t: str) -> DecimalType:
    """Spark DecimalType.forType: tinyint → decimal(3,0), smallint → (5,0), int → (10,0), bigint → (20,0)."""
    return DecimalType({"byte": 3, "short": 5, "int": 10}.get(t, 20), 0)


def result_add(a: DecimalType, b: DecimalType) -> DecimalType:
    s = max(a.scale, b.scale)
    return bounded(max(a.precision - a.scale, b.precision - b.scale) + s + 1, s)


def result_mul(a: DecimalType, b: DecimalType) -> DecimalType:
    return bounded(a.precision + b.precision + 1, a.scale + b.scale)


def result_div(a: DecimalType, b: DecimalType) -> DecimalType:
    s = max(6, a.scale + b.precision + 1)
    return bounded(a.precision - a.scale + b.scale + s, s)


def result_sum(a: DecimalType) -> DecimalType:
    return DecimalType(min(MAX_PRECISION, a.precision + 10), a.scale)


def result_avg(a: DecimalType) -> DecimalType:
    return DecimalType(min(MAX_PRECISION, a.precision + 4), min(MAX_PRECISION, a.scale + 4))


# ---------------------------------------------------------------------------------------------------------------
# 128-bit lane arithmetic (hi signed, lo raw bits) on int64 tensors
# ---------------------------------------------------------------------------------------------------------------

def _ult(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """unsigned a < b on int64 bit patterns."""
    return (a ^ SIGN) < (b ^ SIGN)


def add128(ah, al, bh, bl):
    lo = al + bl
    carry = _ult(lo, al).to(torch.int64)
    return ah + bh + carry, lo


def neg128(h, l):
    lo = -l                                         # two's complement of the low word
    return (~h) + (l == 0).to(torch.int64), lo


def sub128(ah, al, bh, bl):
    nh, nl = neg128(bh, bl)
    return add128(ah, al, nh, nl)


def from_i64(x: torch.Tensor):
    return x >> 63, x


def is_neg(h):
    return h < 0


def abs128(h, l):
    n = is_neg(h)
    nh, nl = neg128(h, l)
    return torch.where(n, nh, h), torch.where(n, nl, l), n


def lt128(ah, al, bh, bl):
    return (ah < bh) | ((ah == bh) & _ult(al, bl))


def eq128(ah, al, bh, bl):
    return (ah == bh) & (al == bl)


def _limbs(h, l):
    """unsigned 128 → four 32-bit limbs (little end first) in int64 tensors."""
    return [l & MASK32, (l >> 32) & MASK32, h & MASK32, (h >> 32) & MASK32]


def _from_limbs(x0, x1, x2, x3):
    lo = (x0 & MASK32) | ((x1 & MASK32) << 32)
    hi = (x2 & MASK32) | ((x3 & MASK32) << 32)
    return hi, lo


def mul_small_u(h, l, c: int):
    """unsigned 128 × c (0 ≤ c < 2^30) → (hi, lo, overflowed beyond 128 bits)."""
    x = _limbs(h, l)
    out, carry = [], torch.zeros_like(l)
    for limb in x:
        t = limb * c + carry                      # < 2^62
        out.append(t & MASK32)
        carry = t >> 32
    hi, lo = _from_limbs(*out)
    return hi, lo, carry != 0


def divmod_small_u(h, l, d: int):
    """unsigned 128 // d, % d for 0 < d < 2^31."""
    x = _limbs(h, l)
    rem = torch.zeros_like(l)
    q = [None] * 4
    for i in (3, 2, 1, 0):
        cur = (rem << 32) | x[i]                   # rem < d < 2^31 → cur < 2^63
        q[i] = cur // d
        rem = cur - q[i] * d
    hi, lo = _from_limbs(*q)
    return hi, lo, rem


_POW10 = [10 ** k for k in range(MAX_PRECISION + 2)]


def mul_pow10(h, l, k: int):
    """signed 128 × 10^k → (hi, lo, overflow)."""
    if k <= 0:
        return h, l, torch.zeros_like(h, dtype=torch.bool)
    ah, al, neg = abs128(h, l)
    ovf = torch.zeros_like(neg)
    while k > 0:
        step = min(k, 9)
        ah, al, o = mul_small_u(ah, al, 10 ** step)
        ovf |= o | (ah < 0)                        # the magnitude must stay below 2^127
        k -= step
    nh, nl = neg128(ah, al)
    return torch.where(neg, nh, ah), torch.where(neg, nl, al), ovf


def div_pow10_round(h, l, k: int, half_even: bool):
    """signed 128 / 10^k rounded HALF_UP (``half_even`` False) or HALF_EVEN (ties to the even quotient), exact: the
    digits below the last dropped one only matter for the tie test, so their remainders are OR-ed."""
    if k <= 0:
        return h, l
    if not half_even:
        return div_pow10_half_up(h, l, k)
    ah, al, neg = abs128(h, l)
    sticky = torch.zeros_like(neg)
    remaining = k - 1
    while remaining > 0:
        step = min(remaining, 9)
        ah, al, r = divmod_small_u(ah, al, 10 ** step)
        sticky |= r != 0
        remaining -= step
    ah, al, last = divmod_small_u(ah, al, 10)
    up = (last > 5) | ((last == 5) & (sticky | ((al & 1) == 1)))
    ah, al = add128(ah, al, torch.zeros_like(ah), up.to(torch.int64))
    nh, nl = neg128(ah, al)
    return torch.where(neg, nh, ah), torch.where(neg, nl, al)


def round_column(col, digits: int, half_even: bool):
    """round / bround of decimal(p, s) to ``digits`` places: Spark 2.4's RoundBase keeps decimal(p, min(s, digits))
    (a larger digit count keeps the scale); the value is rounded HALF_UP / HALF_EVEN and is NULL when it no longer
    fits p digits (Decimal.toPrecision).  Negative digits round left of the point; the result scale is then 0."""
    t: DecimalType = col.dtype
    new_scale = max(0, min(t.scale, digits))
    h, l = lanes(col.data)
    drop = t.scale - digits
    if drop > 0:
        h, l = div_pow10_round(h, l, drop, half_even)          # value · 10^digits, an integer
        # back to the result scale: digits < 0 multiplies the dropped places back in
        h, l, ovf = mul_pow10(h, l, new_scale - digits)
    else:
        ovf = torch.zeros_like(h, dtype=torch.bool)
    rt = DecimalType(t.precision, new_scale)
    ok = fits(h, l, rt.precision) & ~ovf
    valid = ok if col.valid is None else col.valid & ok
    from .column import PrimColumn
    return PrimColumn(rt, pack(h, l, rt), valid)


def div_pow10_half_up(h, l, k: int):
    """signed 128 / 10^k rounded HALF_UP (away from zero at .5), exact."""
    if k <= 0:
        return h, l
    ah, al, neg = abs128(h, l)
    # divide by 10^(k-1) first (truncating), then by 10 keeping the last digit for the rounding decision
    remaining = k - 1
    while remaining > 0:
        step = min(remaining, 9)
        ah, al, _ = divmod_small_u(ah, al, 10 ** step)
        remaining -= step
    # half-up needs to know whether the digits dropped below the last one were all zero only for .5 exactly with a
    # trailing non-zero: HALF_UP rounds .5000… and .5xyz both up, so the last dropped digit alone decides
    ah, al, last = divmod_small_u(ah, al, 10)
    up = last >= 5
    ah, al = add128(ah, al, torch.zeros_like(ah), up.to(torch.int64))
    nh, nl = neg128(ah, al)
    return torch.where(neg, nh, ah), torch.where(neg, nl, al)


def div_u_vec_half_up(h, l, d: torch.Tensor):
    """signed 128 / d per element (0 < d < 2^31, an int64 tensor), rounded HALF_UP, exact: long division over
    four 32-bit limbs, then +1 on the magnitude when 2·remainder ≥ d."""
    ah, al, neg = abs128(h, l)
    x = _limbs(ah, al)
    rem = torch.zeros_like(al)
    q = [None] * 4
    for i in (3, 2, 1, 0):
        cur = (rem << 32) | x[i]                   # rem < d < 2^31 → cur < 2^63
        q[i] = cur // d
        rem = cur - q[i] * d
    qh, ql = _from_limbs(*q)
    up = (2 * rem >= d).to(torch.int64)
    qh, ql = add128(qh, ql, torch.zeros_like(qh), up)
    nh, nl = neg128(qh, ql)
    return torch.where(neg, nh, qh), torch.where(neg, nl, ql)


def pow10_128(k: int, like: torch.Tensor):
    v = _POW10[k]
    lo = v & ((1 << 64) - 1)
    lo = lo - (1 << 64) if lo >= (1 << 63) else lo
    hi = v >> 64
    return torch.full_like(like, hi), torch.full_like(like, lo)


def fits(h, l, precision: int) -> torch.Tensor:
    """|v| < 10^precision."""
    ah, al, _ = abs128(h, l)
    bh, bl = pow10_128(precision, h)
    return lt128(ah, al, bh, bl) & (ah >= 0)


def to_float64(h, l) -> torch.Tensor:
    """nearest-ish double of a signed 128-bit integer (hi·2^64 + unsigned lo)."""
    lo_u = l.to(torch.float64) + (l < 0).to(torch.float64) * 18446744073709551616.0
    return h.to(torch.float64) * 18446744073709551616.0 + lo_u


# ---------------------------------------------------------------------------------------------------------------
# columns
# ---------------------------------------------------------------------------------------------------------------

def lanes(data: torch.Tensor):
    """(hi, lo) of a decimal column's data (narrow [n] or wide [n, 2])."""
    if data.dim() == 1:
        return from_i64(data)
    return data[:, 1], data[:, 0]


def pack(h, l, t: DecimalType) -> torch.Tensor:
    """lanes → storage for type ``t`` (narrow values fit int64 because |v| < 10^18)."""
    if t.narrow:
        return l
    return torch.stack([l, h], 1)


def column(t: DecimalType, h, l, valid):
    from .column import PrimColumn
    return PrimColumn(t, pack(h, l, t), valid)


def rescale(h, l, from_scale: int, to_scale: int):
    """Change scale: multiply (exact, may overflow) or divide with HALF_UP."""
    if to_scale >= from_scale:
        return mul_pow10(h, l, to_scale - from_scale)
    nh, nl = div_pow10_half_up(h, l, from_scale - to_scale)
    return nh, nl, torch.zeros_like(h, dtype=torch.bool)


def change_type(col, t: DecimalType):
    """decimal column → decimal(p, s) (Decimal.changePrecision, HALF_UP; NULL when it does not fit)."""
    from .column import PrimColumn
    src: DecimalType = col.dtype
    h, l = lanes(col.data)
    h, l, ovf = rescale(h, l, src.scale, t.scale)
    ok = fits(h, l, t.precision) & ~ovf
    valid = ok if col.valid is None else col.valid & ok
    return PrimColumn(t, pack(h, l, t), valid)


def from_integral(col, t: DecimalType):
    from .column import PrimColumn
    h, l = from_i64(col.data.to(torch.int64))
    h, l, ovf = mul_pow10(h, l, t.scale)
    ok = fits(h, l, t.precision) & ~ovf
    return PrimColumn(t, pack(h, l, t), ok if col.valid is None else col.valid & ok)


def from_double(col, t: DecimalType):
    """double → decimal(p,s): the double's exact decimal expansion rounded HALF_UP (Spark: Decimal(double) via
    BigDecimal(Double.toString) — the shortest repr; values here go through the shortest repr digits too)."""
    from .column import PrimColumn
    vals = col.data.to(torch.float64)
    finite = torch.isfinite(vals)
    # shortest decimal representation per row on the host for exactness (rare: CASTs of doubles to decimal)
    host = vals.cpu().tolist()
    ok_host = finite.cpu().tolist()
    out = []
    for v, f in zip(host, ok_host):
        if not f:
            out.append(None)
            continue
        out.append(_pd.Decimal(repr(v)))
    return from_python(out, t, col.device, col.valid)


def from_python(values, t: DecimalType, device, valid=None):
    """Python Decimals / ints / None → decimal column (HALF_UP at the scale; NULL when it does not fit)."""
    from .column import PrimColumn
    q = _pd.Decimal(1).scaleb(-t.scale)
    un, ok = [], []
    ctx = _pd.Context(prec=80, rounding=_pd.ROUND_HALF_UP)
    for v in values:
        if v is None:
            un.append(0)
            ok.append(False)
            continue
        d = v if isinstance(v, _pd.Decimal) else _pd.Decimal(str(v))
        r = d.quantize(q, rounding=_pd.ROUND_HALF_UP, context=ctx)
        u = int(r.scaleb(t.scale, context=ctx))
        good = abs(u) < 10 ** t.precision
        un.append(u if good else 0)
        ok.append(good)
    lo = [((u & ((1 << 64) - 1)) ^ (1 << 63)) - (1 << 63) for u in un]
    hi = [u >> 64 for u in un]
    from ..ops.native import h2d
    l = h2d(lo, torch.int64, device)
    h = h2d(hi, torch.int64, device)
    v = h2d(ok, torch.bool, device)
    if valid is not None:
        v = v & valid
    return PrimColumn(t, pack(h, l, t), v)


def to_python(col) -> list:
    """decimal column → Python ``decimal.Decimal`` values (None for nulls)."""
    t: DecimalType = col.dtype
    h, l = lanes(col.data)
    hs, ls = h.cpu().tolist(), l.cpu().tolist()
    vs = col.valid.cpu().tolist() if col.valid is not None else [True] * len(ls)
    out = []
    for hh, ll, ok in zip(hs, ls, vs):
        if not ok:
            out.append(None)
            continue
        u = (hh << 64) | (ll & ((1 << 64) - 1))
        out.append(_pd.Decimal(u).scaleb(-t.scale, context=_CTX))
    return out


def render(v: _pd.Decimal, scale: int) -> str:
    """Java ``BigDecimal.toString`` of the value at the column's scale (what Spark's CAST AS STRING, to_json and
    the sinks print): exactly ``scale`` fraction digits, switching to E-notation only when the adjusted exponent
    is below -6 (e.g. 0.0000001 at scale 7 → ``1E-7``)."""
    u = int(v.scaleb(scale, context=_CTX))
    digits = str(abs(u))
    sign = "-" if u < 0 else ""
    adjusted = len(digits) - 1 - scale
    if adjusted >= -6:
        if scale == 0:
            return sign + digits
        if len(digits) <= scale:
            digits = "0" * (scale - len(digits) + 1) + digits
        return f"{sign}{digits[:-scale]}.{digits[-scale:]}"
    mant = digits if len(digits) == 1 else f"{digits[0]}.{digits[1:]}"
    return f"{sign}{mant}E{adjusted}"


def arith(op: str, a, b, at: DecimalType, bt: DecimalType):
    """a (op) b on decimal columns (integral operands must already be decimals) → decimal column of Spark's
    result type.  ``/`` and ``%`` go through the host (Python decimals, exact, HALF_UP at the result scale)."""
    from .column import and_valid
    if op in ("+", "-"):
        rt = result_add(at, bt)
        s = max(at.scale, bt.scale)
        ah, al = lanes(a.data)
        bh, bl = lanes(b.data)
        ah, al, o1 = mul_pow10(ah, al, s - at.scale)
        bh, bl, o2 = mul_pow10(bh, bl, s - bt.scale)
        h, l = add128(ah, al, bh, bl) if op == "+" else sub128(ah, al, bh, bl)
        if rt.scale < s:
            h, l = div_pow10_half_up(h, l, s - rt.scale)
        ok = fits(h, l, rt.precision) & ~o1 & ~o2
        return column(rt, h, l, _and(and_valid(a.valid, b.valid), ok))
    if op == "*":
        rt = result_mul(at, bt)
        if at.narrow and bt.narrow:
            h, l = mul64x64(a.data, b.data)
            if rt.scale < at.scale + bt.scale:
                h, l = div_pow10_half_up(h, l, at.scale + bt.scale - rt.scale)
            ok = fits(h, l, rt.precision)
            return column(rt, h, l, _and(and_valid(a.valid, b.valid), ok))
    return _arith_host(op, a, b, at, bt)


def _and(v, ok):
    return ok if v is None else v & ok


def mul64x64(a: torch.Tensor, b: torch.Tensor):
    """exact signed int64 × int64 → 128 bits via 21-bit limbs (every partial product stays below 2^63)."""
    neg = (a < 0) ^ (b < 0)
    x = torch.where(a < 0, -a, a)          # |int64| < 2^63 (decimal values are < 10^18)
    y = torch.where(b < 0, -b, b)
    M = (1 << 21) - 1
    xa = [x & M, (x >> 21) & M, (x >> 42) & M]
    ya = [y & M, (y >> 21) & M, (y >> 42) & M]
    cols = [None] * 5
    for i in range(3):
        for j in range(3):
            p = xa[i] * ya[j]
            cols[i + j] = p if cols[i + j] is None else cols[i + j] + p
    # accumulate 21-bit columns into 128 bits: value = Σ cols[k] · 2^(21k)
    h = torch.zeros_like(x)
    l = torch.zeros_like(x)
    for k in range(4, -1, -1):
        # (h, l) <<= 21, then += cols[k]
        h = (h << 21) | ((l >> 43) & ((1 << 21) - 1))
        l = l << 21
        h, l = add128(h, l, torch.zeros_like(h), cols[k])
    nh, nl = neg128(h, l)
    return torch.where(neg, nh, h), torch.where(neg, nl, l)


def _arith_host(op, a, b, at, bt):
    from .column import and_valid
    xs, ys = to_python(a), to_python(b)
    if op == "/":
        rt = result_div(at, bt)
    elif op == "%":
        rt = bounded(min(at.precision - at.scale, bt.precision - bt.scale) + max(at.scale, bt.scale),
                     max(at.scale, bt.scale))
    else:
        rt = result_mul(at, bt) if op == "*" else result_add(at, bt)
    ctx = _pd.Context(prec=80, rounding=_pd.ROUND_HALF_UP)
    out = []
    for x, y in zip(xs, ys):
        if x is None or y is None or (op in ("/", "%") and y == 0):
            out.append(None)
            continue
        out.append({"*": lambda: ctx.multiply(x, y), "/": lambda: ctx.divide(x, y),
                    "%": lambda: ctx.remainder(x, y), "+": lambda: ctx.add(x, y),
                    "-": lambda: ctx.subtract(x, y)}[op]())
    return from_python(out, rt, a.device, and_valid(a.valid, b.valid))


def compare_lanes(op: str, a, b, at: DecimalType, bt: DecimalType):
    """(result bool tensor) a (op) b after bringing both to the larger scale."""
    s = max(at.scale, bt.scale)
    ah, al = lanes(a.data)
    bh, bl = lanes(b.data)
    ah, al, _ = mul_pow10(ah, al, s - at.scale)
    bh, bl, _ = mul_pow10(bh, bl, s - bt.scale)
    lt = lt128(ah, al, bh, bl)
    eq = eq128(ah, al, bh, bl)
    return {"<": lt, "<=": lt | eq, ">": ~(lt | eq), ">=": ~lt, "=": eq, "==": eq, "!=": ~eq, "<>": ~eq}[op]


# ---------------------------------------------------------------------------------------------------------------
# aggregation: SUM over groups exactly (32-bit limb sums in int64 are exact below 2^31 rows per group)
# ---------------------------------------------------------------------------------------------------------------

def group_sum(col, gid: torch.Tensor, ngroups: int, t_out: DecimalType):
    """Σ per group → (hi, lo, any-non-null) of the unscaled sum at the input scale."""
    h, l = lanes(col.data)
    ok = col.valid_mask()
    z = torch.zeros_like(l)
    h = torch.where(ok, h, z)
    l = torch.where(ok, l, z)
    limbs = _limbs(h, l)[:3]                        # three unsigned 32-bit limbs …
    sums = []
    for x in limbs:
        acc = torch.zeros(ngroups, dtype=torch.int64, device=l.device)
        acc.index_add_(0, gid, x)
        sums.append(acc)
    top = torch.zeros(ngroups, dtype=torch.int64, device=l.device)
    top.index_add_(0, gid, (h >> 32))              # … and the signed top limb (two's complement sign)
    # reassemble: value = Σ limb_k · 2^(32k) with the top limb signed
    c = torch.zeros_like(sums[0])
    out = []
    for k in range(3):
        v = sums[k] + c
        out.append(v & MASK32)
        c = v >> 32
    t3 = top + c
    hi = (out[2] & MASK32) | (t3 << 32)
    lo = (out[0] & MASK32) | ((out[1] & MASK32) << 32)
    cnt = torch.zeros(ngroups, dtype=torch.int64, device=l.device)
    cnt.index_add_(0, gid, ok.to(torch.int64))
    return hi, lo, cnt


def agg_sum(col, gid, ngroups):
    t_out = result_sum(col.dtype)
    h, l, cnt = group_sum(col, gid, ngroups, t_out)
    ok = (cnt > 0) & fits(h, l, t_out.precision)
    return column(t_out, h, l, ok)


def agg_avg(col, gid, ngroups):
    """AVG = SUM / COUNT at scale s+4, HALF_UP (the division runs on the host: one value per group)."""
    t_in: DecimalType = col.dtype
    t_out = result_avg(t_in)
    h, l, cnt = group_sum(col, gid, ngroups, result_sum(t_in))
    hs, ls, cs = h.cpu().tolist(), l.cpu().tolist(), cnt.cpu().tolist()
    vals = []
    ctx = _pd.Context(prec=80, rounding=_pd.ROUND_HALF_UP)
    for hh, ll, c in zip(hs, ls, cs):
        if c == 0:
            vals.append(None)
            continue
        u = (hh << 64) | (ll & ((1 << 64) - 1))
        vals.append(ctx.divide(_pd.Decimal(u).scaleb(-t_in.scale, context=ctx), _pd.Decimal(c)))
    return from_python(vals, t_out, col.device)


def avg_from_sum(sum_col, cnt_col, t_in: DecimalType):
    """AVG's final step from merged (exact decimal sum, count) partials: sum / count at scale s+4, HALF_UP."""
    t_sum: DecimalType = sum_col.dtype
    t_out = result_avg(t_in)
    sums = to_python(sum_col)
    cs = cnt_col.data.cpu().tolist()
    vals = [None if (s is None or c == 0) else _CTX.divide(s, _pd.Decimal(c)) for s, c in zip(sums, cs)]
    del t_sum
    return from_python(vals, t_out, sum_col.device)


def agg_minmax(col, gid, ngroups, is_max: bool):
    """MIN / MAX per group: the order-preserving 128-bit key (hi, lo^sign) via two scatter passes."""
    from .column import PrimColumn
    t: DecimalType = col.dtype
    ok = col.valid_mask()
    if t.narrow:
        big = torch.iinfo(torch.int64)
        fill = big.min if is_max else big.max
        v = torch.where(ok, col.data, torch.full_like(col.data, fill))
        out = torch.full((ngroups,), fill, dtype=torch.int64, device=v.device)
        out = out.scatter_reduce(0, gid, v, reduce="amax" if is_max else "amin", include_self=True)
        cnt = torch.zeros(ngroups, dtype=torch.int64, device=v.device)
        cnt.index_add_(0, gid, ok.to(torch.int64))
        return PrimColumn(t, out, cnt > 0)
    h, l = lanes(col.data)
    big = torch.iinfo(torch.int64)
    fill = big.min if is_max else big.max
    hv = torch.where(ok, h, torch.full_like(h, fill))
    best_h = torch.full((ngroups,), fill, dtype=torch.int64, device=h.device)
    best_h = best_h.scatter_reduce(0, gid, hv, reduce="amax" if is_max else "amin", include_self=True)
    on_best = ok & (h == best_h[gid])
    lk = l ^ SIGN                                   # unsigned order of the low word
    lv = torch.where(on_best, lk, torch.full_like(lk, fill))
    best_l = torch.full((ngroups,), fill, dtype=torch.int64, device=h.device)
    best_l = best_l.scatter_reduce(0, gid, lv, reduce="amax" if is_max else "amin", include_self=True)
    cnt = torch.zeros(ngroups, dtype=torch.int64, device=h.device)
    cnt.index_add_(0, gid, ok.to(torch.int64))
    return column(t, best_h, best_l ^ SIGN, cnt > 0)


def to_text_values(col) -> list:
    """Rendered strings (None for null) — the to_json / sink form."""
    sc = col.dtype.scale
    return [None if v is None else render(v, sc) for v in to_python(col)]


def unscaled(value, t: DecimalType) -> Optional[int]:
    """A Python value's unscaled integer at ``t`` (HALF_UP), or None when it does not fit."""
    if value is None:
        return None
    ctx = _pd.Context(prec=80, rounding=_pd.ROUND_HALF_UP)
    d = value if isinstance(value, _pd.Decimal) else _pd.Decimal(str(value))
    u = int(d.quantize(_pd.Decimal(1).scaleb(-t.scale), rounding=_pd.ROUND_HALF_UP, context=ctx).scaleb(
        t.scale, context=ctx))
    return u if abs(u) < 10 ** t.precision else None


def const_column(value, t: DecimalType, n: int, device):
    """A literal decimal broadcast to n rows (no host→device copy: fills)."""
    from .column import PrimColumn
    u = unscaled(value, t)
    if u is None:
        z = torch.zeros(n, dtype=torch.int64, device=device)
        return PrimColumn(t, z if t.narrow else torch.zeros((n, 2), dtype=torch.int64, device=device),
                          torch.zeros(n, dtype=torch.bool, device=device))
    lo = ((u & ((1 << 64) - 1)) ^ (1 << 63)) - (1 << 63)
    if t.narrow:
        return PrimColumn(t, torch.full((n,), lo, dtype=torch.int64, device=device))
    d = torch.empty((n, 2), dtype=torch.int64, device=device)
    d[:, 0].fill_(lo)
    d[:, 1].fill_(u >> 64)
    return PrimColumn(t, d)


# ---------------------------------------------------------------------------------------------------------------
# planner-facing helpers: result types, scalar casts, column conversions
# ---------------------------------------------------------------------------------------------------------------

def result_mod(a: DecimalType, b: DecimalType) -> DecimalType:
    s = max(a.scale, b.scale)
    return bounded(min(a.precision - a.scale, b.precision - b.scale) + s, s)


def result_type(op: str, a: DecimalType, b: DecimalType) -> DecimalType:
    return {"+": result_add, "-": result_add, "*": result_mul, "/": result_div, "%": result_mod}[op](a, b)




def quantize(v, t: DecimalType):
    """A Python value as ``t`` holds it (HALF_UP at the scale), None when it overflows the precision."""
    if v is None:
        return None
    u = unscaled(v, t)
    return None if u is None else _pd.Decimal(u).scaleb(-t.scale, context=_CTX)


def literal_type(text: str) -> Optional[DecimalType]:
    """Spark: an unsuffixed literal with a fraction point is a decimal of exactly its digits (None → double: over
    38 digits)."""
    d = _pd.Decimal(text)
    sign, digits, exp = d.as_tuple()
    scale = max(0, -exp)
    nd = len(digits) + max(0, exp)
    precision = max(nd, scale, 1)
    if precision > MAX_PRECISION:
        return None
    return DecimalType(precision, scale)


def scalar_op(op: str, x, y, rt: DecimalType):
    """Constant folding of ``x op y`` for decimals (Python decimals, result at ``rt``)."""
    if x is None or y is None:
        return None
    if op in ("/", "%") and y == 0:
        return None
    r = {"+": _CTX.add, "-": _CTX.subtract, "*": _CTX.multiply, "/": _CTX.divide, "%": _CTX.remainder}[op](
        _pd.Decimal(x), _pd.Decimal(y))
    return quantize(r, rt)


def cast_scalar(v, frm, t: DecimalType):
    """One value → ``t`` (Spark Cast: strings parse as BigDecimal after trimming; doubles via their shortest repr;
    booleans 1/0; NULL when unparseable or overflowing)."""
    if v is None:
        return None
    if isinstance(v, bool):
        v = int(v)
    if isinstance(v, float):
        if v != v or v in (float("inf"), float("-inf")):
            return None
        v = repr(v)
    if isinstance(v, str):
        txt = v.strip("".join(chr(c) for c in range(33)))
        try:
            v = _pd.Decimal(txt)
        except _pd.InvalidOperation:
            return None
        if not v.is_finite():
            return None
    return quantize(v, t)


def scalar_to(v, t: DecimalType, to: str):
    """A decimal value → another type (Spark Decimal.toLong/toInt truncate toward zero; toDouble rounds)."""
    if v is None:
        return None
    if to in ("byte", "short", "int", "long"):
        from .types import wrap_int_value
        return wrap_int_value(int(v), to)            # truncates toward zero, then the low bits (Decimal.toLong)
    if to in ("double", "float"):
        return float(v)
    if to == "boolean":
        return v != 0
    if to == "string":
        return render(_pd.Decimal(v), t.scale)
    raise TypeError(to)


def true_div(x: torch.Tensor, d: float) -> torch.Tensor:
    """x / d correctly rounded on every device.  PyTorch's GPU division by a Python scalar multiplies by the
    reciprocal (1/d is inexact for d = 10^k, so e.g. 201 / 200 comes out one ulp off); a 0-dim device tensor as the
    divisor takes the true division."""
    if x.device.type == "cpu":
        return x / d
    return x / torch.full((), d, dtype=x.dtype, device=x.device)


def to_double(col):
    """decimal column → double column (correctly rounded while |unscaled| < 2^53, i.e. all narrow values up to
    15-16 digits; wide values round once more)."""
    from .column import PrimColumn
    t: DecimalType = col.dtype
    h, l = lanes(col.data)
    f = l.to(torch.float64) if t.narrow else to_float64(h, l)
    return PrimColumn("double", true_div(f, float(10 ** t.scale)) if t.scale else f, col.valid)


def to_integral(col, to: str):
    """decimal → int / long, truncating toward zero; like Spark the value wraps to the low 64 (32) bits."""
    from .column import PrimColumn
    t: DecimalType = col.dtype
    h, l = lanes(col.data)
    ah, al, neg = abs128(h, l)
    k = t.scale
    while k > 0:
        step = min(k, 9)
        ah, al, _ = divmod_small_u(ah, al, 10 ** step)
        k -= step
    nh, nl = neg128(ah, al)
    r = torch.where(neg, nl, al)
    from .types import wrap_int_tensor
    return PrimColumn(to, wrap_int_tensor(r, to), col.valid)


def ceil_floor_column(col, up: bool):
    """ceil / floor of decimal(p, s): Spark 2.4's Ceil / Floor keep a decimal, decimal(p - s + 1, 0) (bounded),
    exact: the value truncated toward zero, plus one unit away from zero when dropped digits were nonzero and the
    direction (up for ceil on positives, down for floor on negatives) leaves zero behind."""
    from .column import PrimColumn
    t: DecimalType = col.dtype
    rt = bounded(t.precision - t.scale + 1, 0)
    h, l = lanes(col.data)
    ah, al, neg = abs128(h, l)
    sticky = torch.zeros_like(neg)
    k = t.scale
    while k > 0:
        step = min(k, 9)
        ah, al, r = divmod_small_u(ah, al, 10 ** step)
        sticky |= r != 0
        k -= step
    bump = sticky & (~neg if up else neg)
    ah, al = add128(ah, al, torch.zeros_like(ah), bump.to(torch.int64))
    nh, nl = neg128(ah, al)
    h, l = torch.where(neg, nh, ah), torch.where(neg, nl, al)
    return PrimColumn(rt, pack(h, l, rt), col.valid)


def to_boolean(col):
    from .column import PrimColumn
    h, l = lanes(col.data)
    return PrimColumn("boolean", (h != 0) | (l != 0), col.valid)


def negate(col):
    h, l = lanes(col.data)
    nh, nl = neg128(h, l)
    return column(col.dtype, nh, nl, col.valid)


def absolute(col):
    h, l, _ = abs128(*lanes(col.data))
    return column(col.dtype, h, l, col.valid)


def key_parts(col):
    """Hash/equality key columns for grouping and joins: the narrow form is its own key; the wide one splits into
    its two 64-bit words."""
    from .column import PrimColumn
    if col.dtype.narrow:
        return [PrimColumn("long", col.data, col.valid)]
    return [PrimColumn("long", col.data[:, 0].contiguous(), col.valid),
            PrimColumn("long", col.data[:, 1].contiguous(), col.valid)]


def order_key(col) -> torch.Tensor:
    """int64 sort keys, most significant first (a list of 1 or 2 tensors) — callers sort lexicographically."""
    if col.dtype.narrow:
        return [col.data]
    return [col.data[:, 1], col.data[:, 0] ^ SIGN]


def aggregate(groups, col, func: str, n: int):
    """SUM / AVG / MIN / MAX over a decimal column by groups (other aggregates go through doubles)."""
    from .column import ConstColumn
    gid = groups.gid.to(torch.int64)
    ng = groups.ngroups
    if func == "sum":
        if n == 0:
            return ConstColumn(None, result_sum(col.dtype), ng, col.device).materialize()
        return agg_sum(col, gid, ng)
    if func == "sum_keep":         # merging partial sums: the partials' type is already the result type
        if n == 0:
            return ConstColumn(None, col.dtype, ng, col.device).materialize()
        h, l, cnt = group_sum(col, gid, ng, col.dtype)
        return column(col.dtype, h, l, (cnt > 0) & fits(h, l, col.dtype.precision))
    if func in ("avg", "mean"):
        if n == 0:
            return ConstColumn(None, result_avg(col.dtype), ng, col.device).materialize()
        return agg_avg(col, gid, ng)
    if func in ("min", "max"):
        if n == 0:
            return ConstColumn(None, col.dtype, ng, col.device).materialize()
        return agg_minmax(col, gid, ng, func == "max")
    return None


# ---------------------------------------------------------------------------------------------------------------
# text ↔ decimal (device kernels in dxa/ops/csrc/decimal.hip; the CPU evaluator goes through Python decimals)
# ---------------------------------------------------------------------------------------------------------------

_SIGS_DONE = False


def _sigs():
    global _SIGS_DONE
    if _SIGS_DONE:
        return
    import ctypes
    from ..ops import native as N
    p, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    N.register_sigs({"dxa_dec_from_text": [p, p, p, p, i64, i32, i32, i32, i32, p, p, p],
                     "dxa_dec_to_text": [p, i32, i32, p, i64, p, p, p, p]})
    _SIGS_DONE = True


def from_text(col, t: DecimalType, trim: bool = True):
    """string column (or JSON number tokens) → decimal(p,s): exact, HALF_UP, NULL on overflow / bad syntax."""
    from .column import PrimColumn
    n, dev = col.length, col.device
    if not col.starts.is_cuda:
        return from_python([cast_scalar(v, "string", t) if trim or v is None else _strict(v, t)
                            for v in col.to_pylist()], t, dev)
    from ..ops import native as N
    _sigs()
    out = torch.empty((n, 2) if not t.narrow else (n,), dtype=torch.int64, device=dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    N.call("dxa_dec_from_text", N.ptr(col.arena), N.ptr(col.starts.to(torch.int64)), N.ptr(col.lens.to(torch.int32)),
           N.ptr(N.u8(col.valid)), n, t.precision, t.scale, 1 if trim else 0, 0 if t.narrow else 1, N.ptr(out),
           N.ptr(ok), N.stream_handle(dev))
    return PrimColumn(t, out, ok.view(torch.bool))


def _strict(v: str, t: DecimalType):
    try:
        d = _pd.Decimal(v)
    except _pd.InvalidOperation:
        return None
    return quantize(d, t) if d.is_finite() else None


def to_text_column(col, raw: bool = False):
    """decimal column → its Java BigDecimal.toString texts: a StrColumn (CAST AS STRING) or, with ``raw``, a
    JsonColumn the serializers copy verbatim (a JSON number)."""
    from .column import JsonColumn, StrColumn, strings_from_pylist
    n, dev = col.length, col.device
    if not col.data.is_cuda:
        c = strings_from_pylist(to_text_values(col), dev)
        return JsonColumn(c.arena, c.starts, c.lens, c.valid, col.dtype) if raw else c
    from ..ops import native as N
    _sigs()
    slot = 48
    arena = torch.empty(n * slot + 16, dtype=torch.uint8, device=dev)
    starts = torch.empty(n, dtype=torch.int64, device=dev)
    lens = torch.empty(n, dtype=torch.int32, device=dev)
    N.call("dxa_dec_to_text", N.ptr(col.data.contiguous()), 0 if col.dtype.narrow else 1, col.dtype.scale,
           N.ptr(N.u8(col.valid)), n, N.ptr(arena), N.ptr(starts), N.ptr(lens), N.stream_handle(dev))
    if raw:
        return JsonColumn(arena, starts, lens, col.valid, col.dtype)
    return StrColumn(arena, starts, lens, col.valid)
