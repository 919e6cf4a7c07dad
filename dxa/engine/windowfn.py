"""SQL window functions: ``f(args) OVER (PARTITION BY … ORDER BY … [ROWS|RANGE frame])``.

The reference runs these through Spark SQL inside a transform statement (CommonProcessorFactory.scala:249-294 hands
every statement to ``spark.sql``); here each window call is evaluated column-at-a-time over device tensors:

1. partition ids from the hash group-by kernel, then ONE permutation that sorts rows by (partition, order keys) with
   stable argsorts (least significant key first);
2. in sorted order, partition / peer boundaries become flag vectors and ``cummax``/``cummin`` scans give every row its
   partition start/end and peer-group start/end — no per-partition loops;
3. ranking functions are arithmetic on those positions; ``lag``/``lead``/``first_value``/``last_value``/
   ``nth_value`` are gathers; aggregates over a frame ``[a, b]`` use prefix sums for counts and integer / decimal
   sums (exact: int64 and 32-bit decimal limbs), power-of-two block sums for double sums (no prefix differences,
   which cancel catastrophically) and a sparse table for min/max (O(n log n) build, O(1) query);
4. the result is scattered back to input row order.

Distributed scopes are re-partitioned by the PARTITION BY keys (RCCL all-to-all) before evaluation, or gathered when
there is no PARTITION BY (see ``query._exec_select``).
"""
from __future__ import annotations

from typing import Callable, List

import torch

from ..ops import groupby as G
from ..sql import ast as A
from .column import Column, ConstColumn, PrimColumn, materialize

RANKING = {"row_number", "rank", "dense_rank", "percent_rank", "cume_dist", "ntile"}
OFFSET = {"lag", "lead"}
VALUE = {"first_value", "last_value", "first", "last", "nth_value"}
FRAMED_AGGS = {"sum", "count", "avg", "mean", "min", "max"}
WINDOW_FUNCS = RANKING | OFFSET | VALUE | FRAMED_AGGS

_INT_TYPES = ("byte", "short", "int", "integer", "long", "bigint", "tinyint", "smallint")


class WindowError(Exception):
    pass


def window_calls(e: A.Expr) -> List[A.WindowCall]:
    return list(A.summary(e)[1])


def _sort_key(col: Column):
    from .query import _sort_key_tensor
    key, valid = _sort_key_tensor(col)
    return torch.where(valid, key, torch.zeros_like(key)), valid


def _literal_int(e: A.Expr, what: str) -> int:
    if isinstance(e, A.Literal) and e.type in ("int", "long"):
        return int(e.value)
    raise WindowError(f"{what} must be an integer literal")


def _rev_cummin(x: torch.Tensor) -> torch.Tensor:
    return torch.flip(torch.cummin(torch.flip(x, (0,)), 0).values, (0,))


def _minmax_frame(x: torch.Tensor, a: torch.Tensor, b: torch.Tensor, is_max: bool) -> torch.Tensor:
    """min/max of ``x[a[i] .. b[i]]`` for every i (frames assumed non-empty where used) via a sparse table."""
    n = x.shape[0]
    op = torch.maximum if is_max else torch.minimum
    levels = [x]
    k = 1
    while 2 * k <= n:
        prev = levels[-1]
        nxt = prev.clone()
        nxt[: n - k] = op(prev[: n - k], prev[k:])
        levels.append(nxt)
        k *= 2
    table = torch.stack(levels)                       # [L, n]
    length = (b - a + 1).clamp(min=1)
    lvl = torch.floor(torch.log2(length.to(torch.float64))).to(torch.int64).clamp(max=len(levels) - 1)
    # exact floor(log2) (float log2 can round up at powers of two minus epsilon)
    lvl = torch.where((1 << lvl) > length, lvl - 1, lvl)
    span = 1 << lvl
    ai = a.clamp(0, n - 1)
    bi = (b - span + 1).clamp(0, n - 1)
    return op(table[lvl, ai], table[lvl, bi])


def evaluate_window(wc: A.WindowCall, ev: Callable[[A.Expr], Column], n: int, dev) -> Column:
    """Evaluate one window call over ``n`` rows; ``ev`` evaluates a sub-expression over the same rows."""
    name = wc.func.name
    if name == "mean":
        name = "avg"
    if name not in WINDOW_FUNCS:
        raise WindowError(f"{name} is not supported as a window function")
    if wc.func.distinct:
        raise WindowError("DISTINCT is not supported in window aggregates")
    i64 = torch.int64
    if n == 0:
        return ConstColumn(None, "long" if name in RANKING - {"percent_rank", "cume_dist"} else "double", 0, dev)

    # -- one permutation: rows sorted by (partition, order keys) -----------------------------------------------
    if wc.partition:
        keys = [materialize(ev(p)) for p in wc.partition]
        gid = G.group_rows(keys).gid.to(i64)
    else:
        gid = torch.zeros(n, dtype=i64, device=dev)
    from ..ops.sort import argsort_words, sort_spec_words
    okeys = []
    specs = []
    for it in wc.order:
        col = materialize(ev(it.expr))
        okeys.append((it,) + _sort_key(col))
        nulls_first = it.nulls_first if it.nulls_first is not None else it.ascending
        specs.append((col, it.ascending, nulls_first))
    # one stable device radix argsort: partition id most significant, then the ORDER BY items
    words = sort_spec_words(specs) + [gid]
    perm = argsort_words(words)

    # -- partition / peer boundaries in sorted order ------------------------------------------------------------
    idx = torch.arange(n, device=dev, dtype=i64)
    sg = gid[perm]
    pnew = torch.ones(n, dtype=torch.bool, device=dev)
    pnew[1:] = sg[1:] != sg[:-1]
    pend_flag = torch.ones(n, dtype=torch.bool, device=dev)
    pend_flag[:-1] = pnew[1:]
    pstart = torch.cummax(torch.where(pnew, idx, torch.zeros_like(idx)), 0).values
    pend = _rev_cummin(torch.where(pend_flag, idx, torch.full_like(idx, n)))
    peer_new = pnew.clone()
    for _, key, valid in okeys:
        k, v = key[perm], valid[perm]
        if k.is_floating_point():
            same = (k[1:] == k[:-1]) | (torch.isnan(k[1:]) & torch.isnan(k[:-1]))
        else:
            same = k[1:] == k[:-1]
        peer_new[1:] |= ~same | (v[1:] != v[:-1])
    peer_end_flag = torch.ones(n, dtype=torch.bool, device=dev)
    peer_end_flag[:-1] = peer_new[1:]
    peer_start = torch.cummax(torch.where(peer_new, idx, torch.zeros_like(idx)), 0).values
    peer_end = _rev_cummin(torch.where(peer_end_flag, idx, torch.full_like(idx, n)))
    size = pend - pstart + 1
    pos = idx - pstart

    rkey = _range_key(wc, okeys, specs, perm) if _has_range_offsets(wc) else None
    res = _compute(name, wc, ev, perm, idx, pstart, pend, peer_new, peer_start, peer_end, size, pos, n, dev, rkey)
    inv = torch.empty_like(perm)
    inv[perm] = idx
    return res.take(inv)


def _has_range_offsets(wc) -> bool:
    return wc.frame is not None and wc.frame[0] == "range" and any(
        b[0] in ("preceding", "following") for b in wc.frame[1:])


def _range_key(wc, okeys, specs, perm):
    """The ORDER BY value of every row in sorted order, made ascending (DESC keys negated) with nulls mapped to the
    end of the range they sort to, for RANGE frames with value offsets (Spark: one numeric / date / timestamp
    ORDER BY expression; timestamp offsets are INTERVALs, in microseconds here)."""
    if len(wc.order) != 1:
        raise WindowError("a RANGE frame with value offsets needs exactly one ORDER BY expression")
    col, asc, nulls_first = specs[0]
    if not isinstance(col, PrimColumn) or col.dtype in ("string", "boolean"):
        raise WindowError("a RANGE frame with value offsets needs a numeric, date or timestamp ORDER BY")
    x = col.data[perm]
    valid = col.valid_mask()[perm]
    x = x.to(torch.float64) if x.is_floating_point() else x.to(torch.int64)
    if not asc:
        x = -x
    if x.is_floating_point():
        lo, hi = float("-inf"), float("inf")
    else:
        info = torch.iinfo(torch.int64)
        lo, hi = info.min, info.max
    x = torch.where(valid, x, torch.full_like(x, lo if nulls_first else hi))
    return x, valid


def _bound_search(key, lo, hi, v, strict: bool):
    """First index j in [lo, hi+1) with key[j] >= v (``strict``: key[j] > v), per row — a vectorised binary search
    inside every row's partition (key ascending within it)."""
    n = key.shape[0]
    L, R = lo.clone(), hi + 1
    for _ in range(max(1, int(n).bit_length() + 1)):
        active = L < R
        mid = (L + R) // 2
        km = key[mid.clamp(0, n - 1)]
        right = active & ((km <= v) if strict else (km < v))
        L = torch.where(right, mid + 1, L)
        R = torch.where(active & ~right, mid, R)
    return L


def _frame(wc, idx, pstart, pend, peer_start, peer_end, rkey=None):
    if wc.frame is None:
        if wc.order:
            return pstart, peer_end         # RANGE BETWEEN UNBOUNDED PRECEDING AND CURRENT ROW
        return pstart, pend
    kind, lo, hi = wc.frame

    def bound(b, is_start):
        t, k = b
        if t == "unbounded_preceding":
            return pstart
        if t == "unbounded_following":
            return pend
        if t == "current":
            if kind == "range":
                return peer_start if is_start else peer_end
            return idx
        if kind == "range":
            key, valid = rkey
            off = -k if t == "preceding" else k
            if key.is_floating_point():
                v = key + float(off)
            else:
                if isinstance(off, float):
                    raise WindowError("an integral RANGE ORDER BY needs integral offsets")
                v = key + int(off)
            pos = (_bound_search(key, pstart, pend, v, strict=False) if is_start
                   else _bound_search(key, pstart, pend, v, strict=True) - 1)
            return torch.where(valid, pos, peer_start if is_start else peer_end)   # a null key: its peers
        if isinstance(k, float):
            raise WindowError("ROWS frame offsets must be integers")
        return idx - k if t == "preceding" else idx + k

    a = torch.maximum(bound(lo, True), pstart)
    b = torch.minimum(bound(hi, False), pend)
    return a, b


def _compute(name, wc, ev, perm, idx, pstart, pend, peer_new, peer_start, peer_end, size, pos, n, dev, rkey=None):
    from .expr import _select_by_conditions
    from .query import _take_nullable
    args = wc.func.args
    if name == "row_number":
        return PrimColumn("int", (pos + 1))
    if name == "rank":
        return PrimColumn("int", (peer_start - pstart + 1))
    if name == "dense_rank":
        cs = torch.cumsum(peer_new.to(torch.int64), 0)
        return PrimColumn("int", (cs - cs[pstart] + 1))
    if name == "percent_rank":
        r = (peer_start - pstart).to(torch.float64)
        d = (size - 1).to(torch.float64)
        return PrimColumn("double", torch.where(size > 1, r / d.clamp(min=1), torch.zeros_like(r)))
    if name == "cume_dist":
        return PrimColumn("double", (peer_end - pstart + 1).to(torch.float64) / size.to(torch.float64))
    if name == "ntile":
        if len(args) != 1:
            raise WindowError("ntile takes one argument")
        k = _literal_int(args[0], "ntile bucket count")
        if k <= 0:
            raise WindowError("ntile bucket count must be positive")
        base = size // k
        rem = size % k
        big = rem * (base + 1)
        bucket = torch.where(pos < big, pos // (base + 1), rem + (pos - big) // base.clamp(min=1))
        return PrimColumn("int", (bucket + 1))

    if name in OFFSET:
        if not 1 <= len(args) <= 3:
            raise WindowError(f"{name} takes 1 to 3 arguments")
        k = _literal_int(args[1], f"{name} offset") if len(args) > 1 else 1
        col = materialize(ev(args[0])).take(perm)
        src = idx - k if name == "lag" else idx + k
        ok = (src >= pstart) & (src <= pend)
        out = _take_nullable(col, torch.where(ok, src, torch.full_like(src, -1)))
        if len(args) == 3:
            dflt = ev(args[2])
            if not isinstance(dflt, ConstColumn):
                dflt = materialize(dflt).take(perm)
            out = _select_by_conditions([PrimColumn("boolean", ok)], [out], dflt, n, dev)
        return out

    if wc.func.star or (name == "count" and not args):
        x = None
    else:
        if len(args) != (2 if name == "nth_value" else 1):
            raise WindowError(f"wrong number of arguments to {name}")
        x = materialize(ev(args[0]))
        if isinstance(x, ConstColumn):
            x = x.materialize()
        x = x.take(perm)
    a, b = _frame(wc, idx, pstart, pend, peer_start, peer_end, rkey)
    nonempty = a <= b

    if name in VALUE:
        if name in ("first_value", "first"):
            at = a
        elif name in ("last_value", "last"):
            at = b
        else:
            at = a + _literal_int(args[1], "nth_value position") - 1
        ok = nonempty & (at <= b)
        return _take_nullable(x, torch.where(ok, at, torch.full_like(at, -1)))

    # framed aggregates
    if x is None:
        cnt = torch.where(nonempty, b - a + 1, torch.zeros_like(a))
        return PrimColumn("long", cnt)
    if not isinstance(x, PrimColumn):
        raise WindowError(f"{name} OVER needs a numeric argument")
    valid = x.valid_mask()
    c = torch.cumsum(valid.to(torch.int64), 0)

    def frame_sum(pref):
        zero = torch.zeros(1, dtype=pref.dtype, device=dev)
        pz = torch.cat([zero, pref])                     # pz[j] = sum of the first j values
        hi = pz[(b + 1).clamp(0, n)]
        lo = pz[a.clamp(0, n)]
        return torch.where(nonempty, hi - lo, torch.zeros_like(hi))

    cnt = frame_sum(c)
    if name == "count":
        return PrimColumn("long", cnt)
    has = cnt > 0
    from .decimal import is_decimal
    if is_decimal(x.dtype):
        return _decimal_frame_agg(name, x, valid, a, b, nonempty, cnt, has, n, dev)
    data = x.data
    if data.dtype == torch.bool:
        data = data.to(torch.int64)
    if name in ("sum", "avg"):
        integral = x.dtype in _INT_TYPES and not data.is_floating_point()
        if integral:
            # int64 prefix differences are exact (two's complement wraps, as Spark's long sum does)
            s = frame_sum(torch.cumsum(torch.where(valid, data.to(torch.int64), torch.zeros_like(data,
                                                                                                dtype=torch.int64)),
                                       0))
        else:
            s = _float_frame_sum(torch.where(valid, data.to(torch.float64), torch.zeros_like(data,
                                                                                              dtype=torch.float64)),
                                 a, b, nonempty)
        if name == "sum":
            return PrimColumn("long" if integral else "double", s, has)
        return PrimColumn("double", s.to(torch.float64) / cnt.clamp(min=1).to(torch.float64), has)
    is_max = name == "max"
    if data.is_floating_point():
        fill = float("-inf") if is_max else float("inf")
    else:
        info = torch.iinfo(data.dtype)
        fill = info.min if is_max else info.max
    masked = torch.where(valid, data, torch.full_like(data, fill))
    return PrimColumn(x.dtype, _minmax_frame(masked, a, b, is_max), has)


def _float_frame_sum(x: torch.Tensor, a: torch.Tensor, b: torch.Tensor, nonempty: torch.Tensor) -> torch.Tensor:
    """Σ x[a[i] .. b[i]] for doubles WITHOUT prefix-sum differences (those cancel catastrophically: a 2-row frame
    over values of 1.6e12 inherits the rounding of a prefix of 3e17).  Every frame is cut into aligned power-of-two
    blocks by the bits of its length, lowest bit first: level k holds the sums of the 2^k-row runs starting at every
    row (one add of level k-1 per level), so a frame sum adds at most log2(len) block sums — each the sum of values
    inside the frame only, and exact Spark order for frames of one or two rows.  Memory stays O(n): one level at a
    time."""
    n = x.shape[0]
    length = torch.where(nonempty, b - a + 1, torch.zeros_like(a))
    acc = torch.zeros_like(x)
    if n == 0:
        return acc
    maxlen = int(length.max())                                     # one host read (the level count)
    pos = a.clamp(0, n - 1)
    level = x
    k = 0
    while (1 << k) <= maxlen:
        take = ((length >> k) & 1).to(torch.bool)
        acc = acc + torch.where(take, level[pos], torch.zeros_like(acc))
        pos = torch.where(take, (pos + (1 << k)).clamp(max=n - 1), pos)
        step = 1 << k
        if (step << 1) <= maxlen:
            nxt = level.clone()
            nxt[: n - step] = level[: n - step] + level[step:]
            level = nxt
        k += 1
    return acc


def _decimal_frame_agg(name, x, valid, a, b, nonempty, cnt, has, n, dev):
    """Framed SUM / AVG / MIN / MAX over decimal(p, s) with Spark's result types: SUM → decimal(p+10, s), AVG →
    decimal(p+4, s+4) rounded HALF_UP, MIN / MAX → the input type.  Sums are exact: the unscaled 128-bit values are
    split into 32-bit limbs whose int64 prefix sums cannot overflow below 2^31 rows, so frame differences of those
    prefixes are exact; the limbs are then carried back together (as ``decimal.group_sum`` does per group)."""
    from . import decimal as D
    t = x.dtype
    h, l = D.lanes(x.data)
    if name in ("min", "max"):
        is_max = name == "max"
        if t.narrow:
            info = torch.iinfo(torch.int64)
            fill = info.min if is_max else info.max
            masked = torch.where(valid, x.data, torch.full_like(x.data, fill))
            return PrimColumn(t, _minmax_frame(masked, a, b, is_max), has)
        at = _argbest_frame(h, l ^ D.SIGN, valid, a, b, is_max)
        return PrimColumn(t, x.data[at], has)
    z = torch.zeros_like(l)
    h = torch.where(valid, h, z)
    l = torch.where(valid, l, z)
    parts = D._limbs(h, l)[:3] + [h >> 32]                   # three unsigned limbs + the signed top limb
    zero = torch.zeros(1, dtype=torch.int64, device=dev)
    sums = []
    for p in parts:
        pz = torch.cat([zero, torch.cumsum(p, 0)])
        d = pz[(b + 1).clamp(0, n)] - pz[a.clamp(0, n)]
        sums.append(torch.where(nonempty, d, torch.zeros_like(d)))
    c = torch.zeros_like(sums[0])
    out = []
    for k in range(3):
        v = sums[k] + c
        out.append(v & D.MASK32)
        c = v >> 32
    hi = (out[2] & D.MASK32) | ((sums[3] + c) << 32)
    lo = (out[0] & D.MASK32) | ((out[1] & D.MASK32) << 32)
    if name == "sum":
        ts = D.result_sum(t)
        return D.column(ts, hi, lo, has & D.fits(hi, lo, ts.precision))
    ta = D.result_avg(t)
    hh, ll, ovf = D.mul_pow10(hi, lo, ta.scale - t.scale)
    hh, ll = D.div_u_vec_half_up(hh, ll, cnt.clamp(min=1))
    return D.column(ta, hh, ll, has & ~ovf & D.fits(hh, ll, ta.precision))


def _argbest_frame(kh: torch.Tensor, kl: torch.Tensor, valid, a, b, is_max: bool) -> torch.Tensor:
    """Row index of the max / min (kh, kl) key (lexicographic, signed) inside every frame: a sparse table of
    row indices (wide decimals, whose order key is two words)."""
    n = kh.shape[0]
    big = torch.iinfo(torch.int64)
    fill = big.min if is_max else big.max
    kh = torch.where(valid, kh, torch.full_like(kh, fill))
    kl = torch.where(valid, kl, torch.full_like(kl, fill))

    def better(i, j):                               # index of the better of rows i, j (ties: the earlier)
        gt = (kh[j] > kh[i]) | ((kh[j] == kh[i]) & (kl[j] > kl[i]))
        lt = (kh[j] < kh[i]) | ((kh[j] == kh[i]) & (kl[j] < kl[i]))
        return torch.where(gt if is_max else lt, j, i)
    idx = torch.arange(n, device=kh.device)
    levels = [idx]
    k = 1
    while 2 * k <= n:
        prev = levels[-1]
        nxt = prev.clone()
        nxt[: n - k] = better(prev[: n - k], prev[k:])
        levels.append(nxt)
        k *= 2
    table = torch.stack(levels)
    length = (b - a + 1).clamp(min=1)
    lvl = torch.floor(torch.log2(length.to(torch.float64))).to(torch.int64).clamp(max=len(levels) - 1)
    lvl = torch.where((1 << lvl) > length, lvl - 1, lvl)
    span = 1 << lvl
    ai = a.clamp(0, n - 1)
    bi = (b - span + 1).clamp(0, n - 1)
    return better(table[lvl, ai], table[lvl, bi])
