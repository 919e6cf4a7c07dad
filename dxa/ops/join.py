"""Hash equi-join (inner / left / right / full / semi / anti) → (left_idx, right_idx) row pairs.

GPU path: the build side (right) is bucketed in an open-addressed HBM table (insert → per-slot counts → exclusive
scan → scatter), the probe side runs a count pass, an exclusive scan and a write pass (hash_groupby.hip).  Pairs
whose 64-bit hashes match are then checked for exact key equality, so collisions can never produce wrong rows.
A reference table that stays resident across batches (stream–static join) keeps its built table cached
(``BuiltSide``) — only the probe runs per batch.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch

from . import native as N
from .groupby import _next_pow2, _on_gpu
from .hashing import MAX_KEY_COLS, hash_columns, key_cols
from ..engine.decimal import is_decimal, key_parts as decimal_key_parts


@dataclass
class BuiltSide:
    n: int
    hashes: torch.Tensor
    table: Optional[torch.Tensor] = None
    cap: int = 0
    cnt: Optional[torch.Tensor] = None
    start: Optional[torch.Tensor] = None
    rows: Optional[torch.Tensor] = None
    null_rows: Optional[torch.Tensor] = None
    max_mult: Optional[int] = None          # most build rows behind one hash (read once, on a cached build side)


def _any_null(cols) -> Optional[torch.Tensor]:
    m = None
    for c in cols:
        if c.valid is not None:
            m = ~c.valid if m is None else (m | ~c.valid)
    return m


def _flat_keys(keys: List) -> List:
    """Wide decimal keys compare / hash as their two 64-bit words (dxa/engine/decimal.py key_parts)."""
    if not any(is_decimal(k.dtype) for k in keys):
        return keys
    from ..engine.column import materialize
    return [p for k in keys for p in (decimal_key_parts(materialize(k)) if is_decimal(k.dtype) else [k])]


def build_side(keys: List) -> BuiltSide:
    keys = _flat_keys(keys)
    n = keys[0].length
    device = keys[0].device
    h = hash_columns(keys) if n else torch.empty(0, dtype=torch.int64, device=device)
    nulls = _any_null(keys)
    b = BuiltSide(n, h, null_rows=nulls)
    if not _on_gpu(device) or n == 0:
        return b
    st = N.stream_handle(device)
    cap = _next_pow2(2 * n)
    table = torch.full((cap,), -1, dtype=torch.int64, device=device)
    slot = torch.empty(n, dtype=torch.int32, device=device)
    hh = h
    if nulls is not None:
        # null keys never match: route them to a sentinel hash that no probe uses
        hh = torch.where(nulls, torch.full_like(h, 0x3c3c3c3c3c3c3c3c), h)
    N.call("dxa_table_insert", N.ptr(hh), n, N.ptr(table), cap, N.ptr(slot), st)
    cnt = torch.zeros(cap, dtype=torch.int32, device=device)
    N.call("dxa_slot_count", N.ptr(slot), n, N.ptr(cnt), st)
    start = torch.cumsum(cnt, 0, dtype=torch.int64) - cnt.to(torch.int64)
    cursor = torch.zeros(cap, dtype=torch.int32, device=device)
    rows = torch.empty(n, dtype=torch.int32, device=device)
    N.call("dxa_slot_scatter", N.ptr(slot), n, N.ptr(start), N.ptr(cursor), N.ptr(rows), st)
    if nulls is not None:
        # hide null-key rows from probes
        cnt = cnt.clone()
        sentinel_slot = slot[nulls]
        if sentinel_slot.numel():
            cnt[sentinel_slot.long()] = 0
    b.table, b.cap, b.cnt, b.start, b.rows = table, cap, cnt, start, rows
    return b


def probe(built: BuiltSide, keys: List, outer: bool) -> Tuple[torch.Tensor, torch.Tensor]:
    """Candidate pairs by hash.  outer=True emits (i, -1) for probe rows without candidates."""
    keys = _flat_keys(keys)
    n = keys[0].length
    device = keys[0].device
    if n == 0:
        e = torch.empty(0, dtype=torch.int64, device=device)
        return e, e
    h = hash_columns(keys)
    pnull = _any_null(keys)
    if _on_gpu(device):
        st = N.stream_handle(device)
        if built.n == 0:
            if outer:
                return torch.arange(n, device=device), torch.full((n,), -1, dtype=torch.int64, device=device)
            e = torch.empty(0, dtype=torch.int64, device=device)
            return e, e
        slot = torch.empty(n, dtype=torch.int32, device=device)
        ocnt = torch.empty(n, dtype=torch.int64, device=device)
        N.call("dxa_probe_count", N.ptr(h), N.ptr(N.u8(pnull)), n, N.ptr(built.table), built.cap, N.ptr(built.cnt),
               N.ptr(slot), N.ptr(ocnt), 1 if outer else 0, st)
        off = torch.cumsum(ocnt, 0)
        total = int(off[-1].item())
        off = off - ocnt
        li = torch.empty(total, dtype=torch.int64, device=device)
        ri = torch.empty(total, dtype=torch.int64, device=device)
        N.call("dxa_probe_write", N.ptr(slot), n, N.ptr(off), N.ptr(built.start), N.ptr(built.cnt),
               N.ptr(built.rows), N.ptr(li), N.ptr(ri), 1 if outer else 0, st)
        return li, ri
    # CPU reference: sort build hashes, binary-search probes
    bh = built.hashes
    if built.null_rows is not None:
        keep = ~built.null_rows
        bidx = torch.nonzero(keep).flatten()
        bh = bh[keep]
    else:
        bidx = torch.arange(built.n, dtype=torch.int64, device=device)
    sh, order = torch.sort(bh)
    bidx = bidx[order]
    lo = torch.searchsorted(sh, h, right=False)
    hi = torch.searchsorted(sh, h, right=True)
    cnt = hi - lo
    if pnull is not None:
        cnt = torch.where(pnull, torch.zeros_like(cnt), cnt)
    li = torch.repeat_interleave(torch.arange(n, device=device), cnt)
    starts = torch.repeat_interleave(lo, cnt)
    within = torch.arange(li.shape[0], device=device) - torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt)
    ri = bidx[starts + within] if li.numel() else torch.empty(0, dtype=torch.int64, device=device)
    if outer:
        miss = torch.nonzero(cnt == 0).flatten()
        li = torch.cat([li, miss])
        ri = torch.cat([ri, torch.full_like(miss, -1)])
        order = torch.argsort(li, stable=True)
        li, ri = li[order], ri[order]
    return li, ri


def keys_equal(lcols: List, rcols: List, li: torch.Tensor, ri: torch.Tensor) -> torch.Tensor:
    """Exact key equality of candidate pairs (ri == -1 rows are reported unequal)."""
    lcols, rcols = _flat_keys(lcols), _flat_keys(rcols)
    from ..engine.column import StrColumn, PrimColumn, materialize
    device = li.device
    if device.type == "cuda" and len(lcols) <= MAX_KEY_COLS:
        L = key_cols([materialize(c) for c in lcols])
        R = key_cols([materialize(c) for c in rcols])
        if L is not None and R is not None and all(L.c[j].kind == R.c[j].kind for j in range(len(lcols))):
            m = int(li.shape[0])
            out = torch.empty(m, dtype=torch.uint8, device=device)
            if m:
                N.call("dxa_pairs_equal", ctypes.byref(L), ctypes.byref(R), N.ptr(li.to(torch.int64).contiguous()),
                       N.ptr(ri.to(torch.int64).contiguous()), m, N.ptr(out), N.stream_handle(device))
            return out.view(torch.bool)
    ok = torch.ones(li.shape[0], dtype=torch.bool, device=device)
    has = ri >= 0
    rsafe = torch.where(has, ri, torch.zeros_like(ri))
    for lc, rc in zip(lcols, rcols):
        lc, rc = materialize(lc), materialize(rc)
        a = lc.take(li)
        b = rc.take(rsafe)
        if isinstance(a, StrColumn):
            from .strings import eq_columns
            eq = eq_columns(a, b)
        else:
            da, db = a.data, b.data
            if da.dtype != db.dtype:
                da, db = da.to(torch.float64), db.to(torch.float64)
            eq = da == db
        if a.valid is not None:
            eq = eq & a.valid
        if b.valid is not None:
            eq = eq & b.valid
        ok &= eq
    return ok & has


def _unique_join(built: BuiltSide, lkeys: List, rkeys: List, kind: str) -> Tuple[torch.Tensor, torch.Tensor]:
    """A build side with at most one row per hash (a keyed reference table): every probe row has one candidate or
    none, so the pairs are positional — (i, candidate or -1) — with no count pass.  A left join reads nothing back;
    inner / semi / anti read one count."""
    keys = _flat_keys(lkeys)
    n = keys[0].length
    device = keys[0].device
    st = N.stream_handle(device)
    h = hash_columns(keys)
    pnull = _any_null(keys)
    slot = torch.empty(n, dtype=torch.int32, device=device)
    ocnt = torch.empty(n, dtype=torch.int64, device=device)
    N.call("dxa_probe_count", N.ptr(h), N.ptr(N.u8(pnull)), n, N.ptr(built.table), built.cap, N.ptr(built.cnt),
           N.ptr(slot), N.ptr(ocnt), 1, st)
    off = torch.arange(n, dtype=torch.int64, device=device)    # outer counts are all 1: row i writes pair i
    li = torch.empty(n, dtype=torch.int64, device=device)
    ri = torch.empty(n, dtype=torch.int64, device=device)
    N.call("dxa_probe_write", N.ptr(slot), n, N.ptr(off), N.ptr(built.start), N.ptr(built.cnt), N.ptr(built.rows),
           N.ptr(li), N.ptr(ri), 1, st)
    ok = keys_equal(lkeys, rkeys, li, ri)
    if kind == "left":
        return li, torch.where(ok, ri, torch.full_like(ri, -1))
    if kind == "anti":
        idx = torch.nonzero(~ok).flatten()
        return idx, torch.full_like(idx, -1)
    keep = torch.nonzero(ok).flatten()
    if kind == "semi":
        return keep, torch.full_like(keep, -1)
    return keep, ri[keep]


def hash_join(lkeys: List, rkeys: List, kind: str, built: Optional[BuiltSide] = None
              ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Row pairs of an equi-join.  kind: inner | left | right | full | semi | anti.  -1 marks a missing side."""
    device = lkeys[0].device
    nl, nr = lkeys[0].length, rkeys[0].length
    if kind == "right":
        r, l = hash_join(rkeys, lkeys, "left")
        return l, r
    if built is None:
        built = build_side(rkeys)
    elif kind in ("inner", "left", "semi", "anti") and _on_gpu(device) and built.n and nl:
        if built.max_mult is None:
            built.max_mult = int(built.cnt.max())       # once per cached (stream-static) build side
        if built.max_mult <= 1:
            return _unique_join(built, lkeys, rkeys, kind)
    li, ri = probe(built, lkeys, outer=False)
    ok = keys_equal(lkeys, rkeys, li, ri)
    keep = torch.nonzero(ok).flatten()          # one count read for both sides (two boolean indexings read twice)
    li, ri = li[keep], ri[keep]
    if kind == "inner":
        return li, ri
    matched_l = torch.zeros(nl, dtype=torch.bool, device=device)
    if li.numel():
        matched_l[li] = True
    if kind == "semi":
        idx = torch.nonzero(matched_l).flatten()
        return idx, torch.full_like(idx, -1)
    if kind == "anti":
        idx = torch.nonzero(~matched_l).flatten()
        return idx, torch.full_like(idx, -1)
    miss = torch.nonzero(~matched_l).flatten()
    li = torch.cat([li, miss])
    ri = torch.cat([ri, torch.full_like(miss, -1)])
    if kind == "full":
        matched_r = torch.zeros(nr, dtype=torch.bool, device=device)
        if ri.numel():
            matched_r[ri[ri >= 0]] = True
        rmiss = torch.nonzero(~matched_r).flatten()
        li = torch.cat([li, torch.full_like(rmiss, -1)])
        ri = torch.cat([ri, rmiss])
    order = torch.argsort(torch.where(li >= 0, li, torch.full_like(li, nl)) * (nr + 1) +
                          torch.where(ri >= 0, ri, torch.full_like(ri, nr)), stable=True)
    return li[order], ri[order]
