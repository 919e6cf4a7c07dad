"""Sliding time windows over retained micro-batches (reference: DataProcessing/datax-host/src/main/scala/datax/
handler/TimeWindowHandler.scala:15-68 and processor/CommonProcessorFactory.scala:156-236).

Semantics (batch time T, watermark W, windows {w_i}, max window M, batch interval B):
  E = T − W, S = E − M
  K_T  = rows of the current projected batch with ts ≥ E           (retained for later batches)
  evict retained batches with t ≤ T − (W + M)
  U    = K_T ∪ retained   (reference quirk: retained batches are only unioned when there are ≥ 2 of them —
                           ``legacy_union_quirk``, on by default for output parity)
  DataXProcessedInput_Window = U ∩ [S, E),  DataXProcessedInput_<w> = U ∩ [E − w, E),
  DataXProcessedInput rebound to U ∩ [E − B, E),  DataXProcessedInput_Batch = current batch.

MI355X design: every retained pane stays resident in HBM as a compacted columnar table (no re-parse, no host
copy), so a window view is a device-side concat + one timestamp-range mask.  Sized for 288 GB: a 5-minute window at
1 M ev/s/GPU with ~20 projected columns stays well under 100 GB.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .column import PrimColumn, StrColumn, StructColumn, Table, concat_tables, ConstColumn
from .expr import EvalError
from ..telemetry.tracing import host_section

PROCESS_PREFIX_KEY = "timewindow."


@dataclass
class TimeWindowConf:
    windows: Dict[str, int]            # view name → duration µs
    enabled: bool
    timestamp_column: Optional[str]
    watermark_us: int
    max_window_us: int
    legacy_union_quirk: bool = True

    @staticmethod
    def from_settings(d) -> "TimeWindowConf":
        from ..config.settings import PROCESS_PREFIX
        wins = {}
        for name, sub in d.group_by_sub_namespace(PROCESS_PREFIX + "timewindow.").items():
            dur = sub.get_duration_us("windowduration")
            if dur is None:
                raise EvalError(f"time window {name} has no windowduration")
            wins[name] = dur
        wm = d.get(PROCESS_PREFIX + "watermark")
        ts = d.get(PROCESS_PREFIX + "timestampcolumn")
        enabled = bool(wins) and wm is not None and bool(ts)
        quirk = d.get_bool(PROCESS_PREFIX + "timewindow_legacyunion", True)
        if not enabled:
            return TimeWindowConf({}, False, None, 0, 0, quirk)
        from ..sql.parser import parse_duration_micros
        return TimeWindowConf(wins, True, ts, parse_duration_micros(wm), max(wins.values()), quirk)


def _pane_meta(p: "Pane"):
    """The fields ``PanedTable.pieces`` tests: (lo, hi, non-empty, every row has a timestamp)."""
    return p.lo, p.hi, p.table.length > 0, bool(p.all_valid)


def _str_leaves(c, out: List[StrColumn]):
    if isinstance(c, StrColumn):
        out.append(c)
    elif isinstance(c, StructColumn):
        for k in c.children:
            _str_leaves(k, out)


def _rebuild(c, done):
    if isinstance(c, StrColumn):
        return next(done)
    if isinstance(c, StructColumn):
        return StructColumn(c.names, [_rebuild(k, done) for k in c.children], c.length, c.valid, c.is_map, c.dtype,
                            c.device)
    return c


def _compact_table(t: Table, known=None) -> Table:
    """Detach retained rows from the batch's raw input buffer (string views → own compact arena); all string leaves
    are compacted together with one host synchronisation — none when ``known`` = (leaves' concatenated lengths,
    their total) was already read with the pane statistics.  (Module-level recursion: a self-referencing nested
    function is a reference cycle, and this one would pin the batch's raw input buffer until the cyclic collector
    ran.)"""
    from ..ops.strings import compact_many
    leaves: List[StrColumn] = []
    for c in t.columns:
        _str_leaves(c, leaves)
    if known is not None:
        done = iter(compact_many(leaves, lens_all=known[0], total=known[1]))
    else:
        done = iter(compact_many(leaves))
    return Table(t.names, [_rebuild(c, done) for c in t.columns], t.length, t.device)


def _str_lens_all(t: Table):
    """The string leaves' lengths concatenated (device, int32) — None when the table has no string leaf."""
    leaves: List[StrColumn] = []
    for c in t.columns:
        _str_leaves(c, leaves)
    if len(leaves) < 2:
        return None
    from ..ops.strings import lens_concat
    return lens_concat([c.lens for c in leaves])


@dataclass
class Pane:
    """One retained micro-batch: its rows, event-time bounds of its valid rows, and cached per-query partials."""
    key: int
    table: Table
    lo: int                  # min event time of rows with a valid timestamp
    hi: int                  # max event time
    all_valid: bool          # every row has a timestamp
    partials: Dict[str, Table] = field(default_factory=dict)

    def inside(self, lo: Optional[int], hi: Optional[int]) -> bool:
        """All rows fall in [lo, hi): the pane can be used unfiltered (and its cached partials reused)."""
        return self.all_valid and self.table.length > 0 and (lo is None or self.lo >= lo) and (
            hi is None or self.hi < hi)

    def outside(self, lo: Optional[int], hi: Optional[int]) -> bool:
        return self.table.length == 0 or self.lo > self.hi or (lo is not None and self.hi < lo) or (
            hi is not None and self.lo >= hi)


class PanedTable(Table):
    """A window view = union of panes clipped to [lo, hi), kept *virtual*: nothing is concatenated unless a consumer
    needs rows.  Decomposable GROUP BY queries over it are answered from per-pane partial aggregates (cached on the
    pane for panes wholly inside the window), so a 5-minute / 1-second sliding aggregate costs one new pane's
    partials + the boundary panes + a merge of (panes × groups) partial rows, instead of re-aggregating 300 batches."""

    def __init__(self, store: "WindowStore", panes: List[Pane], lo: Optional[int], hi: Optional[int], names,
                 device):
        self.store = store
        self.panes = panes
        self.lo, self.hi = lo, hi
        self.names = list(names)
        self._device = torch.device(device)
        self.dist = panes[0].table.dist if panes else "replicated"
        self._mat: Optional[Table] = None
        self._len: Optional[int] = None
        self._pieces: Optional[List[Tuple[Pane, bool]]] = None

    def pieces(self) -> List[Tuple[Pane, bool]]:
        """(pane, fully inside) for every pane that intersects the range (``Pane.outside`` / ``Pane.inside``, inlined:
        a 5-minute window walks 300 panes, and its statements ask more than once per batch).  The view's panes and
        range are fixed for its batch, so the list is computed once — from the store's bound arrays when the view
        holds the batch's pane list (``WindowStore._batch_meta``)."""
        bm = getattr(self.store, "_batch_meta", None)
        if self._pieces is None and bm is not None and bm[0] is self.panes:
            _, plo, phi, ne, av = bm
            keep = ne & (plo <= phi)
            full = av.copy()
            if self.lo is not None:
                keep &= phi >= self.lo
                full &= plo >= self.lo
            if self.hi is not None:
                keep &= plo < self.hi
                full &= phi < self.hi
            idx = np.flatnonzero(keep)
            panes = self.panes
            self._pieces = [(panes[i], f) for i, f in zip(idx.tolist(), full[idx].tolist())]
        if self._pieces is None:
            lo, hi = self.lo, self.hi
            out = []
            for p in self.panes:
                plo, phi = p.lo, p.hi
                if plo > phi or (lo is not None and phi < lo) or (hi is not None and plo >= hi) or \
                        p.table.length == 0:
                    continue
                out.append((p, p.all_valid and (lo is None or plo >= lo) and (hi is None or phi < hi)))
            self._pieces = out
        return self._pieces

    def clipped(self, pane: Pane) -> Table:
        return self.store._range(pane.table, self.lo, self.hi)

    def _materialize(self) -> Table:
        if self._mat is None:
            parts = [p.table if full else self.clipped(p) for p, full in self.pieces()]
            parts = [t for t in parts if t.length] or [self.panes[0].table.slice(0, 0)]
            t = concat_tables(parts)
            self._mat = Table(self.names, t.columns, t.length, self._device)
            self._len = t.length
        return self._mat

    @property
    def columns(self):
        return self._materialize().columns

    @property
    def length(self):
        if self._len is None:
            n = 0
            for p, full in self.pieces():
                n += p.table.length if full else self.clipped(p).length
            self._len = n
        return self._len

    def _like(self, names, cols, length) -> Table:
        t = Table(names, cols, length, self._device)
        t.dist = self.dist
        return t


_TS_SCRATCH: Dict = {}
# pane statistics computed ahead, on the parse stream, by the JSON parse that produced a timestamp column
# (``queue_pane_stats``): (data pointer, rows) → (min, max, valid count, string bytes of the parse, parse arena)
_PANE_STATS: Dict = {}


def _scratch(dev, stream_key):
    """A ts_stats scratch (partials + a self-resetting ticket) per (device, stream): launches on different streams
    must not share the ticket."""
    from ..ops import native as N
    key = (dev, stream_key)
    scratch = _TS_SCRATCH.get(key)
    if scratch is None:
        N.register_sigs({"dxa_ts_stats_scratch_bytes": [],
                         "dxa_ts_stats": [N.c_p, N.c_p, N.c_i64, N.c_i64, N.c_p, N.c_p, N.c_p],
                         "dxa_ts_stats_lens": [N.c_p, N.c_p, N.c_i64, N.c_i64, N.c_p, N.c_p, N.c_i32, N.c_p,
                                               N.c_p, N.c_p]})
        scratch = _TS_SCRATCH[key] = torch.zeros(N.lib().dxa_ts_stats_scratch_bytes(), dtype=torch.uint8,
                                                 device=dev)
    return scratch


def queue_pane_stats(vals: torch.Tensor, valid: torch.Tensor, lens: torch.Tensor, n: int, shadows) -> torch.Tensor:
    """On the current (parse) stream, behind the parse kernel: for every timestamp-shadow row ``(val_slot,
    valid_row)`` of the parse output, [min, max, valid count, count, total bytes of every assembled string] —
    what a window pane of this batch needs (``WindowStore.process``), computed while the previous batch's
    statements still run, so the batch thread reads it without waiting.  Returns the device tensor [k, 5]."""
    from ..ops import native as N
    dev = vals.device
    st = N.stream_handle(dev)
    scratch = _scratch(dev, st)
    out = torch.zeros((len(shadows), 5), dtype=torch.int64, device=dev)
    la = lens.reshape(-1)
    lp = (ctypes.c_int64 * 1)(la.data_ptr())
    ln = (ctypes.c_int64 * 1)(la.numel())
    for k, (slot, row) in enumerate(shadows):
        N.call("dxa_ts_stats_lens", N.ptr(vals[slot]), N.ptr(valid[row]), n, -(1 << 63), ctypes.addressof(lp),
               ctypes.addressof(ln), 1 if la.numel() else 0, N.ptr(scratch), N.ptr(out[k]), st)
    return out


def register_pane_stats(ts_ptr: int, n: int, stats, arena_ptr: int) -> None:
    """The parse's statistics of one timestamp column, read back behind the parse (PendingParse.result)."""
    if len(_PANE_STATS) > 16:
        _PANE_STATS.clear()
    _PANE_STATS[(ts_ptr, n)] = (int(stats[0]), int(stats[1]), int(stats[2]), int(stats[4]), arena_ptr)


def _ts_stats(ts: torch.Tensor, ok: torch.Tensor, E: int, lens_all: Optional[torch.Tensor] = None) -> List[int]:
    """[min, max, count] of the valid timestamps and the count of valid ones >= E — one reduction launch and one
    4-word read on the GPU (reduce_stats.hip), tensor ops on the CPU.  With ``lens_all`` (the pane's string lengths)
    a fifth word, their sum, comes back in the same read: the pane's compaction then needs no read of its own."""
    if ts.is_cuda and ts.numel():
        from ..ops import native as N
        dev = ts.device
        scratch = _scratch(dev, N.stream_handle(dev))
        out = torch.empty(4 if lens_all is None else 5, dtype=torch.int64, device=dev)
        if lens_all is None:
            N.call("dxa_ts_stats", N.ptr(ts.contiguous()), N.ptr(N.u8(ok.contiguous())), ts.numel(), int(E),
                   N.ptr(scratch), N.ptr(out), N.stream_handle(dev))
        else:
            # the string bytes' total in the same pass (no separate reduction launch)
            la = lens_all.contiguous()
            lp = (ctypes.c_int64 * 1)(la.data_ptr())
            ln = (ctypes.c_int64 * 1)(la.numel())
            N.call("dxa_ts_stats_lens", N.ptr(ts.contiguous()), N.ptr(N.u8(ok.contiguous())), ts.numel(), int(E),
                   ctypes.addressof(lp), ctypes.addressof(ln), 1, N.ptr(scratch), N.ptr(out), N.stream_handle(dev))
        return out.tolist()
    big = torch.iinfo(torch.int64).max
    vals = [torch.where(ok, ts, torch.full_like(ts, big)).min(), torch.where(ok, ts, torch.full_like(ts, -big)).max(),
            ok.sum(), (ok & (ts >= E)).sum()]
    if lens_all is not None:
        vals.append(lens_all.sum(dtype=torch.int64).to(ts.device))
    return torch.stack(vals).tolist()


class WindowStore:
    def __init__(self, conf: TimeWindowConf):
        self.conf = conf
        self.past: Dict[int, Pane] = {}      # batch time µs → retained pane
        self.interval_us = 0
        self.blocks: Dict = {}               # (query fingerprint, block id) → pre-combined partials of a pane block

    def _ts(self, t: Table, lazy_valid: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
        """(timestamps, validity); with ``lazy_valid`` the validity is None when every row has one (no all-true
        mask is filled unless a caller needs it)."""
        c = t.column(self.conf.timestamp_column)
        if c is None:
            raise EvalError(f"timestamp column {self.conf.timestamp_column} not found in {t.names}")
        if isinstance(c, ConstColumn):
            c = c.materialize()
        if c.dtype != "timestamp":
            from .expr import cast_column
            c = cast_column(c, "timestamp")
        return c.data, (c.valid if lazy_valid else c.valid_mask())

    def _range(self, t: Table, lo: Optional[int], hi: Optional[int]) -> Table:
        if t.length == 0:
            return t
        ts, ok = self._ts(t)
        m = ok.clone()
        if lo is not None:
            m &= ts >= lo
        if hi is not None:
            m &= ts < hi
        if bool(m.all()):
            return t
        return t.filter(m)

    def _stats_ahead(self, projected: Table, ts: torch.Tensor, E: int):
        """The statistics the parse already queued for this timestamp column (``queue_pane_stats``), when they
        answer the common case — every event valid and none late (min ≥ E) — and every string leaf of the pane
        views the parse's bytes (so the parse's string total bounds the compaction); else None (read them now)."""
        pre = _PANE_STATS.pop((ts.data_ptr(), projected.length), None) if ts.is_cuda else None
        if pre is None:
            return None
        mn, mx, cnt, total, arena = pre
        n = projected.length
        if cnt != n or mn < E:
            return None
        leaves: List[StrColumn] = []
        for c in projected.columns:
            _str_leaves(c, leaves)
        if any(c.arena.data_ptr() != arena for c in leaves):
            return None
        return [mn, mx, cnt, n, total]

    def _pane(self, key: int, t: Table) -> Pane:
        if t.length == 0:
            return Pane(key, t, 0, -1, True)
        ts, ok = self._ts(t)
        stats = _ts_stats(ts, ok, 0)
        return Pane(key, t, int(stats[0]), int(stats[1]), int(stats[2]) == t.length)

    def process(self, projected: Table, batch_time_us: int, interval_us: int):
        """Returns (views: name → Table, current_count).  Window views are ``PanedTable``s (virtual unions)."""
        self.settle()                             # a batch that ended early left its pane uncompacted
        c = self.conf
        E = batch_time_us - c.watermark_us
        S = E - c.max_window_us
        cur = None
        if projected.length:
            # one host read for the common case (every event valid and not late): the batch's pane statistics and
            # the late-event check come back together; otherwise filter, then take the kept rows' statistics
            with host_section("windows:stats"):
                ts, ok = self._ts(projected, lazy_valid=True)
                lens_all = _str_lens_all(projected)
                got = self._stats_ahead(projected, ts, E)
                if ok is None and got is None:
                    ok = torch.ones(projected.length, dtype=torch.bool, device=ts.device)
                if got is None:
                    got = _ts_stats(ts, ok, E, lens_all)
                lo_, hi_, nok, nkeep = got[:4]
            if int(nkeep) == projected.length:
                # the new pane starts as the batch's own rows (views into the parse output); its compaction into an
                # arena of its own is queued by ``settle`` after the batch's statements, so their kernels (and the
                # status reads waiting on them) are not queued behind it
                kept = projected
                cur = Pane(batch_time_us, kept, int(lo_), int(hi_), True)
                self._pending = (cur, None if lens_all is None else (lens_all, int(got[4])))
            else:
                kept = _compact_table(projected.filter((ts >= E) if ok is None else ok & (ts >= E)))
        else:
            kept = _compact_table(projected)
        kept.dist = projected.dist
        cut = batch_time_us - (c.watermark_us + c.max_window_us)
        gone = [t for t in self.past if t <= cut]
        for t in gone:
            del self.past[t]
        self._meta_drop(gone)
        self.interval_us = interval_us
        if self.blocks:
            live = set(self.past)
            for k in [k for k, ent in self.blocks.items() if not live.issuperset(ent[0])]:
                del self.blocks[k]
        if cur is None:
            cur = self._pane(batch_time_us, kept)
        if len(self.past) > 1 or (not c.legacy_union_quirk and self.past):
            panes = [cur] + list(self.past.values())
        else:
            panes = [cur]
        from ..config.settings import NAME_PREFIX
        base = f"{NAME_PREFIX}ProcessedInput"
        names = projected.names
        dev = projected.device
        views = {f"{base}_Window": PanedTable(self, panes, S, E, names, dev)}
        for name, w in c.windows.items():
            views[name] = PanedTable(self, panes, E - w, E, names, dev)
        views[base] = PanedTable(self, panes, E - interval_us, E, names, dev)
        views[f"{base}_Batch"] = projected
        # the batch's pane bounds as arrays, in the views' pane order (PanedTable.pieces)
        m = self._meta
        cm = _pane_meta(cur)
        if len(panes) == 1:
            self._batch_meta = (panes, *(np.array([v]) for v in cm))
        else:
            self._batch_meta = (panes, *(np.concatenate(([v], a)) for v, a in zip(cm, m[1:])))
        if batch_time_us in self.past:             # a repeated batch time replaces its pane: rebuild the arrays
            self.past[batch_time_us] = cur
            self._meta = None
        else:
            self.past[batch_time_us] = cur
            if m is not None:
                self._meta = (m[0] + [batch_time_us], *(np.append(a, v) for v, a in zip(cm, m[1:])))
        return views, kept.length

    # ---- pane bounds as arrays (the window's pieces without a Python pass over 300 panes) ----------------------
    @property
    def _meta(self):
        """(keys, lo, hi, non-empty, all-valid) of ``past`` in its order; rebuilt when not maintained."""
        m = self.__dict__.get("_pmeta")
        if m is None or len(m[0]) != len(self.past):
            keys = list(self.past)
            cols = list(zip(*(_pane_meta(self.past[k]) for k in keys))) if keys else [(), (), (), ()]
            m = (keys, np.array(cols[0], dtype=np.int64), np.array(cols[1], dtype=np.int64),
                 np.array(cols[2], dtype=bool), np.array(cols[3], dtype=bool))
            self.__dict__["_pmeta"] = m
        return m

    @_meta.setter
    def _meta(self, m):
        self.__dict__["_pmeta"] = m

    def _meta_drop(self, gone):
        m = self.__dict__.get("_pmeta")
        if not gone or m is None:
            return
        k = len(gone)
        if m[0][:k] == gone:                       # the oldest panes leave from the front (keys ascend)
            self.__dict__["_pmeta"] = (m[0][k:], *(a[k:] for a in m[1:]))
        else:
            self.__dict__["_pmeta"] = None

    def settle(self) -> None:
        """Compact the batch's new pane (``process``): its string views move from the batch's input buffer to an
        arena of their own, so the pane outlives the batch without pinning that buffer."""
        p = self.__dict__.pop("_pending", None)
        if p is None:
            return
        pane, known = p
        with host_section("windows:compact"):
            t = _compact_table(pane.table, known)
        t.dist = pane.table.dist
        pane.table = t

    def retained_rows(self) -> int:
        return sum(p.table.length for p in self.past.values())
