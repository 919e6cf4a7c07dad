"""Dense sliding-window GROUP BY: a persistent device group dictionary + a ring of per-pane accumulator rows
(``dxa/ops/csrc/window_ring.hip``).

The reference answers a windowed statement by unioning the retained batches and running the GROUP BY over the union
every batch (DataProcessing/datax-host/src/main/scala/datax/processor/CommonProcessorFactory.scala:156-236).  The
paned path (``query._paned_aggregate``) already avoids re-reading the rows by caching per-pane partial tables, but
it still concatenates ~40 partial tables and re-groups them every batch — host-side work that kept the 300-pane
window flow host-bound.  Here the state a window needs lives in HBM in the shape the merge wants:

* a **group dictionary** (open-addressed table of key hashes → dense group id, plus each group's key values in
  fixed-width columns) that persists from batch to batch — a key seen once keeps its id for the life of the stream;
* a **ring** of accumulator rows ``[ring slot][group][stride]`` (the fused multi-aggregate's layout), one slot per
  retained pane; a pane is aggregated into its slot once, when it first enters a window;
* per batch, one kernel combines the window's slots per (group, word), flags the groups with rows in the window and
  compacts them; the host reads one 12-byte status (groups, collisions, output rows) — the statement's only
  synchronisation — and builds the output columns as views of the dictionary and the finished aggregates.

Eligible: GROUP BY statements whose aggregates are COUNT / SUM / MIN / MAX / AVG over non-decimal numeric,
boolean or timestamp arguments, with plain key columns, deterministic, on a GPU.  With N ranks each rank's window
comes out of its ring as a partial table of ``distagg.local_partials``' layout and goes through the same key
exchange and merge as the paned path (``dense_partials``).  Anything else — and any batch whose dictionary reports a hash collision, an over-long string key or a full
dictionary — is answered by the paned path, which stays the reference implementation (tests compare both).
"""
from __future__ import annotations

import ctypes
import heapq
from typing import Dict, List, Optional

import torch

from ..ops import native as N
from ..ops.groupby import (_F_AVG, _F_COUNT, _F_F64, _F_F64_ORD, _F_I64, _F_NOT, _MA_ADD_F64, _MA_ADD_U64, _MA_MAX,
                           _MV_COUNT, _MV_F64, _MV_F64_ORD, _MV_I64, _MV_NOT)
from ..ops.hashing import MAX_KEY_COLS, _KeyCols, key_cols
from .column import ConstColumn, PrimColumn, StrColumn, materialize
from .decimal import is_decimal

DENSE_GROUPS = 1 << 16            # dictionary capacity per statement (groups ever seen); more → paned path
SCRATCH_SLOTS = 4                 # ring slots for panes only partly inside a window (re-aggregated every batch)
BLOCK = 16                        # consecutive in-window panes pre-combined into one block slot, once
N.register_sigs({"dxa_win_combine_block": [N.c_p, N.c_i32, N.c_i32, N.c_p, N.c_i32, N.c_p, N.c_i32, N.c_p]})
_SUPPORTED = {"count", "sum", "min", "max", "avg", "mean"}

N.register_sigs({
    "dxa_win_sizes": [N.c_p],
    "dxa_win_init": [N.c_p, N.c_p, N.c_i64, N.c_p],
    "dxa_win_combine": [N.c_p, N.c_i32, N.c_i32, N.c_p, N.c_i32, N.c_p, N.c_i32, N.c_p, N.c_p, N.c_p, N.c_p, N.c_p],
    "dxa_win_insert_fused": [N.c_p, N.c_p, N.c_p, N.c_p, N.c_i64, N.c_p, N.c_p, N.c_p, N.c_p],
    "dxa_win_answer": [N.c_p, N.c_i32, N.c_i32, N.c_p, N.c_i32, N.c_p, N.c_i32, N.c_p, N.c_p, N.c_p, N.c_p, N.c_p,
                       N.c_p, N.c_p],
    "dxa_win_emit_size": [],
})


class _DictCol(ctypes.Structure):
    _fields_ = [("vals", ctypes.c_void_p), ("lens", ctypes.c_void_p), ("valid", ctypes.c_void_p),
                ("kind", ctypes.c_int32), ("pad", ctypes.c_int32)]


class _DictCols(ctypes.Structure):
    _fields_ = [("c", _DictCol * MAX_KEY_COLS), ("ncols", ctypes.c_int32), ("gcap", ctypes.c_int32)]


class _EmitArgs(ctypes.Structure):
    _fields_ = [("acc", ctypes.c_void_p), ("stride", ctypes.c_int32), ("nreq", ctypes.c_int32),
                ("kind", ctypes.c_int32 * 64), ("pos", ctypes.c_int32 * 64), ("cnt", ctypes.c_int32 * 64),
                ("dst", ctypes.c_void_p), ("dvalid", ctypes.c_void_p), ("okey", ctypes.c_void_p * MAX_KEY_COLS),
                ("olen", ctypes.c_void_p * MAX_KEY_COLS), ("ovalid", ctypes.c_void_p * MAX_KEY_COLS),
                ("out_idx", ctypes.c_void_p), ("scal", ctypes.c_void_p), ("gcap", ctypes.c_int32)]


_SIZES: Optional[List[int]] = None


def _sizes() -> List[int]:
    global _SIZES
    if _SIZES is None:
        out = (ctypes.c_int32 * 3)()
        N.lib().dxa_win_sizes(out)
        _SIZES = list(out)
        if _SIZES[0] != ctypes.sizeof(_KeyCols) or _SIZES[1] != ctypes.sizeof(_DictCols) or \
                N.lib().dxa_win_emit_size() != ctypes.sizeof(_EmitArgs):
            raise N.NativeError("window_ring.hip struct layout differs from window_dense.py")
    return _SIZES


class Ineligible(Exception):
    """The statement (or this batch) is answered by the paned path."""


def _requests(aggs: Dict):
    """[(agg key, func, arg expr or None)] or Ineligible."""
    out = []
    for ak, call in aggs.items():
        name = call.name
        if call.distinct or name not in _SUPPORTED:
            raise Ineligible(name)
        if call.star or (name == "count" and not call.args):
            out.append((ak, "count_star", None))
            continue
        if len(call.args) != 1:
            raise Ineligible(name)
        out.append((ak, "avg" if name == "mean" else name, call.args[0]))
    return out


class DenseWindow:
    """Persistent state of one windowed statement (one fingerprint) on one device."""

    def __init__(self, device, reqs, ring_slots: int):
        self.device = device
        self.reqs = reqs
        self.gcap = DENSE_GROUPS
        self.R = ring_slots + SCRATCH_SLOTS
        self.NB = ring_slots // BLOCK + 4              # block slots after the pane and scratch slots
        self.blocks: Dict[int, tuple] = {}             # block id → (member entry ids, block slot, entries)
        self.layout = None              # built from the first pane's evaluated argument types
        self.slot_of: Dict[int, tuple] = {}     # pane key → (ring slot, the pane, block id, pane key)
        self.free = list(range(ring_slots))    # free pane slots (a heap: the lowest is taken first)
        self.disabled = False
        self._pinned = [torch.empty(self.R, dtype=torch.int32, pin_memory=True) for _ in range(4)]
        self._scal_pin = [torch.empty(4, dtype=torch.int32, pin_memory=True) for _ in range(2)]
        self._scal_k = 0
        self._pin_k = 0
        cap = 1 << max(10, (2 * self.gcap - 1).bit_length())
        self.hcap = cap
        dev = device
        self.htab = torch.empty(cap, dtype=torch.int64, device=dev)
        self.gid_of_slot = torch.empty(cap, dtype=torch.int32, device=dev)
        self.scal = torch.zeros(4, dtype=torch.int32, device=dev)     # groups, bad flags, kept, pad
        N.call("dxa_win_init", N.ptr(self.htab), N.ptr(self.gid_of_slot), cap, N.stream_handle(dev))
        self.keys = None                # dictionary key columns, built with the layout
        self.ring = None

    # ---- layout -------------------------------------------------------------------------------------------------
    def _build_layout(self, key_cols_in: List, args: Dict):
        kw = _sizes()[2]
        dev = self.device
        if not 1 <= len(key_cols_in) <= MAX_KEY_COLS:
            raise Ineligible("key count")
        dc = _DictCols()
        keys = []
        for j, k in enumerate(key_cols_in):
            if isinstance(k, StrColumn):
                vals = torch.zeros((self.gcap + 1) * kw, dtype=torch.uint8, device=dev)
                lens = torch.zeros(self.gcap + 1, dtype=torch.int32, device=dev)
                kind = 2
            else:
                vals = torch.zeros(self.gcap + 1, dtype=torch.int64, device=dev)
                lens = None
                kind = 1 if k.data.dtype == torch.float64 else 0
            valid = torch.zeros(self.gcap + 1, dtype=torch.uint8, device=dev)
            keys.append((k.dtype, kind, vals, lens, valid))
            dc.c[j] = _DictCol(vals.data_ptr(), 0 if lens is None else lens.data_ptr(), valid.data_ptr(), kind, 0)
        dc.ncols, dc.gcap = len(keys), self.gcap
        self.keys, self.dictcols = keys, dc
        # accumulator slots, packed into 8-word lines of one atomic kind (as groupby.aggregate_many packs them)
        slots, keyed = [], {}

        def slot(key, kind, op):
            s = keyed.get(key)
            if s is None:
                s = keyed[key] = len(slots)
                slots.append((key, kind, op))
            return s

        star = slot(("count", None), _MV_COUNT, _MA_ADD_F64)
        plan = []
        for ak, func, arg in self.reqs:
            if func == "count_star":
                plan.append((ak, "count", star, None, None))
                continue
            col = args[arg.key()]
            ck = arg.key()
            cnt = slot(("count", ck), _MV_COUNT, _MA_ADD_F64)
            if func == "count":
                plan.append((ak, "count", cnt, None, None))
                continue
            is_f = col.data.dtype == torch.float64
            if func == "avg":
                plan.append((ak, "avg", slot(("sumf", ck), _MV_F64, _MA_ADD_F64), cnt, "double"))
            elif func == "sum":
                if col.dtype not in ("byte", "short", "int", "long", "double", "float"):
                    raise Ineligible("sum type")
                plan.append((ak, "sum", slot(("sum", ck), _MV_F64 if is_f else _MV_I64,
                                             _MA_ADD_F64 if is_f else _MA_ADD_U64), cnt,
                             "double" if is_f else "long"))
            else:
                kind = (_MV_F64_ORD if is_f else _MV_I64) | (_MV_NOT if func == "min" else 0)
                plan.append((ak, "f64" if is_f else "i64", slot((func, ck), kind, _MA_MAX), cnt, col.dtype))
        order, line_ops = [], []
        for op in (_MA_ADD_U64, _MA_ADD_F64, _MA_MAX):
            mine = [i for i, sl in enumerate(slots) if sl[2] == op]
            for k in range(0, len(mine), 8):
                chunk = mine[k:k + 8]
                line_ops.append(op)
                order.extend(chunk + [None] * (8 - len(chunk)))
        if len(order) > 64 or len(plan) > 64:
            raise Ineligible("too many aggregates")
        where = {i: pos for pos, i in enumerate(order) if i is not None}
        nslots = len(order)
        while nslots and order[nslots - 1] is None:
            nslots -= 1
        fin = []
        for ak, kind, s, c, dt in plan:
            if kind == "count":
                fin.append((_F_COUNT, where[s], -1))
            elif kind == "avg":
                fin.append((_F_AVG, where[s], where[c]))
            elif kind == "sum":
                fin.append((_F_F64 if dt == "double" else _F_I64, where[s], where[c]))
            else:
                k = (_F_F64_ORD if kind == "f64" else _F_I64) | (_F_NOT if slots[s][1] & _MV_NOT else 0)
                fin.append((k, where[s], where[c]))
        self.stride = 8 * len(line_ops)
        # partial states per aggregate (distagg._partials' suffixes): "cnt" a count, "v" the SUM / MIN / MAX value,
        # "s" AVG's raw double sum
        pfin = {}
        for ak, kind, s, c, dt in plan:
            if kind == "count":
                pfin[ak] = {"cnt": (_F_COUNT, where[s], -1)}
            elif kind == "avg":
                pfin[ak] = {"s": (_F_F64, where[s], where[c]), "cnt": (_F_COUNT, where[c], -1)}
            else:
                pfin[ak] = {"v": fin[len(pfin)], "cnt": (_F_COUNT, where[c], -1)}
        self.stride = 8 * len(line_ops)
        self.layout = dict(slots=slots, order=order, nslots=nslots, line_ops=line_ops, plan=plan,
                           count_word=where[star], fin=fin, pfin=pfin, pspec_of=self._partial_spec)
        self.line_ops_t = torch.tensor(line_ops, dtype=torch.int32)
        self.line_ops_dev = self.line_ops_t.to(dev)
        rows = self.gcap + 1
        self.ring = torch.empty((self.R + self.NB, rows * self.stride), dtype=torch.int64, device=dev)
        self.acc = torch.zeros(rows * self.stride, dtype=torch.int64, device=dev)
        self.keep = torch.empty(self.gcap, dtype=torch.uint8, device=dev)
        self.out_idx = torch.empty(self.gcap, dtype=torch.int64, device=dev)

    # ---- one pane into one ring slot ----------------------------------------------------------------------------
    def accumulate(self, table, slot_idx: int, alias, where, gexprs, ctx):
        from .expr import Scope, evaluate, predicate_mask
        scope = Scope.of_table(table, alias)
        n = scope.length
        keep = None
        if where is not None:
            keep = N.u8(predicate_mask(evaluate(where, scope, ctx)).contiguous())
        keys = []
        for g in gexprs:
            k = materialize(evaluate(g, scope, ctx))
            if isinstance(k, PrimColumn):
                if is_decimal(k.dtype) or k.data.dim() != 1:
                    raise Ineligible("key type")
                if k.data.dtype == torch.bool:
                    k = PrimColumn(k.dtype, k.data.to(torch.int64), k.valid)
                elif k.data.dtype not in (torch.int64, torch.float64):
                    k = PrimColumn(k.dtype, k.data.to(torch.int64), k.valid)
            elif not isinstance(k, StrColumn) or type(k) is not StrColumn:
                raise Ineligible("key type")
            keys.append(k)
        args = {}
        for _, func, arg in self.reqs:
            if arg is None or arg.key() in args:
                continue
            c = evaluate(arg, scope, ctx)
            if isinstance(c, ConstColumn):
                c = c.materialize()
            if not isinstance(c, PrimColumn) or is_decimal(c.dtype) or c.data.dim() != 1:
                raise Ineligible("argument type")
            args[arg.key()] = c
        if self.layout is None:
            self._build_layout(keys, args)
        else:
            for (dt, kind, *_), k in zip(self.keys, keys):
                if (kind == 2) != isinstance(k, StrColumn) or str(dt) != str(k.dtype):
                    raise Ineligible("key types changed")
        L = self.layout
        dev = self.device
        st = N.stream_handle(dev)
        kc = key_cols(keys)
        if kc is None:
            raise Ineligible("key columns")
        kc.ncols, kc.n = len(keys), n
        gid = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        # hash + dictionary lookup / claim + key store + verify: one launch (window_ring.hip win_insert_kernel)
        N.call("dxa_win_insert_fused", ctypes.addressof(kc), ctypes.addressof(self.dictcols), N.ptr(keep),
               N.ptr(self.htab), self.hcap, N.ptr(self.gid_of_slot), N.ptr(self.scal), N.ptr(gid), st)
        spec, hold = [], [gid, keep, kc]
        for i in L["order"][:L["nslots"]]:
            if i is None:
                spec += [0, 0, -1]
                continue
            key, kind, _op = L["slots"][i]
            if key[1] is None:
                spec += [0, 0, kind]
                continue
            c = args[key[1]]
            v = N.u8(c.valid)
            if v is not None:
                v = v.contiguous()
            if key[0] == "count":                  # a count reads only the validity: no value conversion
                hold.append(v)
                spec += [0, 0 if v is None else v.data_ptr(), kind]
                continue
            d = c.data
            if key[0] == "sumf" or (kind & 3) in (_MV_F64, _MV_F64_ORD):
                d = d.to(torch.float64)
            elif d.dtype != torch.int64:
                d = d.to(torch.int64)
            d = d.contiguous()
            hold += [d, v]
            spec += [d.data_ptr(), 0 if v is None else v.data_ptr(), kind]
        spec_t = torch.tensor(spec, dtype=torch.int64)
        ring_ptr = self.ring[slot_idx].data_ptr()
        N.call("dxa_aggregate_multi", N.ptr(gid), n, self.gcap + 1, L["nslots"], spec_t.data_ptr(),
               len(L["line_ops"]), self.line_ops_t.data_ptr(), ring_ptr, st)
        del hold

    def _dev_slots(self, slots: List[int]) -> torch.Tensor:
        pin = self._pinned[self._pin_k]
        self._pin_k = (self._pin_k + 1) % len(self._pinned)
        pin[:len(slots)] = torch.tensor(slots, dtype=torch.int32)
        return pin[:len(slots)].to(self.device, non_blocking=True)

    def block_slot(self, bid: int, mem: list) -> int:
        """The ring slot holding the pre-combined rows of a complete block of panes (combined once, when the block
        is first complete in a window; reused until a member leaves).  ``mem``: the members' slot entries."""
        # members by the identity of their slot entries: an entry is made once per pane assignment and lives in
        # slot_of while the pane is retained; the cache holds the entries too, so no id is reused while cached
        members = frozenset(map(id, mem))
        ent = self.blocks.get(bid)
        if ent is not None and ent[0] == members:
            return ent[1]
        used = {b[1] for k, b in self.blocks.items() if k != bid}
        free = [s for s in range(self.R, self.R + self.NB) if s not in used]
        if not free:
            raise Ineligible("block slots")
        dst = free[0]
        member_slots = [e[0] for e in sorted(mem, key=lambda e: e[3])]
        N.call("dxa_win_combine_block", N.ptr(self.ring), self.gcap, self.stride, N.ptr(self._dev_slots(member_slots)),
               len(member_slots), N.ptr(self.line_ops_dev), dst, N.stream_handle(self.device))
        self.blocks[bid] = (members, dst, list(mem))
        return dst

    # ---- the window's answer --------------------------------------------------------------------------------------
    def answer(self, slots: List[int], partial_proto=None, defer: bool = False):
        """Combine ``slots`` → (key columns, {agg key → column}, groups) or None (fall back: collision / full).
        With ``partial_proto`` (an empty partial table of ``distagg.local_partials``' layout, and its plan) the
        result is instead this rank's window as a partial table of exactly that layout, for the key exchange.
        ``defer``: return a function that completes the answer later — the kernels are queued and the status is on
        its way to pinned memory, so the batch thread can plan independent statements while they run."""
        L = self.layout
        dev = self.device
        st = N.stream_handle(dev)
        slots_dev = self._dev_slots(slots)
        fin = L["pspec_of"](partial_proto) if partial_proto is not None else L["fin"]
        e, bufs = self._emit_args(fin)
        N.call("dxa_win_answer", N.ptr(self.ring), self.gcap, self.stride, N.ptr(slots_dev), len(slots),
               N.ptr(self.line_ops_dev), L["count_word"], N.ptr(self.scal), N.ptr(self.acc), N.ptr(self.keep),
               N.ptr(self.out_idx), ctypes.addressof(e), ctypes.addressof(self.dictcols), st)
        if not defer:
            # the statement's one synchronising read
            return self._finish(self.scal.tolist(), bufs, fin, partial_proto)
        pin = self._scal_pin[self._scal_k]
        self._scal_k ^= 1
        pin.copy_(self.scal, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))

        def finish():
            ev.synchronize()
            return self._finish(pin.tolist(), bufs, fin, partial_proto)
        return finish

    def _finish(self, status, bufs, fin, partial_proto):
        L = self.layout
        ng_all, bad, nout, _ = status
        if bad:
            return None
        okey, olen, ovalid, dst, dvalid = bufs
        out_keys = []
        for j, (dt, kind, vals, lens, valid) in enumerate(self.keys):
            v = ovalid[j, :nout].view(torch.bool)
            if kind == 2:
                sc = StrColumn(vals, okey[j, :nout], olen[j, :nout], v)
                sc.max_len = _sizes()[2]               # a dictionary key slot: bytes per row are bounded
                out_keys.append(sc)
            else:
                d = okey[j, :nout]
                if kind == 1:
                    d = d.view(torch.float64)
                elif dt == "boolean":
                    d = d.to(torch.bool)
                out_keys.append(PrimColumn(dt, d, v))
        cols = [(dst[r, :nout], dvalid[r, :nout].view(torch.bool)) for r in range(len(fin))]
        if partial_proto is not None:
            return self._partials(cols, out_keys, nout, *partial_proto)
        finals = {}
        for (ak, kind, s, c, dt), (v, ok) in zip(L["plan"], cols):
            if kind == "count":
                finals[ak] = PrimColumn("long", v)
            elif kind == "avg":
                finals[ak] = PrimColumn("double", v.view(torch.float64), ok)
            elif kind == "sum":
                finals[ak] = PrimColumn(dt, v.view(torch.float64) if dt == "double" else v, ok)
            elif kind == "f64":
                finals[ak] = PrimColumn(dt, v.view(torch.float64), ok)
            else:
                finals[ak] = PrimColumn(dt, v.to(torch.bool) if dt == "boolean" else v, ok)
        return out_keys, finals, nout

    def _emit_args(self, fin):
        """The emit kernel's descriptor and this batch's output buffers ([gcap]-strided, fresh per batch: the
        previous batch's outputs may still be rendering on the output stream)."""
        g, dev = self.gcap, self.device
        nk, nr = len(self.keys), len(fin)
        words = torch.empty((nk + nr, g), dtype=torch.int64, device=dev)
        flags = torch.empty((nk + nr, g), dtype=torch.uint8, device=dev)
        olen = torch.empty((max(1, nk), g), dtype=torch.int32, device=dev)
        okey, dst = words[:nk], words[nk:]
        ovalid, dvalid = flags[:nk], flags[nk:]
        e = _EmitArgs()
        e.acc, e.stride, e.nreq = self.acc.data_ptr(), self.stride, nr
        for r, (k, pos, cnt) in enumerate(fin):
            e.kind[r], e.pos[r], e.cnt[r] = k, pos, cnt
        e.dst, e.dvalid = dst.data_ptr(), dvalid.data_ptr()
        for j in range(nk):
            e.okey[j], e.olen[j], e.ovalid[j] = okey[j].data_ptr(), olen[j].data_ptr(), ovalid[j].data_ptr()
        e.out_idx, e.scal, e.gcap = self.out_idx.data_ptr(), self.scal.data_ptr(), g
        return e, (okey, olen, ovalid, dst, dvalid)

    def _partial_spec(self, partial_proto):
        """Finishing spec of the partial states, in the partial table's entry order."""
        _proto, pplan, _kn = partial_proto
        L = self.layout
        out = []
        for ak, entries in pplan.items():
            for nm, suffix, _op in entries:
                f = L["pfin"].get(ak, {}).get(suffix)
                if f is None:
                    raise Ineligible(f"partial {suffix}")
                out.append(f)
        return out

    def _partials(self, cols, out_keys, nout, proto, pplan, key_names):
        """This rank's kept groups as a partial table shaped like ``proto`` (column names, types, order)."""
        from .column import Table
        got = {nm: k for nm, k in zip(key_names, out_keys)}
        j = 0
        for ak, entries in pplan.items():
            for nm, suffix, _op in entries:
                like = proto.column(nm)
                v, ok = cols[j]
                j += 1
                if suffix == "cnt":
                    got[nm] = PrimColumn(like.dtype, v)
                elif isinstance(like, PrimColumn) and like.data.dtype == torch.float64:
                    got[nm] = PrimColumn(like.dtype, v.view(torch.float64), ok)
                elif like.dtype == "boolean":
                    got[nm] = PrimColumn(like.dtype, v.to(torch.bool), ok)
                else:
                    got[nm] = PrimColumn(like.dtype, v, ok)
        return Table(list(proto.names), [got[nm] for nm in proto.names], nout, self.device)


def dense_partials(t, sel, alias: str, ctx, items, aggs: Dict, fp: str, empty):
    """Multi-rank window: this rank's window groups from the dense ring as a ``distagg.local_partials``-shaped
    partial table → (partial table, plan, key names, group exprs), or None.  The caller exchanges and merges the
    partials exactly as the paned path does, so both paths issue the same collectives (a rank that falls back
    stays in step with the others)."""
    from . import distagg as D
    from .query import _resolve_group_expr
    from .expr import Scope, evaluate
    states = t.store.__dict__.setdefault("_dense", {})
    st = states.get(fp)
    if st is not None and getattr(st, "disabled", False):
        return None
    proto_key = "_dense_proto_" + fp
    pp = t.store.__dict__.get(proto_key)
    if pp is None:
        scope = Scope.of_table(empty, alias)
        gx = [_resolve_group_expr(g, scope, items) for g in sel.group_by]
        keys = [materialize(evaluate(g, scope, ctx)) for g in gx]
        proto, plan, key_names = D.local_partials(gx, keys, aggs, scope, ctx)
        pp = t.store.__dict__[proto_key] = (proto, plan, key_names)
    got = dense_answer(t, sel, alias, ctx, items, aggs, fp, partial_proto=pp)
    if got is None:
        return None
    table, gexprs = got
    return table, pp[1], pp[2], gexprs


def dense_answer(t, sel, alias: str, ctx, items, aggs: Dict, fp: str, partial_proto=None, defer: bool = False):
    """The window statement's (key columns, finals, groups, group exprs) from the dense ring, or None.
    ``defer``: instead a function returning that tuple (or None: fall back) once the status read completes."""
    from .. import parallel as P
    from .query import _resolve_group_expr
    from .expr import Scope
    store = t.store
    dev = t._device
    if dev.type != "cuda" or not sel.group_by or (partial_proto is None and P.active() and t.dist != P.REPLICATED):
        return None
    states = store.__dict__.setdefault("_dense", {})
    state = states.get(fp)
    if state is not None and state.disabled:
        return None
    pieces = t.pieces()
    if not pieces:
        return None
    try:
        if state is None:
            iv = max(1, store.interval_us)
            panes = store.conf.max_window_us // iv + store.conf.watermark_us // iv + 4
            state = states[fp] = DenseWindow(dev, _requests(aggs), max(panes, len(pieces) + 2))
        proto = pieces[0][0].table
        gexprs = [_resolve_group_expr(g, Scope.of_table(proto, alias), items) for g in sel.group_by]
        # ring slots: a pane keeps its slot while the store retains it (a pane's rows never change — its table is only
        # compacted once; the pane object guards a re-created pane), an expired pane's slot goes back to the free
        # heap.  One pass over the window's panes.
        slot_of = state.slot_of
        past = store.past
        for k in [k for k in slot_of if k not in past]:
            heapq.heappush(state.free, slot_of.pop(k)[0])
        scratch = list(range(state.R - SCRATCH_SLOTS, state.R))
        slots = []
        span = BLOCK * max(1, store.interval_us)
        by_block: Dict[int, list] = {}
        for pane, full in pieces:
            if full:                                   # (pieces' "full" includes every row having a timestamp)
                ent = slot_of.get(pane.key)
                if ent is None or ent[1] is not pane:
                    if ent is not None:
                        heapq.heappush(state.free, ent[0])
                        del slot_of[pane.key]
                    if not state.free:
                        raise Ineligible("ring full")
                    sl = heapq.heappop(state.free)
                    state.accumulate(pane.table, sl, alias, sel.where, gexprs, ctx)
                    ent = slot_of[pane.key] = (sl, pane, pane.key // span, pane.key)
                mem = by_block.get(ent[2])
                if mem is None:
                    by_block[ent[2]] = [ent]
                else:
                    mem.append(ent)
            else:
                # a pane only partly inside the window: its in-range rows, re-aggregated into a scratch slot
                if not scratch:
                    raise Ineligible("too many clipped panes")
                sl = scratch.pop(0)
                state.accumulate(t.clipped(pane), sl, alias, sel.where, gexprs, ctx)
                slots.append(sl)
        # complete blocks of BLOCK consecutive panes: one pre-combined slot each (the per-batch combine then reads
        # ~20 block slots and the loose panes at the window's edges instead of 300 pane slots)
        for bid in [b for b in state.blocks if b not in by_block]:
            del state.blocks[bid]
        for bid, mem in by_block.items():
            if len(mem) == BLOCK:
                slots.append(state.block_slot(bid, mem))
            else:
                state.blocks.pop(bid, None)
                slots.extend(e[0] for e in mem)
        got = state.answer(slots, partial_proto, defer=defer and partial_proto is None)
    except Ineligible:
        state = states.get(fp)
        if state is not None:
            state.disabled = True
            state.ring = state.acc = None
        else:
            states[fp] = _Disabled()
        return None
    if callable(got):
        def finish():
            res = got()
            if res is None:
                state.disabled = True
                state.ring = state.acc = None
                return None
            out_keys, finals, ng = res
            return out_keys, finals, ng, gexprs
        return finish
    if got is None:
        state.disabled = True
        state.ring = state.acc = None
        return None
    if partial_proto is not None:
        return got, gexprs
    out_keys, finals, ng = got
    return out_keys, finals, ng, gexprs


class _Disabled:
    disabled = True
