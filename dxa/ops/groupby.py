"""Hash group-by: row → dense group id, representative rows, and per-group aggregates.

GPU path (hash_groupby.hip): hash → CAS-insert into an open-addressed HBM table → dense ids → LDS-privatised
aggregation.  Group ids are renumbered by first appearance (representative = minimum row index) so results are
deterministic and identical to the CPU reference.  Key equality is *verified* against each group's representative
row after hashing; a 64-bit collision (never observed, but possible) switches that call to an exact host-side
grouping instead of merging distinct keys.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import List, Optional

import torch

from . import native as N
from ..engine.decimal import (aggregate as decimal_aggregate, is_decimal, key_parts as decimal_key_parts,
                              to_double as decimal_to_double)
from .hashing import MAX_KEY_COLS, hash_columns, key_cols

INT32_MAX = 2**31 - 1


@dataclass
class Groups:
    gid: torch.Tensor        # [n] group id per row (int32 on GPU, int64 on CPU)
    ngroups: int
    rep: torch.Tensor        # [ngroups] int64 representative (first) row per group


def _next_pow2(x: int) -> int:
    return 1 << max(6, math.ceil(math.log2(max(1, x))))


def _on_gpu(device) -> bool:
    return torch.device(device).type == "cuda"


def group_rows(keys: List, ordered: bool = True) -> Groups:
    """Group ids of the rows.  ``ordered``: ids follow the groups' first rows (the CPU reference's numbering, and
    the order of a GROUP BY's output); intermediate groupings whose order is never seen (partial aggregates that are
    merged later) pass False and keep the device's claim order."""
    from ..engine.column import materialize, PrimColumn, StrColumn, ConstColumn
    n = keys[0].length
    device = keys[0].device
    if n == 0:
        return Groups(torch.empty(0, dtype=torch.int64, device=device), 0,
                      torch.empty(0, dtype=torch.int64, device=device))
    # constant keys do not partition anything
    keys = [k for k in keys if not (isinstance(k, ConstColumn))]
    if not keys:
        return Groups(torch.zeros(n, dtype=torch.int64, device=device), 1,
                      torch.zeros(1, dtype=torch.int64, device=device))
    keys = [materialize(k) for k in keys]
    if any(is_decimal(k.dtype) for k in keys):
        keys = [p for k in keys for p in (decimal_key_parts(k) if is_decimal(k.dtype) else [k])]
    h = hash_columns(keys)
    if _on_gpu(device):
        st = N.stream_handle(device)
        cap = _next_pow2(2 * n)
        # one allocation, initialised by the build call's own init launch: [table int64 cap | gid_of_slot int32 cap
        # | rep int32 n | gid int32 n | scal int32 2 (ngroups, bad)]
        ws = torch.empty(cap + (cap + 2 * n + 2 + 1) // 2, dtype=torch.int64, device=device)
        table = ws[:cap]
        i32 = ws[cap:].view(torch.int32)
        gid_of_slot = i32[:cap]
        rep = i32[cap:cap + n]
        gid = i32[cap + n:cap + 2 * n]
        scal = i32[cap + 2 * n:cap + 2 * n + 2]
        # initialise, then insert, number and gather in one pass (no scan over the table's slots)
        N.call("dxa_group_build_init", N.ptr(h), n, N.ptr(table), cap, N.ptr(gid_of_slot), N.ptr(scal), N.ptr(gid),
               N.ptr(rep), st)
        bad_ptr = scal.data_ptr() + 4
        kc = key_cols(keys) if 2 <= len(keys) <= MAX_KEY_COLS else None
        if kc is not None:
            N.call("dxa_verify_multi", ctypes.byref(kc), N.ptr(gid), N.ptr(rep), bad_ptr, st)   # all keys, one launch
        for k in ([] if kc is not None else keys):
            if isinstance(k, StrColumn):
                N.call("dxa_verify_str", N.ptr(k.arena), N.ptr(k.starts), N.ptr(k.lens), N.ptr(N.u8(k.valid)),
                       N.ptr(gid), N.ptr(rep), n, bad_ptr, st)
            else:
                d = k.data
                if d.dtype != torch.int64:
                    d = d.view(torch.int64) if d.dtype == torch.float64 else d.to(torch.int64)
                N.call("dxa_verify_i64", N.ptr(d), N.ptr(N.u8(k.valid)), N.ptr(gid), N.ptr(rep), n, bad_ptr, st)
        ng, bad = scal.tolist()
        if bad:
            return _exact_groups(keys, device)
        if not ordered:
            return Groups(gid, ng, rep[:ng].to(torch.int64))
        if 0 < ng and (n <= _RENUMBER_BITMAP_ROWS or ng <= _RENUMBER_MAX):
            inv = torch.empty(ng, dtype=torch.int32, device=device)
            rep_out = torch.empty(ng, dtype=torch.int64, device=device)
            N.call("dxa_group_renumber", N.ptr(gid), n, N.ptr(rep), ng, N.ptr(inv), N.ptr(rep_out), st)
            return Groups(gid, ng, rep_out)
        rep = rep[:ng].to(torch.int64)
        order = torch.argsort(rep)
        inv = torch.empty(ng, dtype=torch.int32, device=device)
        inv[order] = torch.arange(ng, dtype=torch.int32, device=device)
        gid = inv[gid.long()]
        return Groups(gid, ng, rep[order])
    # ---- CPU reference
    uniq, inv = torch.unique(h, return_inverse=True)
    ng = int(uniq.shape[0])
    rows = torch.arange(n, dtype=torch.int64, device=device)
    rep = torch.full((ng,), n, dtype=torch.int64, device=device).scatter_reduce(0, inv, rows, "amin")
    order = torch.argsort(rep)
    remap = torch.empty(ng, dtype=torch.int64, device=device)
    remap[order] = torch.arange(ng, dtype=torch.int64, device=device)
    gid = remap[inv]
    rep = rep[order]
    # verify exact equality against representatives
    for k in keys:
        vals = k.to_pylist()
        rp = rep.tolist()
        g = gid.tolist()
        for i in range(n):
            if vals[i] != vals[rp[g[i]]]:
                return _exact_groups(keys, device)
    return Groups(gid, ng, rep)


def _exact_groups(keys, device) -> Groups:
    cols = [k.to_pylist() for k in keys]
    n = keys[0].length
    seen = {}
    gid = []
    rep = []
    for i in range(n):
        t = tuple(c[i] for c in cols)
        g = seen.get(t)
        if g is None:
            g = seen[t] = len(rep)
            rep.append(i)
        gid.append(g)
    dt = torch.int32 if _on_gpu(device) else torch.int64
    return Groups(N.h2d(gid, dt, device), len(rep),
                  N.h2d(rep, torch.int64, device))


_OPS = {"sum": 0, "min": 1, "max": 2, "count": 3}


def _agg_raw(groups: Groups, data: Optional[torch.Tensor], valid: Optional[torch.Tensor], op: str,
             n: int, device) -> torch.Tensor:
    """One accumulator per group.  data: int64 or float64 tensor (None for COUNT(*))."""
    ng = groups.ngroups
    if _on_gpu(device):
        out = torch.empty(ng, dtype=torch.float64 if (data is not None and data.dtype == torch.float64 and
                                                      op != "count") else torch.int64, device=device)
        gid = groups.gid if groups.gid.dtype == torch.int32 else groups.gid.to(torch.int32)
        vt = 1 if (data is not None and data.dtype == torch.float64) else 0
        N.call("dxa_aggregate", N.ptr(gid), N.ptr(data), N.ptr(N.u8(valid)), n, ng, _OPS[op], vt, N.ptr(out),
               N.stream_handle(device))
        return out
    gid = groups.gid.to(torch.int64)
    if valid is not None:
        keep = valid
        gid = gid[keep]
        if data is not None:
            data = data[keep]
    if op == "count":
        return torch.zeros(ng, dtype=torch.int64, device=device).scatter_add_(
            0, gid, torch.ones_like(gid))
    if op == "sum":
        return torch.zeros(ng, dtype=data.dtype, device=device).scatter_add_(0, gid, data)
    if op == "min":
        init = torch.full((ng,), float("inf") if data.dtype == torch.float64 else 2**63 - 1, dtype=data.dtype,
                          device=device)
        return init.scatter_reduce(0, gid, data, "amin")
    if op == "max":
        init = torch.full((ng,), float("-inf") if data.dtype == torch.float64 else -2**63, dtype=data.dtype,
                          device=device)
        return init.scatter_reduce(0, gid, data, "amax")
    raise ValueError(op)


def aggregate(groups: Groups, col, func: str, n: int):
    """Apply one aggregate over the grouped rows.  ``col`` is None for COUNT(*).  Returns a Column of ngroups rows.

    func: count | count_star | sum | min | max | avg | first | last | stddev(_samp|_pop) | var(_samp|_pop)
    """
    from ..engine.column import PrimColumn, StrColumn, ConstColumn, materialize, column_from_pylist
    device = groups.rep.device
    ng = groups.ngroups
    if func == "count_star":
        return PrimColumn("long", _agg_raw(groups, None, None, "count", n, device))
    col = materialize(col)
    valid = col.valid
    if is_decimal(col.dtype) and func not in ("count", "first", "last"):
        r = decimal_aggregate(groups, col, func, n)
        if r is not None:
            return r
        col = decimal_to_double(col)               # variance / stddev: over doubles, as Spark casts them
        valid = col.valid
    if n == 0 and func != "count":
        # only the global aggregate has a group with no rows: every aggregate but COUNT is NULL there (Spark)
        rdt = {"avg": "double", "stddev": "double", "stddev_samp": "double", "stddev_pop": "double",
               "variance": "double", "var_samp": "double", "var_pop": "double", "std": "double"}.get(func, col.dtype)
        if func == "sum" and col.dtype in ("int", "short", "byte"):
            rdt = "long"
        return ConstColumn(None, rdt, ng, device).materialize()
    if func == "count":
        return PrimColumn("long", _agg_raw(groups, None, valid, "count", n, device))
    if func in ("first", "last"):
        if func == "first":
            idx = groups.rep
        else:
            rows = torch.arange(n, dtype=torch.int64, device=device)
            idx = torch.full((ng,), -1, dtype=torch.int64, device=device).scatter_reduce(
                0, groups.gid.to(torch.int64), rows, "amax")
        return col.take(idx)
    if isinstance(col, StrColumn) or not isinstance(col, PrimColumn):
        if func in ("min", "max"):
            return _host_minmax(groups, col, func, device)
        raise TypeError(f"{func} over {col.dtype} is not supported")
    dt = col.dtype
    data = col.data
    if data.dtype == torch.bool:
        data = data.to(torch.int64)
    cnt = None
    if valid is not None:
        cnt = _agg_raw(groups, None, valid, "count", n, device)
    if func == "sum":
        out = _agg_raw(groups, data, valid, "sum", n, device)
        rdt = "double" if data.dtype == torch.float64 else "long"
        return PrimColumn(rdt, out, None if cnt is None else cnt > 0)
    if func in ("min", "max"):
        out = _agg_raw(groups, data, valid, func, n, device)
        if col.dtype == "boolean":
            out = out.to(torch.bool)
        return PrimColumn(dt, out, None if cnt is None else cnt > 0)
    if func in ("avg", "mean"):
        s = _agg_raw(groups, data.to(torch.float64) if data.dtype != torch.float64 else data, valid, "sum", n, device)
        c = cnt if cnt is not None else _agg_raw(groups, None, None, "count", n, device)
        return PrimColumn("double", s / c.clamp(min=1).to(torch.float64), c > 0)
    if func == "m2":
        # Σ (x − mean)² per group: the partial state of the variance family (Chan merge in engine/distagg.py)
        c = (cnt if cnt is not None else _agg_raw(groups, None, None, "count", n, device)).to(torch.float64)
        return PrimColumn("double", _central_m2(groups, data.to(torch.float64), valid, c, n, device),
                          None if cnt is None else cnt > 0)
    if func in ("stddev", "stddev_samp", "stddev_pop", "variance", "var_samp", "var_pop", "std"):
        c = (cnt if cnt is not None else _agg_raw(groups, None, None, "count", n, device)).to(torch.float64)
        m2 = _central_m2(groups, data.to(torch.float64), valid, c, n, device)
        pop = func.endswith("_pop")
        denom = c if pop else (c - 1)
        var = m2 / denom.clamp(min=1)
        out = var.sqrt() if func.startswith("std") else var
        if not pop:            # Spark 2.4: the sample statistics of ONE row are NaN (null only for no rows)
            out = torch.where(c == 1, torch.full_like(out, float("nan")), out)
        return PrimColumn("double", out, c > 0)
    raise ValueError(f"unsupported aggregate {func}")


def _central_m2(groups, x, valid, c, n, device):
    """Σ (x − mean_g)² per group in two passes (group means, then centred squares): no Σx² − n·mean² cancellation —
    the values 1e9 + {1, 2, 3} have variance 1, which the one-pass form loses entirely.  Spark's CentralMomentAgg
    keeps (n, mean, M2) per partition for the same reason."""
    s = _agg_raw(groups, x, valid, "sum", n, device)
    mean = s / c.clamp(min=1)
    gid = groups.gid.to(torch.int64)
    d = x - mean[gid]
    return _agg_raw(groups, d * d, valid, "sum", n, device)


def _host_minmax(groups, col, func, device):
    """MIN/MAX over strings (and other non-numeric types): host-assisted, rarely on a hot path."""
    from ..engine.column import column_from_pylist
    vals = col.to_pylist()
    gid = groups.gid.cpu().tolist()
    best = [None] * groups.ngroups
    for v, g in zip(vals, gid):
        if v is None:
            continue
        b = best[g]
        if b is None or (v < b if func == "min" else v > b):
            best[g] = v
    return column_from_pylist(best, col.dtype, device)


# ---- fused aggregation ----------------------------------------------------------------------------------------
_MA_ADD_U64, _MA_ADD_F64, _MA_MAX = 0, 1, 2
_RENUMBER_MAX = 4096          # hash_groupby.hip kRenumberMax: one-workgroup bitonic renumbering
_RENUMBER_BITMAP_ROWS = 8192 * 64   # kBitmapRows: first-row bitmap renumbering (any number of groups)
_MV_COUNT, _MV_I64, _MV_F64, _MV_F64_ORD, _MV_NOT = 0, 1, 2, 3, 4
_F_COUNT, _F_I64, _F_F64, _F_AVG, _F_F64_ORD, _F_NOT = 0, 1, 2, 3, 4, 8       # hash_groupby.hip agg_finish_kernel
_FUSABLE = ("count_star", "count", "sum", "min", "max", "avg", "mean")
# below this many groups the per-aggregate LDS-privatised kernels win (hot lines would serialise at the memory side)
FUSED_MIN_GROUPS = 4096
_MAX_SLOTS = 64


def _f64_from_ordered(k: torch.Tensor) -> torch.Tensor:
    return torch.where(k < 0, k ^ 0x7FFFFFFFFFFFFFFF, k).view(torch.float64)


def aggregate_many(groups: Groups, reqs, n: int):
    """Evaluate several aggregates over the same groups: ``reqs`` is a list of (column or None, func) as for
    :func:`aggregate`; returns the list of result Columns.

    On the GPU with many groups the simple ones (COUNT, SUM, MIN, MAX, AVG over numeric columns) share one fused
    pass (``agg_multi_kernel``): one [group][slot] accumulator row, one memory-side atomic request per (row, 8-slot
    line) instead of one per (row, aggregate); COUNTs over the same validity mask — and the hidden counts of SUM /
    MIN / MAX / AVG — are computed once.  Everything else goes through :func:`aggregate`."""
    from ..engine.column import PrimColumn, StrColumn, materialize
    device = groups.rep.device
    ng = groups.ngroups
    if (not _on_gpu(device) or n == 0 or ng < FUSED_MIN_GROUPS or len(reqs) < 2 or
            n > INT32_MAX):
        return [aggregate(groups, c, f, n) for c, f in reqs]
    slots = []                   # (data tensor or None, valid tensor or None, kind, op)
    keyed = {}
    keep = []                    # tensors that must outlive the launch (stream-ordered frees make this implicit)

    def slot(key, data, valid, kind, op):
        s = keyed.get(key)
        if s is None:
            s = keyed[key] = len(slots)
            slots.append((data, valid, kind, op))
        return s

    def count_slot(valid):
        return slot(("count", None if valid is None else id(valid)), None, valid, _MV_COUNT, _MA_ADD_F64)

    plan = []
    for col, func in reqs:
        if func not in _FUSABLE or len(slots) > _MAX_SLOTS - 3 or sum(q is not None for q in plan) >= 64:
            plan.append(None)
            continue
        if func == "count_star":
            plan.append(("count", count_slot(None), None, None))
            continue
        col = materialize(col)
        if func == "count":
            plan.append(("count", count_slot(col.valid), None, None))
            continue
        if isinstance(col, StrColumn) or not isinstance(col, PrimColumn) or is_decimal(col.dtype):
            plan.append(None)
            continue
        data, valid = col.data, col.valid
        if data.dtype == torch.float32:
            data = data.to(torch.float64)
        elif data.dtype != torch.float64:
            data = data.to(torch.int64)
        keep.append(data)
        is_f = data.dtype == torch.float64
        cnt = count_slot(valid) if valid is not None else None
        if func in ("avg", "mean"):
            x = data if is_f else data.to(torch.float64)
            keep.append(x)
            s = slot(("sum", id(x), id(valid)), x, valid, _MV_F64, _MA_ADD_F64)
            plan.append(("avg", s, count_slot(valid), None))
        elif func == "sum":
            s = slot(("sum", id(data), id(valid)), data, valid, _MV_F64 if is_f else _MV_I64,
                     _MA_ADD_F64 if is_f else _MA_ADD_U64)
            plan.append(("sum", s, cnt, "double" if is_f else "long"))
        else:
            kind = (_MV_F64_ORD if is_f else _MV_I64) | (_MV_NOT if func == "min" else 0)
            s = slot((func, id(data), id(valid)), data, valid, kind, _MA_MAX)
            plan.append(("f64" if is_f else "i64", s, cnt, col.dtype))
    if sum(p is not None for p in plan) < 2:
        return [aggregate(groups, c, f, n) for c, f in reqs]
    # pack slots into 8-slot lines of one atomic kind each
    order = []
    line_ops = []
    for op in (_MA_ADD_U64, _MA_ADD_F64, _MA_MAX):
        mine = [i for i, sl in enumerate(slots) if sl[3] == op]
        for k in range(0, len(mine), 8):
            chunk = mine[k:k + 8]
            line_ops.append(op)
            order.extend(chunk + [None] * (8 - len(chunk)))
    nlines = len(line_ops)
    where = {}
    spec = []
    for pos, i in enumerate(order):
        if i is None:
            spec += [0, 0, -1]                # unused slot of a partly filled line
            continue
        where[i] = pos
        d, v, kind, _ = slots[i]
        spec += [0 if d is None else d.data_ptr(), 0 if v is None else N.u8(v).data_ptr(), kind]
    nslots = len(order)
    while nslots > 0 and order[nslots - 1] is None:
        nslots -= 1
    gid = groups.gid if groups.gid.dtype == torch.int32 else groups.gid.to(torch.int32)
    out = torch.empty((ng, 8 * nlines), dtype=torch.int64, device=device)
    spec_t = torch.tensor(spec, dtype=torch.int64)
    ops_t = torch.tensor(line_ops, dtype=torch.int32)
    N.call("dxa_aggregate_multi", N.ptr(gid), n, ng, nslots, spec_t.data_ptr(), nlines, ops_t.data_ptr(), N.ptr(out),
           N.stream_handle(device))
    # one finishing launch for every fused request: output data [R][ng] + validity [R][ng]
    fin, fin_of = [], {}
    for ri, p in enumerate(plan):
        if p is None:
            continue
        kind, s, c, dt = p
        skind = slots[s][2]
        if kind == "count":
            k, cnt = _F_COUNT, -1
        elif kind == "avg":
            k, cnt = _F_AVG, where[c]
        elif kind == "sum":
            k, cnt = (_F_F64 if dt == "double" else _F_I64), (-1 if c is None else where[c])
        else:
            k = (_F_F64_ORD if kind == "f64" else _F_I64) | (_F_NOT if skind & _MV_NOT else 0)
            cnt = -1 if c is None else where[c]
        fin_of[ri] = len(fin)
        fin.append((k, where[s], cnt))
    dst = torch.empty((len(fin), ng), dtype=torch.int64, device=device)
    dvalid = torch.empty((len(fin), ng), dtype=torch.uint8, device=device)
    fspec = torch.tensor([x for f in fin for x in f], dtype=torch.int32)
    N.call("dxa_aggregate_finish", N.ptr(out), ng, 8 * nlines, len(fin), fspec.data_ptr(), N.ptr(dst), N.ptr(dvalid),
           N.stream_handle(device))
    res = []
    for ri, ((col, func), p) in enumerate(zip(reqs, plan)):
        if p is None:
            res.append(aggregate(groups, col, func, n))
            continue
        kind, s, c, dt = p
        j = fin_of[ri]
        v = dst[j]
        ok = dvalid[j].view(torch.bool)
        if kind == "count":
            res.append(PrimColumn("long", v))
        elif kind == "avg":
            res.append(PrimColumn("double", v.view(torch.float64), ok))
        elif kind == "sum":
            res.append(PrimColumn(dt, v.view(torch.float64) if dt == "double" else v, None if c is None else ok))
        else:
            if kind == "f64":
                v = v.view(torch.float64)
            elif dt == "boolean":
                v = v.to(torch.bool)
            res.append(PrimColumn(dt, v, None if c is None else ok))
    del keep
    return res
