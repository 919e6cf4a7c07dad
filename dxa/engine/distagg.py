"""Distributed GROUP BY (two-phase over RCCL) for partitioned inputs — see ``dxa.parallel``.

Phase 1 (rank-local): group the rank's rows and compute *partial* states of every aggregate (count, sum, min, max,
sum of squares …).  Phase 2: route each partial group to ``hash(keys) % world`` with one all-to-all, re-group on the
owner and *merge* the partial states.  Aggregates that have no mergeable partial state (COUNT DISTINCT,
collect_list/set, user UDAFs) fall back to shuffling the input rows by key hash and aggregating once on the owner —
still one exchange, just a bigger one.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Tuple

import torch

from .. import parallel as P
from ..ops import groupby as G
from ..ops.hashing import hash_columns
from ..sql import ast as A
from . import decimal as Dec
from .column import ConstColumn, PrimColumn, Table, materialize, take_columns
from .decimal import is_decimal

DECOMPOSABLE = {"count", "sum", "min", "max", "avg", "mean", "first", "last", "first_value", "last_value",
                "stddev", "stddev_samp", "stddev_pop", "variance", "var_samp", "var_pop", "std", "count_if",
                "bool_and", "bool_or", "every", "any", "some"}


def decomposable(calls: Dict, ctx) -> bool:
    for call in calls.values():
        if call.name in ctx.udafs or call.distinct or call.name not in DECOMPOSABLE:
            return False
    return True


def _partials(call: A.Call, scope, ctx) -> List[Tuple[str, Optional[PrimColumn], str, str]]:
    """[(partial name suffix, input column, aggregate func, merge op)] for one aggregate call; the aggregates of a
    query are then evaluated together (``G.aggregate_many``)."""
    from .expr import evaluate, predicate_mask
    name = call.name
    if call.star or (name == "count" and not call.args):
        return [("cnt", None, "count_star", "sum")]
    arg = materialize(evaluate(call.args[0], scope, ctx))
    if isinstance(arg, ConstColumn):
        arg = arg.materialize()
    if name == "count":
        return [("cnt", arg, "count", "sum")]
    if name == "count_if":
        m = predicate_mask(arg)
        return [("cnt", PrimColumn("long", m.to(torch.int64)), "sum", "sum")]
    if name in ("bool_and", "every", "bool_or", "any", "some"):
        op = "min" if name in ("bool_and", "every") else "max"
        return [("v", PrimColumn("long", arg.data.to(torch.int64), arg.valid), op, op)]
    if name in ("first", "first_value", "last", "last_value"):
        f = "first" if name.startswith("first") else "last"
        return [("v", arg, f, f)]
    if is_decimal(arg.dtype):
        t = arg.dtype
        if name == "sum":          # partial sums are already of SUM's result type; merging keeps that type
            return [("v", arg, "sum", "sum_keep"), ("cnt", arg, "count", "sum")]
        if name in ("avg", "mean"):  # exact: decimal sum + count, divided once at the end (HALF_UP)
            return [(f"davg_{t.precision}_{t.scale}", arg, "sum", "sum_keep"), ("cnt", arg, "count", "sum")]
        if name not in ("min", "max"):
            arg = Dec.to_double(arg)
    if name in ("sum", "min", "max"):
        return [("v", arg, name, name), ("cnt", arg, "count", "sum")]
    if name in ("avg", "mean"):
        x = PrimColumn("double", arg.data.to(torch.float64), arg.valid)
        return [("s", x, "sum", "sum"), ("cnt", arg, "count", "sum")]
    # variance family: (count, sum, centred M2) per partial group — merged with Chan's formula (``_chan_merge``)
    x = PrimColumn("double", arg.data.to(torch.float64), arg.valid)
    return [("s", x, "sum", "sum"), ("m2", x, "m2", "m2"), ("cnt", arg, "count", "sum")]


def _finish(call: A.Call, merged: Dict[str, PrimColumn]) -> PrimColumn:
    name = call.name
    if "v" in merged:
        v = merged["v"]
        if name in ("bool_and", "every", "bool_or", "any", "some"):
            return PrimColumn("boolean", v.data != 0, v.valid)
        if "cnt" in merged:
            return v.with_valid(merged["cnt"].data > 0)
        return v
    davg = next((k for k in merged if k.startswith("davg_")), None)
    if davg is not None:
        _, p, sc = davg.split("_")
        return Dec.avg_from_sum(merged[davg], merged["cnt"], Dec.DecimalType(int(p), int(sc)))
    if set(merged) == {"cnt"}:
        c = merged["cnt"]
        return PrimColumn("long", c.data, None)
    c = merged["cnt"].data.to(torch.float64)
    s = merged["s"].data
    if name in ("avg", "mean"):
        return PrimColumn("double", s / c.clamp(min=1), c > 0)
    m2 = merged["m2"].data
    pop = name.endswith("_pop")
    var = m2 / (c if pop else (c - 1)).clamp(min=1)
    out = var.sqrt() if name.startswith("std") else var
    if not pop:                # Spark 2.4 CentralMomentAgg: NaN for one row, null for none
        out = torch.where(c == 1, torch.full_like(out, float("nan")), out)
    return PrimColumn("double", out, c > 0)


class _PFReq(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("valid", ctypes.c_void_p), ("cnt", ctypes.c_void_p),
                ("out", ctypes.c_void_p), ("out_valid", ctypes.c_void_p), ("kind", ctypes.c_int32),
                ("pad", ctypes.c_int32)]


class _PFArgs(ctypes.Structure):
    _fields_ = [("r", _PFReq * 32), ("nreq", ctypes.c_int32), ("n", ctypes.c_int64)]


def _finish_all(aggs: Dict, merged_by: Dict, ng: int, dev) -> Dict:
    """Every aggregate's final column; on the GPU the SUM / MIN / MAX validity and the AVG division of all of them
    run in one launch (``dxa_partial_finish``) instead of a compare / divide chain per aggregate."""
    out = {}
    reqs = []
    for ak, call in aggs.items():
        m = merged_by[ak]
        simple = ("v" in m and "cnt" in m and call.name not in ("bool_and", "every", "bool_or", "any", "some")
                  and len(m) == 2)
        avg = call.name in ("avg", "mean") and set(m) == {"s", "cnt"}
        if dev.type == "cuda" and ng and (simple or avg) and len(reqs) < 32:
            v = m["v"] if simple else m["s"]
            c = m["cnt"]
            if (isinstance(v, PrimColumn) and isinstance(c, PrimColumn) and v.data.dim() == 1
                    and v.data.element_size() == 8 and c.data.dtype == torch.int64):
                reqs.append((ak, call, simple, v, c))
                continue
        out[ak] = _finish(call, m)
    if reqs:
        from ..ops import native as N
        if N.lib().dxa_partial_finish_size() != ctypes.sizeof(_PFArgs):
            raise N.NativeError("PartialFinishArgs layout mismatch between distagg.py and hash_groupby.hip")
        a = _PFArgs()
        keep = []
        valid_all = torch.empty((len(reqs), ng), dtype=torch.uint8, device=dev)
        avg_out = torch.empty((sum(1 for r in reqs if not r[2]), ng), dtype=torch.float64, device=dev)
        k_avg = 0
        for j, (ak, call, simple, v, c) in enumerate(reqs):
            d = v.data.contiguous()
            cc = c.data.contiguous()
            vv = N.u8(v.valid) if simple else None             # AVG: NULL exactly when the count is 0
            keep += [d, cc] + ([vv] if vv is not None else [])
            o = avg_out[k_avg] if not simple else None
            a.r[j] = _PFReq(d.data_ptr(), 0 if vv is None else vv.data_ptr(), cc.data_ptr(),
                            0 if o is None else o.data_ptr(), valid_all[j].data_ptr(), 0 if simple else 1, 0)
            if simple:
                out[ak] = PrimColumn(v.dtype, v.data, valid_all[j].view(torch.bool))
            else:
                out[ak] = PrimColumn("double", avg_out[k_avg], valid_all[j].view(torch.bool))
                k_avg += 1
        a.nreq, a.n = len(reqs), ng
        N.call("dxa_partial_finish", ctypes.byref(a), N.stream_handle(dev))
    return {ak: out[ak] for ak in aggs}


def _one_group(n, dev):
    return G.Groups(torch.zeros(n, dtype=torch.int32 if dev.type == "cuda" else torch.int64, device=dev), 1,
                    torch.zeros(1, dtype=torch.int64, device=dev))


def local_partials(gexprs, keys, aggs: Dict, scope, ctx):
    """Phase 1: (partial table, plan, key names).  One row per local group: key columns ``__k<i>`` and partial
    states ``__a<j>_<suffix>``; ``plan[agg key] = [(column, suffix, merge op)]``.  An empty global aggregate
    contributes no row."""
    dev = scope.device
    n = scope.length
    groups = G.group_rows(keys, ordered=False) if gexprs else _one_group(n, dev)     # partials: order unseen
    names: List[str] = []
    cols = []
    key_names = []
    for i, k in enumerate(keys):
        nm = f"__k{i}"
        key_names.append(nm)
        names.append(nm)
    cols.extend(take_columns(list(keys), groups.rep if groups.ngroups and n else groups.rep[:0]))
    plan = {}
    reqs = []
    for ak, call in aggs.items():
        parts = _partials(call, scope, ctx)
        plan[ak] = []
        for suffix, arg, func, op in parts:
            nm = f"__a{len(plan)}_{suffix}"
            plan[ak].append((nm, suffix, op))
            names.append(nm)
            reqs.append((arg, func))
    cols.extend(G.aggregate_many(groups, reqs, n))
    ng_local = groups.ngroups if (gexprs or n) else 0
    if not gexprs and n == 0:
        cols = [c.take(torch.empty(0, dtype=torch.int64, device=dev)) for c in cols]
        ng_local = 0
    return Table(names, cols, ng_local, dev), plan, key_names


def exchange_partials(partial: Table, key_names: List[str], grouped: bool) -> Tuple[Table, str]:
    """Route partial groups to their key owner (grouped) or to every rank (global aggregate)."""
    dev = partial.device
    if grouped:
        dest = P.owner_of(hash_columns([partial.column(k) for k in key_names])) if partial.length else \
            torch.empty(0, dtype=torch.int64, device=dev)
        return P.shuffle_table(partial, dest), P.HASHED
    return P.allgather_table(partial), P.REPLICATED


def merge_partials(got: Table, plan, key_names: List[str], aggs: Dict, grouped: bool):
    """Phase 2: re-group partial rows and merge their states → (key columns, {agg key → final column}, ngroups)."""
    dev = got.device
    m = got.length
    if grouped:
        g2 = G.group_rows([got.column(k) for k in key_names]) if m else G.Groups(
            torch.empty(0, dtype=torch.int64, device=dev), 0, torch.empty(0, dtype=torch.int64, device=dev))
    else:
        g2 = _one_group(m, dev)
    ng = g2.ngroups
    out_keys = take_columns([got.column(k) for k in key_names], g2.rep) if grouped else []
    entries = [(ak, nm, suffix, op) for ak in aggs for nm, suffix, op in plan[ak]]
    if m == 0:
        vals = [_empty_merge(got.column(nm), op, ng, dev) for _, nm, _, op in entries]
    else:
        vals = G.aggregate_many(g2, [(got.column(nm), _merge_op(op)) for _, nm, _, op in entries], m)
        vals = _chan_merge(g2, got, entries, vals, m)
    merged_by = {ak: {} for ak in aggs}
    for (ak, _, suffix, _), v in zip(entries, vals):
        merged_by[ak][suffix] = v
    finals = _finish_all(aggs, merged_by, ng, dev)
    return out_keys, finals, ng


def combine_partials(got: Table, plan, key_names: List[str], grouped: bool) -> Table:
    """Merge partial rows into fewer partial rows of the *same* layout (partial states stay partial) — used to
    pre-combine blocks of window panes."""
    dev = got.device
    m = got.length
    if m == 0:
        return got
    g2 = G.group_rows([got.column(k) for k in key_names]) if grouped else _one_group(m, dev)
    names, cols = [], []
    for k in key_names:
        names.append(k)
        cols.append(got.column(k).take(g2.rep))
    reqs = []
    ents = []
    for ak, entries in plan.items():
        for nm, suffix, op in entries:
            names.append(nm)
            reqs.append((got.column(nm), _merge_op(op)))
            ents.append((ak, nm, suffix, op))
    cols.extend(_chan_merge(g2, got, ents, G.aggregate_many(g2, reqs, m), m))
    t = Table(names, cols, g2.ngroups, dev)
    return t


def _merge_op(op: str) -> str:
    return "sum" if op == "m2" else op


def _chan_merge(g2, got: Table, entries, vals, m: int):
    """Complete the M2 merges of the variance family: the partial M2s were summed; Chan et al.'s pairwise update
    adds Σ n_i (mean_i − mean)² over the partials of each merged group (mean = Σ s_i / Σ n_i), which is exact
    algebra for any number of partials and keeps every term centred."""
    by_agg = {}
    for j, (ak, nm, suffix, _op) in enumerate(entries):
        by_agg.setdefault(ak, {})[suffix] = (j, nm)
    gid = g2.gid.to(torch.int64)
    for ak, parts in by_agg.items():
        if "m2" not in parts:
            continue
        jm, _ = parts["m2"]
        js, ns = parts["s"]
        jc, nc = parts["cnt"]
        n_i = got.column(nc).data.to(torch.float64)
        s_i = got.column(ns).data.to(torch.float64)
        n = vals[jc].data.to(torch.float64)
        mean = vals[js].data.to(torch.float64) / n.clamp(min=1)
        mean_i = s_i / n_i.clamp(min=1)
        d = mean_i - mean[gid]
        corr = G.aggregate(g2, PrimColumn("double", torch.where(n_i > 0, n_i * d * d, torch.zeros_like(d))), "sum",
                           m)
        mv = vals[jm]
        vals[jm] = PrimColumn("double", mv.data + corr.data, mv.valid)
    return vals


def distributed_aggregate(gexprs, keys, aggs: Dict, scope, ctx):
    """Returns (key columns, {agg key → final column}, ngroups, dist tag)."""
    partial, plan, key_names = local_partials(gexprs, keys, aggs, scope, ctx)
    got, tag = exchange_partials(partial, key_names, bool(gexprs))
    out_keys, finals, ng = merge_partials(got, plan, key_names, aggs, bool(gexprs))
    return out_keys, finals, ng, tag


def _empty_merge(c, op, ng, dev):
    if is_decimal(c.dtype):
        return Dec.const_column(0 if op in ("sum", "sum_keep") else None, c.dtype, ng, dev)
    if op == "sum":
        return PrimColumn(c.dtype, torch.zeros(ng, dtype=c.data.dtype if hasattr(c, "data") else torch.int64,
                                               device=dev))
    return PrimColumn(c.dtype, torch.zeros(ng, dtype=c.data.dtype if hasattr(c, "data") else torch.int64,
                                           device=dev), torch.zeros(ng, dtype=torch.bool, device=dev))


def shuffle_rows_by_keys(scope, keys, ctx):
    """Non-decomposable fallback: route input rows to the owner of their key hash."""
    from .expr import Scope
    dev = scope.device
    names = [f"__c{i}" for i in range(len(scope.cols))] + [f"__k{i}" for i in range(len(keys))]
    t = Table(names, list(scope.cols) + list(keys), scope.length, dev)
    if keys:
        dest = P.owner_of(hash_columns(keys)) if scope.length else torch.empty(0, dtype=torch.int64, device=dev)
        got = P.shuffle_table(t, dest)
    else:
        got = P.allgather_table(t)
    nc = len(scope.cols)
    new_scope = Scope(scope.names, got.columns[:nc], scope.quals, got.length, dev)
    return new_scope, got.columns[nc:]
