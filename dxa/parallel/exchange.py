"""Row exchange between ranks over RCCL (xGMI) / gloo: variable-size all-to-all of columnar tables.

A table is flattened into (a) one [rows × C] int64 matrix — every fixed-width leaf becomes one column (doubles
bit-cast, booleans widened), every string leaf contributes its byte lengths, validity travels as 63-bit masks — and
(b) one byte stream per string leaf.  Rows are stably sorted by destination so each destination's block is
contiguous; a single ``all_to_all_single`` moves the matrix (plus one per string leaf and one tiny one for the
counts).  Sized for xGMI: all blocks of a rank leave in one collective, so the 7 links are driven concurrently and the
per-call latency is paid once per exchange, not per column.
"""
from __future__ import annotations

from typing import Any, List, Optional, Tuple

import torch
import torch.distributed as dist



def _g():
    from . import group
    return group()


def _w():
    from . import _WORLD
    return _WORLD


def _staged(t: torch.Tensor) -> bool:
    """Device tensors over gloo go through host memory: lets a multi-rank run share one GPU (rehearsal of the RCCL
    path on a single-GPU machine — every kernel on the device, only the collectives on the host)."""
    return t.is_cuda and dist.get_backend(_g()) == "gloo"


def _all_reduce(t: torch.Tensor, op) -> None:
    if _staged(t):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=_g())
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=_g())


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None) -> None:
    if _staged(out):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(h, inp.cpu(), out_splits, in_splits, group=_g())
        out.copy_(h)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=_g())


def _all_gather(outs: List[torch.Tensor], t: torch.Tensor) -> None:
    if _staged(t):
        hs = [torch.empty(o.shape, dtype=o.dtype) for o in outs]
        dist.all_gather(hs, t.cpu(), group=_g())
        for o, h in zip(outs, hs):
            o.copy_(h)
    else:
        dist.all_gather(outs, t, group=_g())


def all_reduce_sum(t: torch.Tensor) -> torch.Tensor:
    if _w() > 1:
        _all_reduce(t, dist.ReduceOp.SUM)
    return t


def all_reduce_max(t: torch.Tensor) -> torch.Tensor:
    if _w() > 1:
        _all_reduce(t, dist.ReduceOp.MAX)
    return t


class MetricKeysMismatch(RuntimeError):
    """Ranks entered the batch-metrics reduction with different key sets."""


def is_max_metric(name: str) -> bool:
    """Metrics whose job-wide value is the maximum over ranks: latencies (``Latency-Blobs`` is measured from the
    earliest blob time of the whole batch, CommonProcessorFactory.scala:573-576 — the largest per-rank latency)."""
    return name.startswith("Latency-")


def _keys_digest(keys: List[str]) -> int:
    import hashlib
    h = hashlib.blake2b("\n".join(keys).encode("utf-8"), digest_size=8).digest()
    return int.from_bytes(h, "little") & ((1 << 52) - 1)       # exact in a float64


def reduce_metrics(metrics: dict, device) -> dict:
    """Job-wide batch metrics: counts summed, latencies maxed over ranks (``is_max_metric``).

    The values travel as vectors ordered by sorted key, so every rank must hold the same key set.  That is checked
    first with one 4-element MAX all-reduce of (digest, −digest, count, −count) of the key list: a mismatch shows on
    every rank (the largest digest differs from some rank's own, the smallest from another's) and raises
    ``MetricKeysMismatch`` instead of handing RCCL mismatched buffers (a hang or a silent mis-sum).  Then one SUM and
    one MAX all-reduce, read back with one host sync.  A MAX metric holding ``-inf`` on every rank (declared but
    not measured anywhere, e.g. ``Latency-Blobs`` of a batch without file times) is dropped, as the reference omits
    it."""
    if _w() <= 1:
        return {k: v for k, v in metrics.items() if not (is_max_metric(k) and v == float("-inf"))}
    keys = sorted(metrics)
    d = _keys_digest(keys)
    chk = torch.tensor([d, -d, len(keys), -len(keys)], dtype=torch.float64, device=device)
    _all_reduce(chk, dist.ReduceOp.MAX)
    got = chk.tolist()
    if got != [float(d), float(-d), float(len(keys)), float(-len(keys))]:
        from . import rank
        raise MetricKeysMismatch(f"rank {rank()}: batch metric keys differ across ranks ({len(keys)} keys here: "
                                 f"{keys})")
    skeys = [k for k in keys if not is_max_metric(k)]
    mkeys = [k for k in keys if is_max_metric(k)]
    vs = torch.tensor([float(metrics[k]) for k in skeys], dtype=torch.float64, device=device)
    vm = torch.tensor([float(metrics[k]) for k in mkeys], dtype=torch.float64, device=device)
    if skeys:
        _all_reduce(vs, dist.ReduceOp.SUM)
    if mkeys:
        _all_reduce(vm, dist.ReduceOp.MAX)
    out = dict(metrics)
    vals = torch.cat([vs, vm]).tolist()
    for k, v in zip(skeys + mkeys, vals):
        if is_max_metric(k) and v == float("-inf"):
            out.pop(k, None)
        else:
            out[k] = v
    return out


def order_point(device) -> None:
    """A point every rank's later stream work is ordered after: one 1-element all-reduce on the current stream.
    Over RCCL it does not block the host — work queued after it on this stream (and host threads waiting on events
    recorded after it) cannot run before every rank has issued it, i.e. before every rank's host got here; over gloo
    it is a host barrier."""
    if _w() > 1:
        t = torch.zeros(1, dtype=torch.float32, device=device)
        _all_reduce(t, dist.ReduceOp.SUM)


def _a2a_counts(counts: torch.Tensor) -> torch.Tensor:
    out = torch.empty_like(counts)
    _a2a(out, counts)
    return out


# ---------------------------------------------------------------------------------------------------------------
# flatten / rebuild
# ---------------------------------------------------------------------------------------------------------------

class _Leaf:
    __slots__ = ("kind", "dtype", "col", "mcol", "vbit", "value", "torch_dtype")

    def __init__(self, kind, dtype, col=None, value=None):
        self.kind, self.dtype, self.col, self.value = kind, dtype, col, value
        self.mcol = -1
        self.vbit = -1
        self.torch_dtype = None


def _flatten(col, leaves: List[_Leaf], spec: list):
    """Walk a column tree; record leaves (data-bearing) and a rebuild spec."""
    from ..engine.column import ArrayColumn, ConstColumn, JsonColumn, PrimColumn, StrColumn, StructColumn
    if isinstance(col, ConstColumn):
        spec.append(("const", col.value, col.dtype))
        return
    if isinstance(col, StructColumn):
        has_valid = col.valid is not None
        vleaf = None
        if has_valid:
            vleaf = len(leaves)
            leaves.append(_Leaf("valid_only", "boolean", col))
        sub = []
        for c in col.children:
            _flatten(c, leaves, sub)
        spec.append(("struct", col.names, col.is_map, col.dtype, vleaf, sub))
        return
    if isinstance(col, ArrayColumn):
        has_valid = col.valid is not None
        vleaf = None
        if has_valid:
            vleaf = len(leaves)
            leaves.append(_Leaf("valid_only", "boolean", col))
        sub = []
        for c in col.elements:
            _flatten(c, leaves, sub)
        spec.append(("array", col.drop_nulls, vleaf, sub))
        return
    if isinstance(col, StrColumn):
        spec.append(("str", len(leaves), type(col), col.dtype))
        leaves.append(_Leaf("str", col.dtype, col))
        return
    if isinstance(col, PrimColumn):
        spec.append(("prim", len(leaves), col.dtype))
        lf = _Leaf("prim", col.dtype, col)
        lf.torch_dtype = col.data.dtype
        leaves.append(lf)
        return
    raise TypeError(f"cannot exchange column {col!r}")


def _rebuild(spec_item, leaves_out, n, device):
    from ..engine.column import ArrayColumn, ConstColumn, PrimColumn, StrColumn, StructColumn
    kind = spec_item[0]
    if kind == "const":
        return ConstColumn(spec_item[1], spec_item[2], n, device)
    if kind == "prim" or kind == "str":
        return leaves_out[spec_item[1]]
    if kind == "struct":
        _, names, is_map, dtype, vleaf, sub = spec_item
        kids = [_rebuild(s, leaves_out, n, device) for s in sub]
        valid = leaves_out[vleaf] if vleaf is not None else None
        return StructColumn(names, kids, n, valid, is_map, dtype, device)
    if kind == "array":
        _, drop, vleaf, sub = spec_item
        els = [_rebuild(s, leaves_out, n, device) for s in sub]
        valid = leaves_out[vleaf] if vleaf is not None else None
        return ArrayColumn(els, n, valid, drop, device)
    raise ValueError(kind)


def split_by_destination(dest: torch.Tensor, world: int):
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=world).to(torch.int64)
    return order, counts


def shuffle_table(table, dest: torch.Tensor):
    """Send row i to rank dest[i]; returns the rows this rank receives (in source-rank order).

    One host synchronisation per exchange: the row count and every string leaf's byte count per destination are
    computed on the device as one [W, 1 + S] matrix, exchanged with one all-to-all, and read back together with
    the send side; every later collective (the int64 row matrix, one byte stream per string leaf) has its sizes
    from that single read-back."""
    from ..engine.column import PrimColumn, StrColumn, Table
    from ..ops import strings as sops
    W = _w()
    device = table.device
    n = table.length
    dest = dest.to(torch.int64)
    order, counts = split_by_destination(dest, W)
    t = table.take(order)
    sorted_dest = dest[order]
    leaves: List[_Leaf] = []
    spec: list = []
    for c in t.columns:
        _flatten(c, leaves, spec)
    # matrix columns
    mats = []
    nvalid = 0
    str_leaves = []
    for li, lf in enumerate(leaves):
        c = lf.col
        if lf.kind == "prim":
            d = c.data
            if d.dtype == torch.float64:
                d = d.view(torch.int64)
            elif d.dtype != torch.int64:
                d = d.to(torch.int64)
            lf.mcol = len(mats)
            mats.append(d)
        elif lf.kind == "str":
            lf.mcol = len(mats)
            mats.append(c.lens.to(torch.int64))
            str_leaves.append(li)
        if c.valid is not None:
            lf.vbit = nvalid
            nvalid += 1
    nmask = (nvalid + 62) // 63
    masks = [torch.zeros(n, dtype=torch.int64, device=device) for _ in range(nmask)]
    for lf in leaves:
        if lf.vbit >= 0:
            w, b = divmod(lf.vbit, 63)
            masks[w] |= lf.col.valid.to(torch.int64) << b
    mat_cols = mats + masks
    C = len(mat_cols)
    # [W, 1 + S] send sizes: rows, then bytes of each string leaf, per destination (device side)
    size_cols = [counts]
    for li in str_leaves:
        by_dest = torch.zeros(W, dtype=torch.int64, device=device)
        if n:
            by_dest.index_add_(0, sorted_dest, mats[leaves[li].mcol])
        size_cols.append(by_dest)
    send_sizes = torch.stack(size_cols, 1).contiguous()
    recv_sizes = _a2a_counts(send_sizes)
    both = torch.stack([send_sizes, recv_sizes]).tolist()            # the exchange's one host sync
    send_rows = [r[0] for r in both[0]]
    recv_rows = [r[0] for r in both[1]]
    n_out = sum(recv_rows)
    if C:
        send = torch.stack(mat_cols, 1).contiguous() if n else torch.empty((0, C), dtype=torch.int64, device=device)
        recv = torch.empty((n_out, C), dtype=torch.int64, device=device)
        _a2a(recv, send, recv_rows, send_rows)
    else:
        recv = torch.empty((n_out, 0), dtype=torch.int64, device=device)
    # string bytes: rows are already grouped by destination, so each leaf's packed bytes are too
    str_out = {}
    for si, li in enumerate(str_leaves):
        lf = leaves[li]
        send_bytes = [r[1 + si] for r in both[0]]
        recv_bytes = [r[1 + si] for r in both[1]]
        sc = sops.compact_known(lf.col, sum(send_bytes))
        total = sum(recv_bytes)
        out = torch.zeros(total + 16, dtype=torch.uint8, device=device)
        _a2a(out[:total], sc.arena[:sum(send_bytes)].contiguous(), recv_bytes, send_bytes)
        rlens = recv[:, lf.mcol]
        starts = torch.cumsum(rlens, 0) - rlens
        str_out[li] = (out, starts, rlens.to(torch.int32))
    # rebuild leaves
    leaves_out = {}
    for li, lf in enumerate(leaves):
        valid = None
        if lf.vbit >= 0:
            w, b = divmod(lf.vbit, 63)
            valid = ((recv[:, len(mats) + w] >> b) & 1).to(torch.bool)
        if lf.kind == "prim":
            d = recv[:, lf.mcol].contiguous()
            if lf.torch_dtype == torch.float64:
                d = d.view(torch.float64)
            elif lf.torch_dtype == torch.bool:
                d = d.to(torch.bool)
            leaves_out[li] = PrimColumn(lf.dtype, d, valid)
        elif lf.kind == "str":
            arena, starts, lens = str_out[li]
            leaves_out[li] = type(lf.col)(arena, starts, lens, valid, lf.col.dtype)
        else:   # valid_only
            leaves_out[li] = valid if valid is not None else None
    cols = [_rebuild(s, leaves_out, n_out, device) for s in spec]
    out = Table(t.names, cols, n_out, device)
    return out


def _broadcast(t: torch.Tensor, src: int) -> None:
    if _staged(t):
        h = t.cpu()
        dist.broadcast(h, src=src, group=_g())
        t.copy_(h)
    else:
        dist.broadcast(t, src=src, group=_g())


def broadcast_bytes(data: bytes, src: int = 0) -> bytes:
    """``data`` from rank ``src`` on every rank: one broadcast of the length, one of the bytes (a device buffer over
    RCCL when the ranks own GPUs — xGMI moves it; host memory over gloo)."""
    from . import _DEVICE, _RANK
    dev = _DEVICE if (_DEVICE is not None and dist.get_backend(_g()) != "gloo") else torch.device("cpu")
    n = torch.tensor([len(data) if _RANK == src else 0], dtype=torch.int64, device=dev)
    _broadcast(n, src)
    size = int(n.item())
    if _RANK == src:
        buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev) if size else \
            torch.empty(0, dtype=torch.uint8, device=dev)
    else:
        buf = torch.empty(size, dtype=torch.uint8, device=dev)
    if size:
        _broadcast(buf, src)
    return data if _RANK == src else buf.cpu().numpy().tobytes()


def broadcast_tensor(t: Optional[torch.Tensor], src: int = 0, dtype=torch.uint8, device=None) -> torch.Tensor:
    """A 1-D tensor from rank ``src`` on every rank (others pass None): length, then data — two collectives."""
    from . import _RANK
    dev = torch.device(device) if device is not None else (t.device if t is not None else torch.device("cpu"))
    n = torch.tensor([t.numel() if _RANK == src else 0], dtype=torch.int64, device=dev)
    _broadcast(n, src)
    out = t.contiguous() if _RANK == src else torch.empty(int(n.item()), dtype=dtype, device=dev)
    if out.numel():
        _broadcast(out, src)
    return out


def allgather_table(table):
    """Every rank receives the concatenation of all ranks' rows (rank order)."""
    from ..engine.column import Table
    W = _w()
    if W <= 1:
        return table
    n = table.length
    idx = torch.arange(n, device=table.device).repeat(W)
    dest = torch.arange(W, device=table.device).repeat_interleave(n)
    return shuffle_table(table.take(idx), dest)


def _pack(table):
    """Flatten a table for a collective: (spec, leaves, [n, C] int64 matrix, {leaf: compacted string bytes})."""
    from ..ops import strings as sops
    device = table.device
    n = table.length
    leaves: List[_Leaf] = []
    spec: list = []
    for c in table.columns:
        _flatten(c, leaves, spec)
    mats, nvalid = [], 0
    strs = {}
    for li, lf in enumerate(leaves):
        c = lf.col
        if lf.kind == "prim":
            d = c.data
            d = d.view(torch.int64) if d.dtype == torch.float64 else (d if d.dtype == torch.int64 else d.to(torch.int64))
            lf.mcol = len(mats)
            mats.append(d)
        elif lf.kind == "str":
            lf.mcol = len(mats)
            mats.append(c.lens.to(torch.int64))
            total = int(c.lens.to(torch.int64).sum().item()) if n else 0
            strs[li] = sops.compact_known(c, total).arena[:total].contiguous() if n else \
                torch.empty(0, dtype=torch.uint8, device=device)
        if c.valid is not None:
            lf.vbit = nvalid
            nvalid += 1
    masks = [torch.zeros(n, dtype=torch.int64, device=device) for _ in range((nvalid + 62) // 63)]
    for lf in leaves:
        if lf.vbit >= 0:
            w, b = divmod(lf.vbit, 63)
            masks[w] |= lf.col.valid.to(torch.int64) << b
    cols = mats + masks
    mat = torch.stack(cols, 1).contiguous() if (cols and n) else torch.empty((n, len(cols)), dtype=torch.int64,
                                                                              device=device)
    return spec, leaves, mat, strs, len(mats)


def _leaf_meta(leaves):
    """Picklable per-leaf layout (what a receiver needs to rebuild columns it has never seen)."""
    return [(lf.kind, lf.dtype, lf.mcol, lf.vbit, lf.torch_dtype,
             type(lf.col) if lf.kind == "str" else None, getattr(lf.col, "dtype", None)) for lf in leaves]


def _unpack(table_names, spec, meta, mat, strs, nmats, device):
    from ..engine.column import PrimColumn, Table
    n = int(mat.shape[0])
    out = {}
    for li, (kind, dtype, mcol, vbit, tdt, scls, cdt) in enumerate(meta):
        valid = None
        if vbit >= 0:
            w, b = divmod(vbit, 63)
            valid = ((mat[:, nmats + w] >> b) & 1).to(torch.bool)
        if kind == "prim":
            d = mat[:, mcol].contiguous()
            if tdt == torch.float64:
                d = d.view(torch.float64)
            elif tdt == torch.bool:
                d = d.to(torch.bool)
            elif tdt is not None and tdt != torch.int64:
                d = d.to(tdt)
            out[li] = PrimColumn(dtype, d, valid)
        elif kind == "str":
            lens = mat[:, mcol]
            starts = torch.cumsum(lens, 0) - lens
            arena = torch.zeros(int(strs[li].shape[0]) + 16, dtype=torch.uint8, device=device)
            arena[:strs[li].shape[0]] = strs[li]
            out[li] = scls(arena, starts, lens.to(torch.int32), valid, cdt)
        else:
            out[li] = valid
    return Table(table_names, [_rebuild(sp, out, n, device) for sp in spec], n, device)


def broadcast_table(table, src: int = 0):
    """Rank ``src``'s table on every rank (the others pass any table with the same column names, e.g. empty): the
    layout travels as one small object broadcast, the data as one broadcast of the packed [rows × C] int64 matrix
    plus one per string leaf's bytes — the source sends each byte once (ncclBroadcast's pipelined ring/tree over
    xGMI), never W copies."""
    from . import _RANK
    W = _w()
    if W <= 1:
        return table
    device = table.device
    if _RANK == src:
        spec, leaves, mat, strs, nmats = _pack(table)
        layout = [spec, _leaf_meta(leaves), nmats, int(mat.shape[0]), int(mat.shape[1]), sorted(strs)]
    else:
        layout, mat, strs = [None] * 6, None, {}
    obj = [layout]
    dist.broadcast_object_list(obj, src=src, group=_g())
    spec, meta, nmats, rows, C, str_ids = obj[0]
    flat = broadcast_tensor(mat.reshape(-1) if _RANK == src else None, src, torch.int64, device)
    mat = flat.reshape(rows, C)
    got = {li: broadcast_tensor(strs[li] if _RANK == src else None, src, torch.uint8, device) for li in str_ids}
    out = _unpack(table.names, spec, meta, mat, got, nmats, device)
    out.dist = P_REPLICATED
    return out


P_REPLICATED = "replicated"


def rebalance_table(table):
    """Round-robin full shuffle: global row g goes to rank g % W, so every rank ends up with an equal share of the
    batch however skewed the source partitions were (the reference's optional input ``rdd.repartition(n)``,
    DataProcessing/datax-host/src/main/scala/datax/host/StreamingHost.scala:68-69).  One all-gather of row counts
    gives each rank its global row offset; the rows move in one all-to-all (``shuffle_table``)."""
    from . import _RANK
    W = _w()
    if W <= 1:
        return table
    device = table.device
    n = table.length
    counts = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(W)]
    _all_gather(counts, torch.tensor([n], dtype=torch.int64, device=device))
    offset = int(sum(torch.cat(counts).tolist()[:_RANK]))          # one host read-back
    dest = (torch.arange(n, dtype=torch.int64, device=device) + offset) % W
    return shuffle_table(table, dest)
