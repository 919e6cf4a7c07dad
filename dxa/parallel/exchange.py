"""Row exchange between ranks over RCCL (xGMI) / gloo: variable-size all-to-all of columnar tables.

A table is flattened into (a) one [rows × C] int64 matrix — every fixed-width leaf becomes one column (doubles
bit-cast, booleans widened), every string leaf contributes its byte lengths, validity travels as 63-bit masks — and
(b) one byte stream per string leaf.  Rows are stably sorted by destination so each destination's block is
contiguous; a single ``all_to_all_single`` moves the matrix, one more moves the bytes of every string leaf (one
destination-major buffer), and one tiny one the counts — three collectives per exchange whatever the column count.  Sized for xGMI: all blocks of a rank leave in one collective, so the 7 links are driven concurrently and the
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
# table collectives (wire format: dxa.parallel.packing)
# ---------------------------------------------------------------------------------------------------------------

def split_by_destination(dest: torch.Tensor, world: int):
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=world).to(torch.int64)
    return order, counts


def _force_torch() -> bool:
    """The torch reference implementation of the exchange wire format runs only where the device kernels cannot
    (CPU tensors); ``packing`` picks it by device, this flag never forces it on a GPU."""
    return False


def shuffle_table(table, dest: torch.Tensor):
    """Send row i to rank dest[i]; returns the rows this rank receives (in source-rank order).

    Device path (``exchange.hip``): plan (histogram + scan: the [W × (1+S)] send sizes) → one all-to-all of the
    sizes and ONE host read-back of sent and received sizes → scatter (matrix + string arenas, destination-ordered)
    → one all-to-all of the matrix and ONE of every string leaf's bytes (coalesced, destination-major) → one
    unpack launch.  Three kernel launches on the send
    side and one on the receive side, however many columns the table has."""
    from . import packing as PK
    W = _w()
    device = table.device
    lay = PK.Layout(table)
    # the per-leaf "has validity" flags ride along with the sizes (written by the plan's scan kernel): every rank
    # ORs what it receives, so all ranks agree on the matrix layout without another collective
    ext, state = PK.plan(lay, dest.to(torch.int64), W, _force_torch(), extra=lay.flags())
    recv_sizes = _a2a_counts(ext)
    both = torch.stack([ext, recv_sizes]).tolist()              # the exchange's one host sync
    lay.assign_flags(_or_rows([r[1 + lay.S:] for r in both[1]]))
    send_rows = [r[0] for r in both[0]]
    recv_rows = [r[0] for r in both[1]]
    send_bytes = [[r[1 + s] for r in both[0]] for s in range(lay.S)]
    recv_bytes = [[r[1 + s] for r in both[1]] for s in range(lay.S)]
    mat, arenas = PK.scatter(lay, state, send_rows, send_bytes, coalesce=True)
    n_out = sum(recv_rows)
    recv = torch.empty((n_out, lay.C), dtype=torch.int64, device=device)
    if lay.C:
        _a2a(recv, mat, recv_rows, send_rows)
    rarenas, byte_base = [], []
    if lay.S:
        # every string leaf in ONE byte all-to-all: destination-major blocks [leaf 0 | leaf 1 | …] per rank
        send_split, _ = PK.coalesced_bytes(send_bytes)
        recv_split, byte_base = PK.coalesced_bytes(recv_bytes)
        total = sum(recv_split)
        out = torch.zeros(total + 16, dtype=torch.uint8, device=device)      # +16: string kernels over-read
        _a2a(out[:total], arenas[0][:sum(send_split)], recv_split, send_split)
        rarenas = [out] * lay.S
    row_prefix = _prefix(recv_rows)
    return PK.unpack(lay.names, lay.spec, lay.meta(), recv, rarenas, row_prefix, row_prefix[:W], byte_base, n_out,
                     device, _force_torch())


def _or_rows(rows):
    out = [0] * len(rows[0])
    for r in rows:
        out = [a | int(b) for a, b in zip(out, r)]
    return out


def _prefix(xs):
    out = [0]
    for x in xs:
        out.append(out[-1] + int(x))
    return out


def _gsrc(src: int, g=None) -> int:
    """torch.distributed takes a broadcast's source as a GLOBAL rank; ``src`` is a rank of the communicator."""
    g = _g() if g is None else g
    if g is None or g == dist.group.WORLD:
        return src
    return dist.get_global_rank(g, src)


def _broadcast(t: torch.Tensor, src: int) -> None:
    if _staged(t):
        h = t.cpu()
        dist.broadcast(h, src=_gsrc(src), group=_g())
        t.copy_(h)
    else:
        dist.broadcast(t, src=_gsrc(src), group=_g())


def _all_gather_into(out: torch.Tensor, t: torch.Tensor) -> None:
    """``out`` = the ranks' equal-size ``t`` concatenated in rank order — ``all_gather_into_tensor`` over RCCL
    (one output buffer, no per-rank copies); a list all-gather over gloo."""
    W = _w()
    if not _staged(t) and dist.get_backend(_g()) != "gloo":
        dist.all_gather_into_tensor(out, t.contiguous(), group=_g())
        return
    parts = [torch.empty(t.shape, dtype=t.dtype) for _ in range(W)]
    dist.all_gather(parts, t.cpu(), group=_g())
    out.copy_(torch.cat(parts).to(out.device))


def broadcast_bytes(data: bytes, src: int = 0) -> bytes:
    """``data`` from rank ``src`` (a rank of the job's group) on every rank, as host bytes (small payloads:
    configuration, layouts).  Bulk payloads that end on the device use ``broadcast_device_bytes``."""
    from . import _RANK
    g = _gloo_or_default()
    gsrc = _gsrc(src, g)
    n = torch.tensor([len(data) if _RANK == src else 0], dtype=torch.int64)
    dist.broadcast(n, src=gsrc, group=g)
    size = int(n.item())
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8) if (_RANK == src and size) else \
        torch.empty(size, dtype=torch.uint8)
    if size:
        dist.broadcast(buf, src=gsrc, group=g)
    return data if _RANK == src else buf.numpy().tobytes()


def _gloo_or_default():
    """Host-tensor broadcasts need a gloo communicator; with RCCL as the job's backend that is the host group
    ``parallel.init`` created on every rank (same ranks as the job's group)."""
    g = _g()
    if dist.get_backend(g) == "gloo":
        return g
    if _HOST_GROUP is None:
        raise RuntimeError("broadcast_bytes under RCCL needs parallel.init() (it creates the host group)")
    return _HOST_GROUP


_HOST_GROUP = None


def broadcast_device_bytes(data: Optional[bytes], src: int, device, pad: int = 64) -> Tuple[torch.Tensor, int]:
    """A byte payload from rank ``src`` as a device buffer on every rank → (buffer of length + ``pad`` zeroed
    bytes, length).  The source copies its bytes to the device once (pinned staging) and the RCCL broadcast moves
    them over xGMI straight into every receiver's HBM: receivers never stage the payload in host memory (SURVEY
    §2.G X3 — a 100 M-row reference table's CSV crosses each receiver's PCIe link zero times).  Over gloo (CPU
    ranks) the buffer is a host tensor."""
    from . import _RANK
    device = torch.device(device)
    n = torch.tensor([len(data) if _RANK == src else 0], dtype=torch.int64, device=device)
    _broadcast(n, src)
    size = int(n.item())
    if _RANK == src:
        if device.type == "cuda":
            host = torch.empty(size + pad, dtype=torch.uint8, pin_memory=True)
            host[size:].zero_()
            if size:
                host[:size] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
            buf = host.to(device, non_blocking=True)
            buf.record_stream(torch.cuda.current_stream(device))
        else:
            buf = torch.zeros(size + pad, dtype=torch.uint8)
            if size:
                buf[:size] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    else:
        buf = torch.zeros(size + pad, dtype=torch.uint8, device=device)
    if size:
        _broadcast(buf[:size], src) if not _staged(buf) else _broadcast_staged_slice(buf, size, src)
    return buf, size


def _broadcast_staged_slice(buf, size, src):
    h = buf[:size].cpu()
    dist.broadcast(h, src=_gsrc(src), group=_g())
    buf[:size].copy_(h)


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
    """Every rank receives the concatenation of all ranks' rows (rank order).

    The table is packed once (identity order), the per-rank sizes are all-gathered (the one host read-back), and
    the matrix and the string bytes (every leaf in one buffer) travel with one ``all_gather_into_tensor`` each,
    padded to the largest rank's share: the receive buffer is W × the largest share — the result's size for balanced ranks — and no rank
    ever materialises W copies of its own rows.  One unpack launch reads the padded buffers in place (strings stay
    views into the gathered arenas)."""
    from . import packing as PK
    from ..engine.column import Table
    W = _w()
    if W <= 1:
        return table
    device = table.device
    lay = PK.Layout(table)
    # [1, 1+S+F]: rows, bytes per string leaf, then the validity flags
    ext, state = PK.plan(lay, None, 1, _force_torch(), extra=lay.flags())
    allsz = torch.empty((W, ext.shape[1]), dtype=torch.int64, device=device)
    _all_gather_into(allsz, ext)
    got = allsz.tolist()                                           # the one host sync
    lay.assign_flags(_or_rows([r[1 + lay.S:] for r in got]))      # the ranks' agreed validity layout
    rows = [r[0] for r in got]
    bts = [[r[1 + s] for r in got] for s in range(lay.S)]
    maxr = max(rows)
    me = _rank()
    # every string leaf's bytes in one buffer per rank ([leaf 0 | leaf 1 | …]), padded to the largest rank's total:
    # one all-gather moves them all
    tot = [sum(bts[s][k] for s in range(lay.S)) for k in range(W)]
    maxb = max(tot) if lay.S else 0
    mat, arenas = PK.scatter(lay, state, [lay.n], [[bts[s][me]] for s in range(lay.S)], rows_alloc=maxr,
                             bytes_alloc=[maxb], coalesce=True)
    n_out = sum(rows)
    gm = torch.empty((W * maxr, lay.C), dtype=torch.int64, device=device)
    if lay.C and maxr:
        _all_gather_into(gm, mat[:maxr])
    gar, byte_base = [], [[0] * W for _ in range(lay.S)]
    if lay.S:
        ga = torch.zeros(W * maxb + 16, dtype=torch.uint8, device=device)
        if maxb:
            _all_gather_into(ga[:W * maxb], arenas[0][:maxb])
        gar = [ga] * lay.S
        for k in range(W):
            pos = k * maxb
            for s in range(lay.S):
                byte_base[s][k] = pos
                pos += bts[s][k]
    out = PK.unpack(lay.names, lay.spec, lay.meta(), gm, gar, _prefix(rows), [k * maxr for k in range(W)],
                    byte_base, n_out, device, _force_torch())
    return Table(out.names, out.columns, out.length, device)


def _rank():
    from . import _RANK
    return _RANK


def broadcast_table(table, src: int = 0):
    """Rank ``src``'s table on every rank (the others pass any table with the same column names, e.g. empty): the
    layout travels as one small object broadcast, the data as one broadcast of the packed [rows × C] int64 matrix
    plus one of every string leaf's bytes — the source sends each byte once (ncclBroadcast's pipelined ring/tree over
    xGMI), never W copies."""
    from . import packing as PK
    from . import _RANK
    W = _w()
    if W <= 1:
        return table
    device = table.device
    if _RANK == src:
        lay = PK.Layout(table)
        sizes, state = PK.plan(lay, None, 1, _force_torch())
        szl = sizes.tolist()[0]
        mat, arenas = PK.scatter(lay, state, [lay.n], [[szl[1 + s]] for s in range(lay.S)], coalesce=True)
        layout = [lay.spec, lay.meta(), lay.n, lay.C, [int(szl[1 + s]) for s in range(lay.S)]]
    else:
        layout, mat, arenas = None, None, None
    obj = [layout]
    dist.broadcast_object_list(obj, src=_gsrc(src), group=_g())
    spec, meta, rows, C, nbytes = obj[0]
    if _RANK != src:
        mat = torch.empty((rows, C), dtype=torch.int64, device=device)
    if rows and C:
        _broadcast(mat, src)
    # every string leaf's bytes in one broadcast ([leaf 0 | leaf 1 | …])
    nb = sum(nbytes)
    buf = torch.zeros(nb + 16, dtype=torch.uint8, device=device)
    if _RANK == src and nb:
        buf[:nb] = arenas[0][:nb]
    if nb:
        if _staged(buf):
            _broadcast_staged_slice(buf, nb, src)
        else:
            _broadcast(buf[:nb], src)
    got = [buf] * len(nbytes)
    out = PK.unpack(table.names, spec, meta, mat, got, [0, rows], [0], [[sum(nbytes[:s])] for s in range(len(nbytes))],
                    rows, device, _force_torch())
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


def _h2d(data, dtype, device):
    from ..ops.native import h2d
    return h2d(data, dtype, device)
