"""Kafka / Event Hubs record batches decoded on the GPU.

The host path (``dxa.io.kafka.decode_records``) decompresses and frames records in C++, which caps a source at a
few GB/s of JSON per process.  Here the host only walks batch and LZ4-frame headers (``dxa_kafka_plan``: no record
bytes are touched), the Fetch bytes go to HBM as they arrived from the broker (compressed), and the GPU
decompresses every LZ4 block (``lz4.hip``, 16 lanes per block, capacity slots because Kafka frames carry no
content size) and frames the records (``kafka_records.hip``).  The JSON parser then reads each record's value in
place through per-record [start, end) ranges — the bytes cross PCIe once, compressed, and are never copied on the
device.

gzip batches (codec 1, the Event Hubs Kafka endpoint's codec) are inflated on the GPU too (``inflate.hip``: the
planner strips the gzip header and takes the size from the ISIZE trailer), snappy batches (codec 2: snappy-java's
xerial stream split into its raw blocks, exact sizes from their preambles) by ``snappy.hip`` and zstd batches
(codec 4: one frame per batch, a capacity slot of blocks x block maximum, size reported by the kernel) by
``zstd.hip``.  Batches the GPU path does not take (dependent-block LZ4 frames, zstd dictionaries, compacted
batches with offset gaps) make ``plan_fetch`` raise ``Unsupported``; the source then decodes that fetch on the
host.
CRC-32C (the consumer's ``check.crcs``, on by default) is verified by the host planner (SSE4.2 ``crc32``, ~8 GB/s
per planner thread) or, with ``DeviceRecordDecoder(verify_crc=True)``, on the GPU over the compressed bytes already
in HBM (``kafka_crc_kernel``: one wave per batch, lane-interleaved words combined in GF(2)).  Measured on MI355X
(profiles/crc/README.md): the GPU check takes ~0.6 ms per 441 MB batch but steals LDS and CU time from the LZ4
decode, which is the pipeline's critical path, costing ~20 % of the groupby rate, while the host check is free at
one GPU — so the host is the default and the device check is the option for CPU-starved hosts.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

_PLAN_ERRS = {-2: "message format is not v2", -3: "CRC mismatch", -5: "codec decoded on the host only",
              -7: "malformed compressed payload (LZ4 / snappy / zstd)", -8: "dependent-block LZ4 frame", -9: "offset deltas with gaps"}


TORCH_DT = {np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64, np.dtype(np.uint8): torch.uint8}


class Unsupported(Exception):
    """The fetch needs the host decoder."""


_BOUND = False


def _lib():
    global _BOUND
    from ..ops.serialize import lib
    L = lib()
    if not _BOUND:
        p, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        L.dxa_kafka_plan.argtypes = [p, i64, i64, i32, p, p] + [p] * 14
        L.dxa_kafka_plan.restype = ctypes.c_int
        _BOUND = True
    return L


@dataclass
class FetchPlan:
    """Host-side plan of one or more Fetch record sets laid out back to back in one staging buffer."""
    b_count: np.ndarray           # int32 [nbat] records in the batch
    b_base: np.ndarray            # int64 [nbat] base offset
    b_skip: np.ndarray            # int32 [nbat] leading records below the fetch offset
    b_keep: np.ndarray            # int32 [nbat] records emitted after the skipped ones
    b_first: np.ndarray           # int32 [nbat] first block
    b_nblk: np.ndarray            # int32 [nbat]
    b_rec0: np.ndarray            # int64 [nbat] index of the batch's first emitted record
    k_comp_off: np.ndarray        # int64 [nblk] block payload offset in the staging buffer
    k_comp_len: np.ndarray        # int32 [nblk]
    k_stored: np.ndarray          # uint8 [nblk]
    k_out_off: np.ndarray         # int64 [nblk] output slot
    k_cap: np.ndarray             # int64 [nblk] slot capacity
    out_bytes: int
    next_offset: int
    nbytes: int = 0               # staging bytes covered
    packed: Optional[torch.Tensor] = None      # pinned bytes holding every array above (one H2D copy), if any
    layout: Optional[list] = None              # [(name, byte offset, count)] of the arrays inside ``packed``
    b_crc_off: Optional[np.ndarray] = None     # int64 [nbat] CRC-covered range start (attributes) in the staging
    b_crc_len: Optional[np.ndarray] = None     # int32 [nbat] CRC-covered length
    b_crc: Optional[np.ndarray] = None         # int32 [nbat] stored CRC-32C (bits)

    def __post_init__(self):
        n = int(self.b_count.shape[0])
        for name, dt in (("b_crc_off", np.int64), ("b_crc_len", np.int32), ("b_crc", np.int32)):
            if getattr(self, name) is None:
                setattr(self, name, np.zeros(n, dt))

    @property
    def nbat(self) -> int:
        return int(self.b_count.shape[0])

    @property
    def nblk(self) -> int:
        return int(self.k_comp_off.shape[0])

    @property
    def nrec(self) -> int:
        return int(self.b_keep.sum()) if self.nbat else 0

    def last_offsets(self) -> np.ndarray:
        """Kafka offset of the last emitted record of each batch (for commit ranges)."""
        return self.b_base + self.b_skip + self.b_keep - 1


def plan_fetch(data, min_offset: int, verify_crc: bool = True) -> FetchPlan:
    """Plan one Fetch record set (bytes / uint8 ndarray) → FetchPlan (offsets relative to ``data``).
    ``verify_crc``: check every batch's CRC-32C here on the host (False: left to the device, or not checked)."""
    a = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    L = _lib()
    counts = np.zeros(5, dtype=np.int64)
    nxt = ctypes.c_int64(0)
    rc = L.dxa_kafka_plan(a.ctypes.data, a.size, min_offset, int(verify_crc), counts.ctypes.data,
                          ctypes.byref(nxt), *([None] * 14))
    if rc:
        raise Unsupported(_PLAN_ERRS.get(rc, f"plan error {rc}"))
    nbat, nblk = int(counts[0]), int(counts[1])
    arr = dict(b_count=np.zeros(nbat, np.int32), b_base=np.zeros(nbat, np.int64),
               b_skip=np.zeros(nbat, np.int32), b_first=np.zeros(nbat, np.int32), b_nblk=np.zeros(nbat, np.int32),
               b_rec0=np.zeros(nbat, np.int64), k_comp_off=np.zeros(nblk, np.int64),
               k_comp_len=np.zeros(nblk, np.int32), k_stored=np.zeros(nblk, np.uint8),
               k_out_off=np.zeros(nblk, np.int64), k_cap=np.zeros(nblk, np.int64),
               b_crc_off=np.zeros(nbat, np.int64), b_crc_len=np.zeros(nbat, np.int32), b_crc=np.zeros(nbat, np.int32))
    order = ["b_count", "b_base", "b_skip", "b_first", "b_nblk", "b_rec0", "k_comp_off", "k_comp_len", "k_stored",
             "k_out_off", "k_cap", "b_crc_off", "b_crc_len", "b_crc"]
    rc = L.dxa_kafka_plan(a.ctypes.data, a.size, min_offset, int(verify_crc), counts.ctypes.data,
                          ctypes.byref(nxt), *[arr[k].ctypes.data for k in order])
    if rc:
        raise Unsupported(_PLAN_ERRS.get(rc, f"plan error {rc}"))
    keep = (arr["b_count"] - arr["b_skip"]).astype(np.int32)
    return FetchPlan(b_keep=keep, out_bytes=int(counts[3]), next_offset=nxt.value, nbytes=int(a.size), **arr)


_ARRAYS = [("b_count", np.int32, "b"), ("b_base", np.int64, "b"), ("b_skip", np.int32, "b"),
           ("b_keep", np.int32, "b"), ("b_first", np.int32, "b"), ("b_nblk", np.int32, "b"),
           ("b_rec0", np.int64, "b"), ("k_comp_off", np.int64, "k"), ("k_comp_len", np.int32, "k"),
           ("k_stored", np.uint8, "k"), ("k_out_off", np.int64, "k"), ("k_cap", np.int64, "k"),
           ("b_crc_off", np.int64, "b"), ("b_crc_len", np.int32, "b"), ("b_crc", np.int32, "b")]


class PlanBuffer:
    """Reusable pinned buffer the multi-set planner writes its arrays into (no per-step pinned allocation).
    ``busy`` is the event of the last H2D copy out of it; see ``PlanBufferPool``."""

    def __init__(self):
        self.buf: Optional[torch.Tensor] = None
        self.busy = None
        self.reserved = False          # handed out by a pool, its plan not yet consumed

    def free(self) -> bool:
        return not self.reserved and (self.busy is None or self.busy.query())

    def release(self, event=None):
        """The plan is consumed: the buffer is free once ``event`` (its H2D copy) completes."""
        self.busy = event
        self.reserved = False

    def carve(self, nbat: int, nblk: int):
        layout, pos = [], 0
        for name, dt, kind in _ARRAYS:
            cnt = nbat if kind == "b" else nblk
            layout.append((name, pos, cnt))
            pos += (cnt * np.dtype(dt).itemsize + 15) // 16 * 16
        if self.buf is None or self.buf.numel() < pos:
            self.buf = torch.empty(max(pos, 1) * 5 // 4 + 64, dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        raw = self.buf.numpy()
        arrs = {name: raw[off:off + cnt * np.dtype(dt).itemsize].view(dt)
                for (name, off, cnt), (_, dt, _k) in zip(layout, _ARRAYS)}
        return arrs, layout, pos


class PlanBufferPool:
    """Plan buffers for pipelined ingest: a buffer is reused only once the copy of its previous plan is done."""

    def __init__(self):
        self.bufs: List[PlanBuffer] = []
        self._lock = __import__("threading").Lock()

    def get(self) -> PlanBuffer:
        with self._lock:
            for b in self.bufs:
                if b.free():
                    b.reserved = True
                    return b
            b = PlanBuffer()
            b.reserved = True
            self.bufs.append(b)
            return b


def plan_many(data: np.ndarray, bounds: Sequence[Tuple[int, int]], min_offsets: Sequence[int],
              threads: int = 16, buffer: Optional[PlanBuffer] = None, verify_crc: bool = True) -> FetchPlan:
    """Plan many record sets of one staging buffer (``data[lo:hi]`` each, one per partition fetch) with the sets
    walked in parallel native threads; the merged arrays land in ``buffer`` (pinned) for one H2D copy.
    ``verify_crc`` checks every record batch's CRC-32C here on the host (SSE4.2 ``crc32`` in host_kafka.cpp, in the
    planner threads); False leaves it to the device decode (``DeviceRecordDecoder(verify_crc=True)``) or skips it."""
    L = _lib()
    if not hasattr(L, "_plan_many_bound"):
        p, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        L.dxa_kafka_plan_count.argtypes = [p, i64, p, p, p, i32, i32, p, p]
        L.dxa_kafka_plan_fill.argtypes = [p, i64, p, p, p, i32, p] + [p] * 14
        L._plan_many_bound = True
    ns = len(bounds)
    so = np.array([b[0] for b in bounds], np.int64)
    sl = np.array([b[1] - b[0] for b in bounds], np.int64)
    mo = np.array(list(min_offsets), np.int64)
    counts = np.zeros((ns, 4), np.int64)
    nxt = np.zeros(ns, np.int64)
    rc = L.dxa_kafka_plan_count(data.ctypes.data, ns, so.ctypes.data, sl.ctypes.data, mo.ctypes.data,
                                int(verify_crc), threads,
                                counts.ctypes.data, nxt.ctypes.data)
    if rc:
        raise Unsupported(_PLAN_ERRS.get(rc, f"plan error {rc}"))
    nbat, nblk = int(counts[:, 0].sum()), int(counts[:, 1].sum())
    buffer = buffer or PlanBuffer()
    arrs, layout, used = buffer.carve(nbat, nblk)
    rc = L.dxa_kafka_plan_fill(data.ctypes.data, ns, so.ctypes.data, sl.ctypes.data, mo.ctypes.data, threads,
                               counts.ctypes.data, *[arrs[n].ctypes.data for n in
                                                     ("b_count", "b_base", "b_skip", "b_first", "b_nblk", "b_rec0",
                                                      "k_comp_off", "k_comp_len", "k_stored", "k_out_off",
                                                      "k_cap", "b_crc_off", "b_crc_len", "b_crc")])
    if rc:
        raise Unsupported(_PLAN_ERRS.get(rc, f"plan error {rc}"))
    np.subtract(arrs["b_count"], arrs["b_skip"], out=arrs["b_keep"])
    plan = FetchPlan(out_bytes=int(counts[:, 3].sum()), next_offset=int(nxt.max()) if ns else 0,
                     nbytes=int((so + sl).max()) if ns else 0, packed=buffer.buf[:used], layout=layout, **arrs)
    plan.buffer = buffer
    return plan


def merge(plans: Sequence[Tuple[FetchPlan, int]]) -> FetchPlan:
    """Concatenate plans of record sets staged at the given byte offsets of one buffer."""
    if not plans:
        return FetchPlan(*(np.zeros(0, t) for t in (np.int32, np.int64, np.int32, np.int32, np.int32, np.int32,
                                                      np.int64, np.int64, np.int32, np.uint8, np.int64, np.int64)),
                         out_bytes=0, next_offset=0)
    cat = lambda k: np.concatenate([getattr(p, k) for p, _ in plans])  # noqa: E731
    blk0, out0, rec0 = [], [], []
    nb = ob = nr = 0
    for p, _ in plans:
        blk0.append(nb)
        out0.append(ob)
        rec0.append(nr)
        nb += p.nblk
        ob += p.out_bytes
        nr += p.nrec
    return FetchPlan(
        b_count=cat("b_count"), b_base=cat("b_base"), b_skip=cat("b_skip"), b_keep=cat("b_keep"),
        b_first=np.concatenate([p.b_first + b for (p, _), b in zip(plans, blk0)]).astype(np.int32),
        b_nblk=cat("b_nblk"),
        b_rec0=np.concatenate([_rec0(p) + r for (p, _), r in zip(plans, rec0)]),
        k_comp_off=np.concatenate([p.k_comp_off + at for p, at in plans]),
        k_comp_len=cat("k_comp_len"), k_stored=cat("k_stored"),
        k_out_off=np.concatenate([p.k_out_off + o for (p, _), o in zip(plans, out0)]),
        k_cap=cat("k_cap"), out_bytes=ob, next_offset=plans[-1][0].next_offset,
        nbytes=max(at + p.nbytes for p, at in plans),
        b_crc_off=np.concatenate([p.b_crc_off + at for p, at in plans]), b_crc_len=cat("b_crc_len"),
        b_crc=cat("b_crc"))


def _rec0(p: FetchPlan) -> np.ndarray:
    """Emitted-record index of each batch's first record, from the keep counts (a trim may have changed them)."""
    if not p.nbat:
        return np.zeros(0, np.int64)
    c = np.cumsum(p.b_keep, dtype=np.int64)
    return c - p.b_keep


def trim(p: FetchPlan, max_records: int) -> FetchPlan:
    """Keep at most ``max_records`` records (a source's maxRate): later batches emit nothing, the batch at the cut
    emits its first records only.  ``next_offset`` becomes the first offset not emitted."""
    if p.nrec <= max_records:
        return p
    keep = p.b_keep.copy()
    cum = np.cumsum(keep, dtype=np.int64)
    cut = int(np.searchsorted(cum, max_records, side="left"))      # first batch reaching the limit
    before = int(cum[cut - 1]) if cut else 0
    keep[cut] = max_records - before
    keep[cut + 1:] = 0
    q = FetchPlan(**{**p.__dict__, "b_keep": keep.astype(np.int32)})
    q.b_rec0 = _rec0(q)
    q.next_offset = int(p.b_base[cut] + p.b_skip[cut] + keep[cut])
    return q


class DeviceRecordDecoder:
    """Staged Fetch bytes (pinned host) → device RawBatch of record values, on copy + decode streams.

    ``chunks`` splits the H2D copy of the compressed bytes at block boundaries so chunk k's copy overlaps chunk
    k-1's decode (as ``lz4.ChunkedIngest``) — but never below ``min_blocks_per_chunk`` LZ4 blocks per decode launch:
    each block is one serial sequence chain on 16 lanes, so a launch needs ~4 waves per SIMD of chains (CUs × 64
    blocks) to hide the chain's latency.  Small producer batches (26 records, ~77 K blocks per 2 M events) keep 4
    chunks; Java-producer-sized ones (batch.size 16 KiB compressed ≈ 84 records, ~24 K blocks) decode in one launch:
    4.4 ms per quarter-batch launch at 1.5 waves/SIMD, against ~the same for the whole batch at once."""

    def __init__(self, device, chunks: int = 4, copy_stream=None, decode_stream=None, track: bool = True,
                 verify_crc: bool = False):
        self.device = torch.device(device)
        self.verify_crc = verify_crc          # CRC-32C of every batch on the device (check.crcs)
        # the CRC check runs on its own stream, concurrently with the LZ4 decode (which is latency-bound and leaves
        # CUs idle); only the batch's status waits for it, never the consumer of the decoded records
        self.crc_stream = torch.cuda.Stream(self.device) if verify_crc else None
        self.chunks = max(1, chunks)
        cus = torch.cuda.get_device_properties(self.device).multi_processor_count
        self.min_blocks_per_chunk = cus * 64          # 4 SIMDs x 4 waves x 4 blocks (16-lane groups) per wave
        self.copy_stream = copy_stream or torch.cuda.Stream(self.device)
        self.decode_stream = decode_stream or torch.cuda.Stream(self.device)
        # per-batch DecodeStatus objects, drained by check(); ``track=False``: the caller checks each batch's
        # ``RawBatch.status`` itself (KafkaSource.verify) and nothing accumulates here
        self.track = track
        self.checks: List["DecodeStatus"] = []

    def decode(self, staging: torch.Tensor, plan: FetchPlan):
        """Returns (RawBatch, done_event).  ``staging`` is a pinned uint8 tensor holding the record sets at the
        plan's offsets (+32 readable bytes)."""
        from ..engine.processor import RawBatch
        from ..ops import native as N
        dev = self.device
        n = plan.nrec
        if plan.packed is None:                      # pack the arrays for one H2D copy
            if not hasattr(self, "_packs"):
                self._packs = PlanBufferPool()
            pb = self._packs.get()
            plan.buffer = pb
            arrs, layout, used = pb.carve(plan.nbat, plan.nblk)
            for name, _dt, _k in _ARRAYS:
                arrs[name][...] = getattr(plan, name)
            packed = pb.buf[:used]
        else:
            packed, layout = plan.packed, plan.layout
        with torch.cuda.stream(self.copy_stream):
            dtab = packed.to(dev, non_blocking=True)
            ddata = torch.empty(plan.nbytes + 32, dtype=torch.uint8, device=dev)
            tab_ev = torch.cuda.Event()
            tab_ev.record(self.copy_stream)
        if getattr(plan, "buffer", None) is not None:
            plan.buffer.release(tab_ev)
        views = {name: dtab[off:off + cnt * np.dtype(dt).itemsize].view(TORCH_DT[np.dtype(dt)])
                 for (name, off, cnt), (_, dt, _k) in zip(layout, _ARRAYS)}
        tabs = [views[k] for k in ("k_comp_off", "k_comp_len", "k_stored", "k_out_off", "k_cap", "b_count",
                                   "b_skip", "b_keep", "b_first", "b_nblk", "b_rec0")]
        crc_tabs = [views[k] for k in ("b_crc_off", "b_crc_len", "b_crc")]
        co, cl, sd, oo, cap, bc, bs, bk, bf, bn, br = tabs
        with torch.cuda.stream(self.decode_stream):
            out = torch.empty(plan.out_bytes + 64, dtype=torch.uint8, device=dev)
            produced = torch.empty(max(1, plan.nblk), dtype=torch.int64, device=dev)
            bstat = torch.empty(max(1, plan.nblk), dtype=torch.int32, device=dev)
            offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
            ends = torch.empty(max(1, n), dtype=torch.int64, device=dev)
            rstat = torch.empty(max(1, plan.nbat), dtype=torch.int32, device=dev)
        self.decode_stream.wait_event(tab_ev)
        st = self.decode_stream.cuda_stream
        nb = plan.nblk
        chunks = max(1, min(self.chunks, nb // max(1, self.min_blocks_per_chunk)))
        kinds = set(np.unique(plan.k_stored[:nb]).tolist()) if nb else set()
        has_gzip, has_snappy, has_zstd = 2 in kinds, 3 in kinds, 4 in kinds
        bounds = np.linspace(0, nb, chunks + 1).astype(np.int64)
        ev_last = tab_ev
        copied = 0                 # staging bytes already sent: chunks are contiguous from byte 0 (the batch headers
        for k in range(chunks):            # between blocks travel too — the device CRC check reads them)
            b0, b1 = int(bounds[k]), int(bounds[k + 1])
            if b1 <= b0:
                continue
            lo = copied
            hi = plan.nbytes if b1 == nb else int(plan.k_comp_off[b1])
            copied = hi
            N.call("dxa_memcpy_h2d_async", ddata.data_ptr() + lo, staging.data_ptr() + lo, hi - lo,
                   self.copy_stream.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
            ev_last = ev
            self.decode_stream.wait_event(ev)
            N.call("dxa_lz4_decode_into", N.ptr(ddata), N.ptr(co[b0:b1]), N.ptr(cl[b0:b1]), N.ptr(sd[b0:b1]),
                   N.ptr(oo[b0:b1]), N.ptr(cap[b0:b1]), b1 - b0, N.ptr(out), N.ptr(produced[b0:b1]),
                   N.ptr(bstat[b0:b1]), st)
            # the other codecs' entries of the chunk: gzip members (kind 2, inflate.hip), snappy raw blocks
            # (kind 3, snappy.hip), zstd frames (kind 4, zstd.hip); each kernel skips the kinds it does not own
            for present, entry in ((has_gzip, "dxa_inflate_into"), (has_snappy, "dxa_snappy_decode_into"),
                                   (has_zstd, "dxa_zstd_decode_into")):
                if present:
                    N.call(entry, N.ptr(ddata), N.ptr(co[b0:b1]), N.ptr(cl[b0:b1]), N.ptr(sd[b0:b1]),
                           N.ptr(oo[b0:b1]), N.ptr(cap[b0:b1]), b1 - b0, N.ptr(out), N.ptr(produced[b0:b1]),
                           N.ptr(bstat[b0:b1]), st)
        with torch.cuda.stream(self.decode_stream):
            offs[n:].fill_(plan.out_bytes)
        N.call("dxa_kafka_records", N.ptr(out), plan.nbat, N.ptr(bc), N.ptr(bs), N.ptr(bk), N.ptr(bf), N.ptr(bn),
               N.ptr(br), N.ptr(oo), N.ptr(cap), N.ptr(produced), N.ptr(bstat), N.ptr(offs), N.ptr(ends),
               N.ptr(rstat), st)
        done = torch.cuda.Event()
        done.record(self.decode_stream)
        if self.verify_crc:
            cs = self.crc_stream
            cs.wait_event(ev_last)                       # every staging byte is in HBM
            with torch.cuda.stream(cs):
                cstat = torch.empty(max(1, plan.nbat), dtype=torch.int32, device=dev)
            N.call("dxa_kafka_crc", N.ptr(ddata), plan.nbat, *[N.ptr(t) for t in crc_tabs], N.ptr(cstat),
                   cs.cuda_stream)
            cs.wait_event(done)
            with torch.cuda.stream(cs):
                bad = (rstat[:plan.nbat] != 0).sum() + (cstat[:plan.nbat] != 0).sum()
                status = DecodeStatus(bad, cs)
            for t in (ddata, dtab, rstat):
                t.record_stream(cs)
        else:
            with torch.cuda.stream(self.decode_stream):
                status = DecodeStatus((rstat[:plan.nbat] != 0).sum(), self.decode_stream)
        for t in (ddata, produced, bstat, dtab):
            t.record_stream(self.decode_stream)
        if self.track:
            self.checks.append(status)
        # the pinned bytes (record sets and plan tables) must outlive their async copies
        self._inflight = [(e, b) for e, b in getattr(self, "_inflight", []) if not e.query()] + \
            [(status.event if self.verify_crc else done, (staging, packed))]
        return RawBatch(out, offs, n, ends=ends[:n], source_bytes=plan.nbytes, status=status), done

    def check(self):
        """Raise if any decoded batch failed (reads the pending batches' status words, already copied to pinned
        host memory behind their decodes)."""
        pending, self.checks = self.checks, []
        bad = sum(s.failed() for s in pending)
        if bad:
            raise DecodeError(f"{bad} Kafka record batch(es) failed to decode on the device")


class DecodeError(ValueError):
    pass


class DecodeStatus:
    """Number of record batches of one fetch that failed to decode (corrupt LZ4 block, record framing past the
    batch), copied device → pinned host on the decode stream right behind the decode, so reading it later costs
    no device synchronisation beyond that batch's own decode."""

    __slots__ = ("host", "event")

    def __init__(self, bad: torch.Tensor, stream):
        self.host = torch.empty(1, dtype=torch.int64, pin_memory=True)
        self.host.copy_(bad.reshape(1), non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record(stream)

    def failed(self) -> int:
        self.event.synchronize()
        return int(self.host[0])

    def raise_if_failed(self, what: str = "batch"):
        """Called by the processor before a batch's rows reach a state table or a sink."""
        bad = self.failed()
        if bad:
            raise DecodeError(f"{what}: {bad} Kafka record batch(es) failed to decode on the device")


_CRC_POLY = 0x82F63B78


def _multmodp(a: int, b: int) -> int:
    p = 0
    m = 1 << 31
    while m:
        if a & m:
            p ^= b
        b = (b >> 1) ^ _CRC_POLY if b & 1 else b >> 1
        m >>= 1
    return p


def _x2n_table():
    t, p = [], 1 << 30
    for _ in range(32):
        t.append(p)
        p = _multmodp(p, p)
    return t


_X2N = _x2n_table()


def _raw_crc(reg: int, data: bytes) -> int:
    for byte in data:
        reg ^= byte
        for _ in range(8):
            reg = (reg >> 1) ^ _CRC_POLY if reg & 1 else reg >> 1
    return reg


def _x8n(n: int) -> int:
    p, sq = 1 << 31, 1 << 30
    for _ in range(3):
        sq = _multmodp(sq, sq)
    while n:
        if n & 1:
            p = _multmodp(sq, p)
        sq = _multmodp(sq, sq)
        n >>= 1
    return p


def crc32c_segmented(data: bytes, base_align: int = 0) -> int:
    """CPU mirror of ``kafka_crc_kernel``: 512-B rows right-aligned on the 8-B boundary at or below the end (the data
    starts ``base_align`` bytes past an 8-B boundary), lane l accumulating the 8-B word at l*8 of every row with the
    zero-init register (acc = T8(acc ^ w), then ·x^(8·504) between rows), the init folded into the first 4 bytes,
    bytes before the start as zeros, lane results scaled by x^(64·(63-l)) and XORed, the tail folded serially —
    equal to the serial CRC-32C of ``data`` (≥ 4 bytes)."""
    n = len(data)
    e = base_align + n                         # positions relative to the 8-B aligned origin
    E = e - (e & 7)
    if E - base_align < 8:                     # tiny: all serial
        return ~_raw_crc(0xFFFFFFFF, data) & 0xFFFFFFFF
    nrow = (E - base_align + 511) // 512
    r0 = E - nrow * 512
    msg = bytearray(data)
    for q in range(min(4, n)):
        msg[q] ^= 0xFF

    def byte_at(pos):
        q = pos - base_align
        return msg[q] if 0 <= q < n else 0
    total = 0
    for lane in range(64):
        acc = 0
        for r in range(nrow):
            a = r0 + r * 512 + lane * 8
            acc = _raw_crc(acc, bytes(byte_at(a + k) for k in range(8)))
            if r + 1 < nrow:
                acc = _multmodp(_x8n(504), acc)
        if acc:
            total ^= _multmodp(_x8n((63 - lane) * 8), acc)
    reg = _raw_crc(total, bytes(msg[E - base_align:]))
    return ~reg & 0xFFFFFFFF


def decode_on_host_like(staging: np.ndarray, plan: FetchPlan, verify_crc: bool = False):
    """CPU reference of ``DeviceRecordDecoder.decode`` (tests): (values buffer, starts, ends).  ``verify_crc``
    raises on a batch whose CRC-32C does not match (the device's status 7)."""
    from ..ops import lz4
    out = np.zeros(plan.out_bytes + 64, dtype=np.uint8)
    starts, ends = [], []
    for i in range(plan.nbat):
        if verify_crc:
            lo = int(plan.b_crc_off[i])
            got = crc32c_segmented(staging[lo:lo + int(plan.b_crc_len[i])].tobytes(), lo & 7)
            if got != int(plan.b_crc[i]) & 0xFFFFFFFF:
                raise DecodeError(f"batch {i}: CRC-32C mismatch")
        f, nb = int(plan.b_first[i]), int(plan.b_nblk[i])
        p = int(plan.k_out_off[f])
        end = p
        for b in range(f, f + nb):                 # a frame's blocks back to back from its first slot
            src = staging[plan.k_comp_off[b]: plan.k_comp_off[b] + plan.k_comp_len[b]]
            kind = int(plan.k_stored[b])
            if kind == 2:                          # deflate data of a gzip member (header / trailer stripped)
                import zlib
                raw = zlib.decompressobj(-15).decompress(src.tobytes())
            elif kind == 3:                        # a snappy raw block
                from .kafka import snappy_decompress
                raw = snappy_decompress(src.tobytes())
            elif kind == 4:                        # a zstd frame
                from .kafka import zstd_decompress
                raw = zstd_decompress(src.tobytes())
            else:
                raw = src.tobytes() if kind else lz4.decompress_block(src.tobytes(), int(plan.k_cap[b]))
            out[end:end + len(raw)] = np.frombuffer(raw, np.uint8)
            end += len(raw)
        data = out

        def varint(p):
            u, s = 0, 0
            while True:
                c = int(data[p])
                p += 1
                u |= (c & 0x7F) << s
                s += 7
                if not c & 0x80:
                    return (u >> 1) ^ -(u & 1), p
        skip, keep, count = int(plan.b_skip[i]), int(plan.b_keep[i]), int(plan.b_count[i])
        for r in range(min(count, skip + keep)):
            ln, p = varint(p)
            rec_end = p + ln
            p += 1
            _, p = varint(p)
            _, p = varint(p)
            kl, p = varint(p)
            p += max(kl, 0)
            vl, p = varint(p)
            if r >= skip:
                starts.append(p)
                ends.append(p + max(vl, 0))
            p = rec_end
        assert p <= end
    return out, np.array(starts, np.int64), np.array(ends, np.int64)
