"""LZ4 frames: host codec (``host_lz4.cpp``) and the device block decoder (``lz4.hip``).

Compressed ingest: a batch of newline-delimited events travels host → HBM as an LZ4 frame (≈2.5x fewer PCIe bytes
for SimulatedData-shaped JSON), is decoded by 16 lanes per block, and framed into records on the device.
The same frames are Kafka's compression codec 3 payload (``io/kafka.py``).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import native as N

DEFAULT_BLOCK = 16 * 1024
_HOST = None


class Lz4Error(RuntimeError):
    pass


def _host():
    global _HOST
    if _HOST is None:
        from .serialize import lib
        L = lib()
        i64, i32, p = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
        L.dxa_lz4_frame_bound.restype = i64
        L.dxa_lz4_frame_bound.argtypes = [i64, i32]
        L.dxa_lz4_compress_frame.restype = i64
        L.dxa_lz4_compress_frame.argtypes = [p, i64, p, i64, i32, i32]
        L.dxa_lz4_compress_frame_level.restype = i64
        L.dxa_lz4_compress_frame_level.argtypes = [p, i64, p, i64, i32, i32, i32]
        L.dxa_lz4_decompress_frame.restype = i64
        L.dxa_lz4_decompress_frame.argtypes = [p, i64, p, i64]
        L.dxa_lz4_frame_blocks.restype = i64
        L.dxa_lz4_frame_blocks.argtypes = [p, i64, p, p, p, i64, p, p, p]
        L.dxa_lz4_compress_block.restype = i64
        L.dxa_lz4_compress_block.argtypes = [p, i64, p]
        L.dxa_lz4_decompress_block.restype = i64
        L.dxa_lz4_decompress_block.argtypes = [p, i64, p, i64]
        L.dxa_xxh32.restype = ctypes.c_uint32
        L.dxa_xxh32.argtypes = [p, i64, ctypes.c_uint32]
        _HOST = L
    return _HOST


def _as_np(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data.view(np.uint8).reshape(-1))
    if isinstance(data, torch.Tensor):
        return data.detach().cpu().contiguous().view(torch.uint8).numpy().reshape(-1)
    return np.frombuffer(bytes(data), dtype=np.uint8)


def xxh32(data, seed: int = 0) -> int:
    a = _as_np(data)
    return int(_host().dxa_xxh32(a.ctypes.data, a.size, seed))


def compress_frame(data, block_size: int = DEFAULT_BLOCK, threads: Optional[int] = None, level: int = 0
                   ) -> np.ndarray:
    """LZ4 frame of ``data``.  ``level`` <= 2: fast greedy compressor; >= 3: high-compression mode (hash chains,
    2^(level-1) candidates, lazy matching) — the producer-side setting (Kafka ``compression.lz4.level``) that
    trades compression time for fewer, longer sequences: a smaller frame and a cheaper decode."""
    a = _as_np(data)
    L = _host()
    cap = L.dxa_lz4_frame_bound(a.size, block_size)
    out = np.empty(cap, dtype=np.uint8)
    m = L.dxa_lz4_compress_frame_level(a.ctypes.data, a.size, out.ctypes.data, cap, block_size,
                                       threads or min(16, os.cpu_count() or 4), level)
    if m < 0:
        raise Lz4Error("lz4 frame compression failed")
    return out[:m]


def decompress_frame(data, size_hint: Optional[int] = None) -> bytes:
    a = _as_np(data)
    try:
        content = frame_table(a).content_size
    except Lz4Error as e:
        if "dependent" not in str(e):
            raise
        content = -1          # linked blocks (liblz4's default above one block): host decode, size unknown up front
    cap = content if content >= 0 else (size_hint or max(1, a.size) * 8)
    while True:
        out = np.empty(max(cap, 1), dtype=np.uint8)
        m = _host().dxa_lz4_decompress_frame(a.ctypes.data, a.size, out.ctypes.data, cap)
        if m >= 0:
            return out[:m].tobytes()
        if content >= 0 or cap > (1 << 34):
            raise Lz4Error(f"lz4 frame decode failed ({m})")
        cap *= 4


def compress_block(data) -> bytes:
    a = _as_np(data)
    out = np.empty(a.size + a.size // 255 + 16, dtype=np.uint8)
    m = _host().dxa_lz4_compress_block(a.ctypes.data, a.size, out.ctypes.data)
    return out[:m].tobytes()


def decompress_block(data, size: int) -> bytes:
    a = _as_np(data)
    out = np.empty(max(size, 1), dtype=np.uint8)
    m = _host().dxa_lz4_decompress_block(a.ctypes.data, a.size, out.ctypes.data, size)
    if m < 0:
        raise Lz4Error("lz4 block decode failed")
    return out[:m].tobytes()


@dataclass
class FrameTable:
    comp_off: np.ndarray          # int64 [nb]  block payload offsets in the frame
    comp_len: np.ndarray          # int32 [nb]
    stored: np.ndarray            # uint8 [nb]  1 = stored uncompressed
    content_size: int             # -1 when the frame does not carry it
    max_block: int
    frame_end: int

    @property
    def nblocks(self) -> int:
        return int(self.comp_off.shape[0])

    def out_offsets(self, block_size: Optional[int] = None):
        """(out_off, out_len) when every block but the last is full — true for frames from ``compress_frame`` (and
        Kafka's producer); None otherwise (the device size pass then computes them)."""
        if self.content_size < 0 or block_size is None:
            return None
        nb = self.nblocks
        off = np.arange(nb, dtype=np.int64) * block_size
        ln = np.minimum(block_size, self.content_size - off).astype(np.int64)
        if nb and (ln[-1] <= 0 or off[-1] + ln[-1] != self.content_size):
            return None
        return off, ln


def frame_table(data) -> FrameTable:
    a = _as_np(data)
    L = _host()
    cs, mb, fe = ctypes.c_int64(0), ctypes.c_int32(0), ctypes.c_int64(0)
    nb = L.dxa_lz4_frame_blocks(a.ctypes.data, a.size, None, None, None, 0, ctypes.byref(cs), ctypes.byref(mb),
                                ctypes.byref(fe))
    if nb == -2:
        raise Lz4Error("dependent-block or dictionary LZ4 frames are decoded on the host only")
    if nb < 0:
        raise Lz4Error("malformed LZ4 frame")
    off = np.zeros(nb, dtype=np.int64)
    ln = np.zeros(nb, dtype=np.int32)
    st = np.zeros(nb, dtype=np.uint8)
    L.dxa_lz4_frame_blocks(a.ctypes.data, a.size, off.ctypes.data, ln.ctypes.data, st.ctypes.data, nb,
                           ctypes.byref(cs), ctypes.byref(mb), ctypes.byref(fe))
    return FrameTable(off, ln, st, cs.value, mb.value, fe.value)


@dataclass
class DeviceFrame:
    """An LZ4 frame staged for the device: frame bytes + block table (host pinned or already in HBM)."""
    data: torch.Tensor            # uint8 frame bytes (padded by 32: decoder lanes read ahead of the block end)
    comp_off: torch.Tensor
    comp_len: torch.Tensor
    stored: torch.Tensor
    out_off: Optional[torch.Tensor]
    out_len: Optional[torch.Tensor]
    content_size: int
    max_block: int
    max_out: int = -1             # largest decompressed block when out_len is known (sizes the LDS staging)

    @staticmethod
    def from_frame(frame: np.ndarray, block_size: Optional[int] = DEFAULT_BLOCK, pin: bool = False) -> "DeviceFrame":
        t = frame_table(frame)
        padded = np.zeros(frame.size + 32, dtype=np.uint8)
        padded[:frame.size] = frame
        oo = t.out_offsets(block_size)

        def T(x):
            x = torch.from_numpy(np.ascontiguousarray(x))
            return x.pin_memory() if pin else x
        return DeviceFrame(T(padded), T(t.comp_off), T(t.comp_len), T(t.stored),
                           T(oo[0]) if oo else None, T(oo[1]) if oo else None, t.content_size, t.max_block,
                           int(oo[1].max()) if oo and oo[1].size else -1)

    def to(self, device, non_blocking: bool = True) -> "DeviceFrame":
        f = lambda x: None if x is None else x.to(device, non_blocking=non_blocking)  # noqa: E731
        return DeviceFrame(f(self.data), f(self.comp_off), f(self.comp_len), f(self.stored), f(self.out_off),
                           f(self.out_len), self.content_size, self.max_block, self.max_out)

    def tensors(self):
        return [x for x in (self.data, self.comp_off, self.comp_len, self.stored, self.out_off, self.out_len)
                if x is not None]


def decompress_device(fr: DeviceFrame, check: bool = False) -> torch.Tensor:
    """Decode a device-resident frame → uint8 tensor [content + 16 zero pad bytes] on the same device.  No host
    synchronisation when the block sizes are known (``out_off``); ``check=True`` verifies every block's status."""
    dev = fr.data.device
    if dev.type != "cuda":
        raw = decompress_frame(fr.data.numpy()[:-32])
        out = torch.zeros(len(raw) + 16, dtype=torch.uint8)
        out[:len(raw)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
        return out
    nb = int(fr.comp_off.shape[0])
    st = N.stream_handle(dev)
    status = torch.empty(max(nb, 1), dtype=torch.int32, device=dev)
    if fr.out_off is None:
        ln = torch.empty(max(nb, 1), dtype=torch.int64, device=dev)
        N.call("dxa_lz4_block_sizes", N.ptr(fr.data), N.ptr(fr.comp_off), N.ptr(fr.comp_len), N.ptr(fr.stored), nb,
               fr.max_block, N.ptr(ln), N.ptr(status), st)
        ln = ln[:nb]
        off = torch.cumsum(ln, 0) - ln
        total = int(ln.sum().item()) if nb else 0
        max_out = int(ln.max().item()) if nb else 0
        if nb and bool((status[:nb] != 0).any()):
            raise Lz4Error("malformed LZ4 block")
    else:
        off, ln, total, max_out = fr.out_off, fr.out_len, fr.content_size, fr.max_out
    out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    out[total:].zero_()
    N.call("dxa_lz4_decode", N.ptr(fr.data), N.ptr(fr.comp_off), N.ptr(fr.comp_len), N.ptr(fr.stored), N.ptr(off),
           N.ptr(ln), nb, max_out, N.ptr(out), N.ptr(status), st)
    if check and nb and bool((status[:nb] != 0).any()):
        raise Lz4Error(f"LZ4 block decode failed: status {status[:nb].unique().tolist()}")
    return out


class ChunkedIngest:
    """Pipelined compressed ingest of a pinned host frame: the frame is cut into ``chunks`` runs of whole blocks;
    chunk k's H2D copy (copy stream) overlaps chunk k-1's decode (decode stream), so the critical path is about
    max(copy, decode) instead of copy + decode.  Blocks read up to 32 bytes past their end, which may land in the
    next chunk while its copy is still in flight — the decoder never uses those bytes.

    ``stage(frame)`` returns ``(raw, done_event)``: ``raw`` is the decompressed batch (+16 zero bytes) on the
    device, valid on any stream that waits on ``done_event``."""

    def __init__(self, device, chunks: int = 8, copy_stream=None, decode_stream=None):
        # HIP multiplexes streams onto GPU_MAX_HW_QUEUES (4) hardware queues: callers that already own a copy
        # stream should pass it, so the pipeline adds one stream, not two
        self.device = device
        self.chunks = max(1, chunks)
        self.copy_stream = copy_stream or torch.cuda.Stream(device)
        self.decode_stream = decode_stream or torch.cuda.Stream(device)

    def stage(self, fr: "DeviceFrame"):
        dev = self.device
        if fr.out_off is None:
            raise Lz4Error("chunked ingest needs frames with known block sizes")
        nb = int(fr.comp_off.shape[0])
        total = fr.content_size
        # Allocation streams: `out`/`status` belong to the decode stream (consumers on other streams must
        # record_stream `out`); the compressed staging buffer belongs to the copy stream that fills it and is
        # recorded on the decode stream, so it is not recycled while a decode still reads it.
        with torch.cuda.stream(self.decode_stream):
            out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
            status = torch.empty(max(nb, 1), dtype=torch.int32, device=dev)
        with torch.cuda.stream(self.copy_stream):
            ddata = torch.empty(fr.data.shape[0], dtype=torch.uint8, device=dev)
        with torch.cuda.stream(self.copy_stream):
            # block tables are small: one copy up front
            tabs = [x.to(dev, non_blocking=True) for x in (fr.comp_off, fr.comp_len, fr.stored, fr.out_off,
                                                           fr.out_len)]
            tab_ev = torch.cuda.Event()
            tab_ev.record(self.copy_stream)
        comp_off_h = fr.comp_off.numpy() if fr.comp_off.device.type == "cpu" else fr.comp_off.cpu().numpy()
        bounds = np.linspace(0, nb, self.chunks + 1).astype(np.int64)
        nbytes = int(fr.data.shape[0])
        st = self.decode_stream.cuda_stream
        self.decode_stream.wait_event(tab_ev)
        with torch.cuda.stream(self.decode_stream):
            out[total:].zero_()
        for k in range(self.chunks):
            b0, b1 = int(bounds[k]), int(bounds[k + 1])
            if b1 <= b0:
                continue
            lo = 0 if k == 0 else int(comp_off_h[b0])
            hi = nbytes if b1 == nb else int(comp_off_h[b1])
            if fr.data.device.type == "cpu":
                if not fr.data.is_pinned():
                    raise Lz4Error("chunked ingest needs a pinned host frame")
                N.call("dxa_memcpy_h2d_async", ddata.data_ptr() + lo, fr.data.data_ptr() + lo, hi - lo,
                       self.copy_stream.cuda_stream)
            else:
                with torch.cuda.stream(self.copy_stream):
                    ddata[lo:hi].copy_(fr.data[lo:hi], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
            self.decode_stream.wait_event(ev)
            co, cl, sd, oo, ol = tabs
            N.call("dxa_lz4_decode", N.ptr(ddata), N.ptr(co[b0:b1]), N.ptr(cl[b0:b1]), N.ptr(sd[b0:b1]),
                   N.ptr(oo[b0:b1]), N.ptr(ol[b0:b1]), b1 - b0, fr.max_out, N.ptr(out), N.ptr(status[b0:b1]), st)
        done = torch.cuda.Event()
        done.record(self.decode_stream)
        for t in (ddata, *tabs):
            t.record_stream(self.decode_stream)
        # the host frame must outlive its async copies
        self._inflight = [(e, f) for e, f in getattr(self, "_inflight", []) if not e.query()] + [(done, fr)]
        return out, done
