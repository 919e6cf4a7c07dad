"""Batched device copies (dxa/ops/csrc/copy_batch.hip): many (source, destination, bytes) segments — or fills — in
one launch, described by one pinned chunk table that crosses to the device in one copy."""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import native as N

N.register_sigs({"dxa_copy_chunk_size": [], "dxa_copy_chunk_bytes": [],
                 "dxa_copy_batch": [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]})
N.lib().dxa_copy_chunk_bytes.restype = ctypes.c_int64
_CHUNK = None

# (source tensor or None for a fill, source byte offset, destination tensor, destination byte offset, bytes, fill)
Segment = Tuple[Optional[torch.Tensor], int, torch.Tensor, int, int, int]


def _chunk_size() -> int:
    global _CHUNK
    if _CHUNK is None:
        if N.lib().dxa_copy_chunk_size() != 32:
            raise N.NativeError("CopyChunk layout mismatch between copybatch.py and copy_batch.hip")
        _CHUNK = int(N.lib().dxa_copy_chunk_bytes())
    return _CHUNK


class Segments:
    """Copy / fill segments accumulated as flat arrays (source pointer or 0 for a fill, destination pointer, bytes,
    fill byte): a table concatenation appends one array block per column instead of a Python tuple per part."""

    def __init__(self):
        self.src: List[np.ndarray] = []
        self.dst: List[np.ndarray] = []
        self.nb: List[np.ndarray] = []
        self.fill: List[np.ndarray] = []
        self.keep: List[torch.Tensor] = []        # temporaries the segments read (alive until the launch is queued)

    def add(self, src, dst, nb, fill=0) -> None:
        nb = np.asarray(nb, dtype=np.int64)
        k = nb.shape[0] if nb.ndim else 1
        nb = nb.reshape(k)
        self.src.append(np.broadcast_to(np.asarray(src, dtype=np.int64), (k,)))
        self.dst.append(np.broadcast_to(np.asarray(dst, dtype=np.int64), (k,)))
        self.nb.append(nb)
        self.fill.append(np.broadcast_to(np.asarray(fill, dtype=np.int64), (k,)))

    def extend(self, segments: Sequence[Segment]) -> None:
        for src, so, dst, do, nb, fill in segments:
            self.add(0 if src is None else src.data_ptr() + so, dst.data_ptr() + do, nb, fill)

    def __bool__(self):
        return bool(self.nb)

    def launch(self, device) -> None:
        if not self.nb:
            return
        chunk = _chunk_size()
        src, dst = np.concatenate(self.src), np.concatenate(self.dst)
        nb, fill = np.concatenate(self.nb), np.concatenate(self.fill)
        keep = nb > 0
        if not keep.all():
            src, dst, nb, fill = src[keep], dst[keep], nb[keep], fill[keep]
        if nb.size == 0:
            return
        rows = chunk_rows(src, dst, nb, fill, chunk)
        tab = torch.from_numpy(rows).pin_memory()
        dtab = tab.to(device, non_blocking=True)
        N.call("dxa_copy_batch", N.ptr(dtab), int(rows.shape[0]), N.stream_handle(device))
        self.keep.clear()                           # freed after the launch: reuse is ordered behind it


def chunk_rows(src: np.ndarray, dst: np.ndarray, nb: np.ndarray, fill: np.ndarray, chunk: int) -> np.ndarray:
    """Segments (all ``nb > 0``) split into rows of at most ``chunk`` bytes — (src | 0, dst, bytes, fill) int64, one
    workgroup's work each (copy_batch.hip CopyChunk)."""
    per = (nb + chunk - 1) // chunk
    if (per == 1).all():
        rows = np.stack([src, dst, nb, fill], axis=1)
    else:
        seg = np.repeat(np.arange(nb.size), per)
        off = (np.arange(seg.size) - np.repeat(np.cumsum(per) - per, per)) * chunk
        rows = np.stack([np.where(src[seg] != 0, src[seg] + off, 0), dst[seg] + off,
                         np.minimum(chunk, nb[seg] - off), fill[seg]], axis=1)
    return np.ascontiguousarray(rows, dtype=np.int64)


def copy_batch(segments, device) -> None:
    """Run segments — a ``Segments`` or a sequence of (src tensor | None, src offset, dst tensor, dst offset, bytes,
    fill) — as one launch."""
    if not isinstance(segments, Segments):
        sg = Segments()
        sg.extend(segments)
        segments = sg
    segments.launch(device)


def concat_prims(parts: Sequence, device, segs: Optional[Segments] = None):
    """Row-concatenation of 1-D / [n, 2] PrimColumns of one storage dtype → (data, valid or None, segments), every
    part's bytes as one block of segment arrays (None when the parts do not share a storage layout)."""
    d0 = parts[0].data
    dt, dim, tail = d0.dtype, d0.dim(), d0.shape[1:]
    lens = np.empty(len(parts), dtype=np.int64)
    ptrs = np.empty(len(parts), dtype=np.int64)
    any_null = False
    for k, p in enumerate(parts):
        d = p.data
        if d.dtype != dt or d.dim() != dim or d.shape[1:] != tail or not d.is_contiguous():
            return None
        lens[k] = p.length
        ptrs[k] = d.data_ptr()
        any_null = any_null or p.valid is not None
    total = int(lens.sum())
    data = torch.empty((total,) + tuple(tail), dtype=dt, device=device)
    row_bytes = d0.element_size() * (d0.shape[1] if dim == 2 else 1)
    segs = Segments() if segs is None else segs
    starts = np.cumsum(lens) - lens
    segs.add(ptrs, data.data_ptr() + starts * row_bytes, lens * row_bytes)
    valid = _valid_into(parts, lens, starts, total, device, segs) if any_null else None
    return data, valid, segs


def _valid_into(parts, lens, starts, total, device, segs: Segments):
    valid = torch.empty(total, dtype=torch.bool, device=device)
    vp = np.zeros(len(parts), dtype=np.int64)
    for k, p in enumerate(parts):
        if p.valid is not None:
            v = p.valid if p.valid.is_contiguous() else p.valid.contiguous()
            vp[k] = v.data_ptr()
            if v is not p.valid:
                segs.keep.append(v)                  # a contiguous copy must outlive the launch
    segs.add(vp, valid.data_ptr() + starts, lens, np.where(vp == 0, 1, 0))
    return valid


def valid_segments(parts: Sequence, device, segs: Optional[Segments] = None):
    """Concatenated validity of columns (None when none has nulls) as copy / fill segments."""
    segs = Segments() if segs is None else segs
    if not any(p.valid is not None for p in parts):
        return None, segs
    lens = np.fromiter((p.length for p in parts), dtype=np.int64, count=len(parts))
    starts = np.cumsum(lens) - lens
    return _valid_into(parts, lens, starts, int(lens.sum()), device, segs), segs
