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
    """Copy / fill segments accumulated as flat lists (source pointer or 0 for a fill, destination pointer, bytes,
    fill byte): a table concatenation appends one block per column instead of a Python tuple per part, and the few
    segments of a typical concatenation never pay numpy's per-call overhead until the one conversion at launch."""

    def __init__(self):
        self.src: List[int] = []
        self.dst: List[int] = []
        self.nb: List[int] = []
        self.fill: List[int] = []
        self.keep: List[torch.Tensor] = []        # temporaries the segments read (alive until the launch is queued)

    @staticmethod
    def _as_list(v, k: int) -> List[int]:
        if isinstance(v, (list, tuple)):
            return [int(x) for x in v]
        if isinstance(v, np.ndarray) and v.ndim:
            return v.astype(np.int64, copy=False).tolist()
        return [int(v)] * k

    def add(self, src, dst, nb, fill=0) -> None:
        """Scalars or length-k sequences (lists / numpy arrays); scalars repeat for every segment."""
        nbl = self._as_list(nb, 1)
        k = len(nbl)
        self.nb.extend(nbl)
        self.src.extend(self._as_list(src, k))
        self.dst.extend(self._as_list(dst, k))
        self.fill.extend(self._as_list(fill, k))

    def extend(self, segments: Sequence[Segment]) -> None:
        for src, so, dst, do, nb, fill in segments:
            self.add(0 if src is None else src.data_ptr() + so, dst.data_ptr() + do, nb, fill)

    def __bool__(self):
        return bool(self.nb)

    def launch(self, device) -> None:
        if not self.nb:
            return
        chunk = _chunk_size()
        src, dst = np.array(self.src, dtype=np.int64), np.array(self.dst, dtype=np.int64)
        nb, fill = np.array(self.nb, dtype=np.int64), np.array(self.fill, dtype=np.int64)
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
    part's bytes as one block of segments (None when the parts do not share a storage layout)."""
    d0 = parts[0].data
    dt, dim, tail = d0.dtype, d0.dim(), d0.shape[1:]
    lens, ptrs, starts = [], [], []
    total = 0
    any_null = False
    for p in parts:
        d = p.data
        if d.dtype != dt or d.dim() != dim or d.shape[1:] != tail or not d.is_contiguous():
            return None
        starts.append(total)
        lens.append(p.length)
        total += p.length
        ptrs.append(d.data_ptr())
        any_null = any_null or p.valid is not None
    data = torch.empty((total,) + tuple(tail), dtype=dt, device=device)
    row_bytes = d0.element_size() * (d0.shape[1] if dim == 2 else 1)
    segs = Segments() if segs is None else segs
    base = data.data_ptr()
    segs.add(ptrs, [base + s0 * row_bytes for s0 in starts], [n * row_bytes for n in lens])
    valid = _valid_into(parts, lens, starts, total, device, segs) if any_null else None
    return data, valid, segs


def _valid_into(parts, lens, starts, total, device, segs: Segments):
    valid = torch.empty(total, dtype=torch.bool, device=device)
    vp = []
    for p in parts:
        if p.valid is None:
            vp.append(0)
            continue
        v = p.valid if p.valid.is_contiguous() else p.valid.contiguous()
        vp.append(v.data_ptr())
        if v is not p.valid:
            segs.keep.append(v)                      # a contiguous copy must outlive the launch
    base = valid.data_ptr()
    segs.add(vp, [base + s0 for s0 in starts], list(lens), [1 if q == 0 else 0 for q in vp])
    return valid


def valid_segments(parts: Sequence, device, segs: Optional[Segments] = None):
    """Concatenated validity of columns (None when none has nulls) as copy / fill segments."""
    segs = Segments() if segs is None else segs
    if not any(p.valid is not None for p in parts):
        return None, segs
    lens, starts, total = [], [], 0
    for p in parts:
        starts.append(total)
        lens.append(p.length)
        total += p.length
    return _valid_into(parts, lens, starts, total, device, segs), segs
