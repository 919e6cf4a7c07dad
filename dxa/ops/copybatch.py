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


def copy_batch(segments: Sequence[Segment], device) -> None:
    global _CHUNK
    if _CHUNK is None:
        if N.lib().dxa_copy_chunk_size() != 32:
            raise N.NativeError("CopyChunk layout mismatch between copybatch.py and copy_batch.hip")
        _CHUNK = int(N.lib().dxa_copy_chunk_bytes())
    rows: List[Tuple[int, int, int, int]] = []
    for src, so, dst, do, nb, fill in segments:
        if nb <= 0:
            continue
        sp = 0 if src is None else src.data_ptr() + so
        dp = dst.data_ptr() + do
        for k in range(0, nb, _CHUNK):
            rows.append((0 if src is None else sp + k, dp + k, min(_CHUNK, nb - k), fill))
    if not rows:
        return
    tab = torch.from_numpy(np.array(rows, dtype=np.uint64).view(np.int64)).pin_memory()
    dtab = tab.to(device, non_blocking=True)
    N.call("dxa_copy_batch", N.ptr(dtab), len(rows), N.stream_handle(device))


def concat_prims(parts: Sequence, device):
    """Row-concatenation of 1-D / [n, 2] PrimColumns of one storage dtype → (data, valid or None), all segments in
    one launch (None when the parts do not share a storage layout)."""
    d0 = parts[0].data
    if any(p.data.dtype != d0.dtype or p.data.dim() != d0.dim() or p.data.shape[1:] != d0.shape[1:]
           or not p.data.is_contiguous() for p in parts):
        return None
    total = sum(p.length for p in parts)
    data = torch.empty((total,) + tuple(d0.shape[1:]), dtype=d0.dtype, device=device)
    row_bytes = d0.element_size() * (d0.shape[1] if d0.dim() == 2 else 1)
    any_null = any(p.valid is not None for p in parts)
    valid = torch.empty(total, dtype=torch.bool, device=device) if any_null else None
    segs, r = [], 0
    for p in parts:
        n = p.length
        segs.append((p.data, 0, data, r * row_bytes, n * row_bytes, 0))
        if any_null:
            if p.valid is not None:
                v = p.valid if p.valid.is_contiguous() else p.valid.contiguous()
                segs.append((v, 0, valid, r, n, 0))
            else:
                segs.append((None, 0, valid, r, n, 1))
        r += n
    return data, valid, segs


def valid_segments(parts: Sequence, device):
    """Concatenated validity of columns (None when none has nulls) as copy / fill segments."""
    if not any(p.valid is not None for p in parts):
        return None, []
    total = sum(p.length for p in parts)
    valid = torch.empty(total, dtype=torch.bool, device=device)
    segs, r = [], 0
    for p in parts:
        n = p.length
        if p.valid is not None:
            v = p.valid if p.valid.is_contiguous() else p.valid.contiguous()
            segs.append((v, 0, valid, r, n, 0))
        else:
            segs.append((None, 0, valid, r, n, 1))
        r += n
    return valid, segs
