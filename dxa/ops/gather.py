"""Multi-column row gather (``gather.hip``): every leaf tensor of a table take in one launch per 48 leaves.

``gather_many(tensors, idx)`` returns ``[t[idx] for t in tensors]`` (1-D tensors of equal length; element size 1, 2,
4 or 8 bytes; negative indices count from the end as in torch).  ``dxa.engine.column.take_columns`` uses it for
``Table.take`` / struct / array takes on the GPU.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence

import torch

from . import native as N

N.register_sigs({
    "dxa_multi_gather_max_cols": [],
    "dxa_multi_gather": [N.c_p, N.c_p, N.c_p, N.c_i32, N.c_i64, N.c_p, N.c_i64, N.c_p],
})

_MAX_COLS = 48


_BLOCK_DT = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


def _alloc_rows(dtypes: Sequence[torch.dtype], n: int, dev) -> List[torch.Tensor]:
    """One device allocation per element size, carved into 256-byte aligned rows of ``n`` elements (a take of a
    30-leaf table is 3-4 allocator calls instead of 30).  The rows share their block's lifetime, as the rows of the
    JSON parser's value block already do."""
    by_size: dict = {}
    for k, dt in enumerate(dtypes):
        by_size.setdefault(torch.empty((), dtype=dt).element_size() if dt not in _ESIZE else _ESIZE[dt],
                           []).append(k)
    outs: List[torch.Tensor] = [None] * len(dtypes)  # type: ignore[list-item]
    for es, ks in by_size.items():
        per = max(1, 256 // es)
        stride = (max(n, 1) + per - 1) // per * per
        block = torch.empty((len(ks), stride), dtype=_BLOCK_DT[es], device=dev)
        for k, row in zip(ks, block[:, :n].unbind(0)):
            dt = dtypes[k]
            outs[k] = row if dt == _BLOCK_DT[es] else row.view(dt)
    return outs


_ESIZE = {torch.bool: 1, torch.uint8: 1, torch.int8: 1, torch.int16: 2, torch.float16: 2, torch.bfloat16: 2,
          torch.int32: 4, torch.float32: 4, torch.int64: 8, torch.float64: 8}


def gather_many(tensors: Sequence[torch.Tensor], idx: torch.Tensor) -> List[torch.Tensor]:
    tensors = list(tensors)
    if not tensors:
        return []
    dev = idx.device
    if dev.type != "cuda":
        return [t[idx] for t in tensors]
    n_idx = int(idx.shape[0])
    idx = idx.to(torch.int64).contiguous()
    n_src = int(tensors[0].shape[0])
    for t in tensors:
        if t.dim() != 1 or int(t.shape[0]) != n_src or t.device != dev:
            raise ValueError("gather_many: 1-D tensors of one length on the index's device")
    outs = _alloc_rows([t.dtype for t in tensors], n_idx, dev)
    if n_idx == 0:
        return outs
    srcs = [t.contiguous() for t in tensors]
    st = N.stream_handle(dev)
    for lo in range(0, len(srcs), _MAX_COLS):
        part = range(lo, min(lo + _MAX_COLS, len(srcs)))
        k = len(part)
        sp = (ctypes.c_void_p * k)(*[srcs[i].data_ptr() for i in part])
        dp = (ctypes.c_void_p * k)(*[outs[i].data_ptr() for i in part])
        el = (ctypes.c_int32 * k)(*[srcs[i].element_size() for i in part])
        N.call("dxa_multi_gather", ctypes.cast(sp, ctypes.c_void_p), ctypes.cast(dp, ctypes.c_void_p),
               ctypes.cast(el, ctypes.c_void_p), k, n_src, N.ptr(idx), n_idx, st)
    return outs
