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
    outs = []
    for t in tensors:
        if t.dim() != 1 or int(t.shape[0]) != n_src or t.device != dev:
            raise ValueError("gather_many: 1-D tensors of one length on the index's device")
        outs.append(torch.empty(n_idx, dtype=t.dtype, device=dev))
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
