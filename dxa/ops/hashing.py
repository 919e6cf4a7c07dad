"""Row hashing of key columns (group-by / join / distinct / shuffle partitioning).

GPU: ``dxa_hash_{i64,f64,str}`` kernels (hash_groupby.hip).  CPU: a bit-exact numpy re-implementation of the same
functions so GPU results can be differential-tested against it.
"""
from __future__ import annotations

import ctypes
from typing import List

import numpy as np
import torch

from . import native as N
from ..engine.decimal import is_decimal, key_parts as decimal_key_parts

SEED = np.uint64(0x5bd1e9955bd1e995)
GOLD = np.uint64(0x9E3779B97F4A7C15)
NULL_HASH = np.uint64(0x6e756c6c6e756c6c)
C1 = np.uint64(0xff51afd7ed558ccd)
C2 = np.uint64(0xc4ceb9fe1a85ec53)


def _fmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(33))
        x = x * C1
        x = x ^ (x >> np.uint64(33))
        x = x * C2
        x = x ^ (x >> np.uint64(33))
    return x


def _hash_i64_np(v: np.ndarray) -> np.ndarray:
    return _fmix64(v.astype(np.int64).view(np.uint64) ^ SEED)


def _combine_np(acc: np.ndarray, h: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        return _fmix64(acc ^ (h + GOLD + (acc << np.uint64(6)) + (acc >> np.uint64(2))))


def _hash_bytes_np(b: bytes) -> np.uint64:
    n = len(b)
    with np.errstate(over="ignore"):
        h = SEED ^ (np.uint64(n) * GOLD)
        i = 0
        while i + 8 <= n:
            w = np.uint64(int.from_bytes(b[i:i + 8], "little"))
            h = _fmix64(np.array([h ^ w], dtype=np.uint64))[0]
            i += 8
        if i < n:
            w = np.uint64(int.from_bytes(b[i:], "little"))
            h = _fmix64(np.array([h ^ w], dtype=np.uint64))[0]
        return _fmix64(np.array([h ^ np.uint64(n)], dtype=np.uint64))[0]


def _hash_strs_np(arena: np.ndarray, starts: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """``_hash_bytes_np`` of every string at once: word k of all strings in one vector step (little-endian 8-byte
    words, the short tail word zero-extended), so the CPU path costs O(longest / 8) numpy passes, not a Python loop
    per string."""
    n = len(lens)
    lens = lens.astype(np.int64)
    starts = starts.astype(np.int64)
    pad = np.zeros(arena.size + 8, dtype=np.uint8)
    pad[:arena.size] = arena
    nw = lens // 8
    tail = lens - nw * 8
    lane = np.arange(8, dtype=np.int64)

    def word(off):
        return pad[off[:, None] + lane].view(np.uint64).reshape(-1)

    with np.errstate(over="ignore"):
        h = SEED ^ (lens.astype(np.uint64) * GOLD)
        for k in range(int(nw.max()) if n else 0):
            m = nw > k
            h[m] = _fmix64(h[m] ^ word(starts[m] + 8 * k))
        m = tail > 0
        if m.any():
            w = word(starts[m] + 8 * nw[m])
            keep = (np.uint64(1) << (tail[m].astype(np.uint64) * np.uint64(8))) - np.uint64(1)
            h[m] = _fmix64(h[m] ^ (w & keep))
        return _fmix64(h ^ lens.astype(np.uint64))


def _col_hash_np(col) -> np.ndarray:
    from ..engine.column import PrimColumn, StrColumn, ConstColumn, materialize
    col = materialize(col)
    n = col.length
    if isinstance(col, StrColumn):
        out = _hash_strs_np(col.arena.cpu().numpy(), col.starts.cpu().numpy(), col.lens.cpu().numpy())
    elif isinstance(col, PrimColumn):
        d = col.data.cpu()
        if d.dtype == torch.float64:
            a = d.numpy().copy()
            a[a == 0.0] = 0.0
            bits = a.view(np.uint64).copy()
            bits[np.isnan(a)] = np.uint64(0x7ff8000000000000)
            out = _fmix64(bits ^ SEED)
        else:
            out = _hash_i64_np(d.to(torch.int64).numpy())
    else:
        raise TypeError(f"cannot hash column {col!r}")
    if col.valid is not None:
        v = col.valid.cpu().numpy()
        out = np.where(v, out, NULL_HASH)
    return out


MAX_KEY_COLS = 16
_KC_I64, _KC_F64, _KC_STR = 0, 1, 2


class _KeyCol(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("starts", ctypes.c_void_p), ("lens", ctypes.c_void_p),
                ("valid", ctypes.c_void_p), ("kind", ctypes.c_int32), ("pad", ctypes.c_int32)]


class _KeyCols(ctypes.Structure):
    _fields_ = [("c", _KeyCol * MAX_KEY_COLS), ("ncols", ctypes.c_int32), ("n", ctypes.c_int64)]


N.register_sigs({"dxa_key_cols_size": [], "dxa_hash_multi": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
                 "dxa_verify_multi": [ctypes.c_void_p] * 5,
                 "dxa_pairs_equal": [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]})


def key_cols(cols):
    """By-value descriptor of materialised device key columns for the fused hash / verify kernels (None when a
    column is not a plain string / 8-byte column).  The descriptor keeps the tensors it points at alive."""
    from ..engine.column import PrimColumn, StrColumn
    if N.lib().dxa_key_cols_size() != ctypes.sizeof(_KeyCols):
        raise N.NativeError("KeyCols layout mismatch between hashing.py and hash_groupby.hip")
    a = _KeyCols()
    keep = []
    for j, c in enumerate(cols):
        v = N.u8(c.valid)
        if v is not None:
            v = v.contiguous()
            keep.append(v)
        if isinstance(c, StrColumn):
            st, ln = c.starts, c.lens
            if st.dtype != torch.int64 or ln.dtype != torch.int32:
                return None
            a.c[j] = _KeyCol(c.arena.data_ptr(), st.data_ptr(), ln.data_ptr(), 0 if v is None else v.data_ptr(),
                             _KC_STR, 0)
        elif isinstance(c, PrimColumn) and c.data.dim() == 1:
            d = c.data
            kind = _KC_F64 if d.dtype == torch.float64 else _KC_I64
            if d.dtype not in (torch.float64, torch.int64):
                d = d.to(torch.int64)
            d = d.contiguous()
            keep.append(d)
            a.c[j] = _KeyCol(d.data_ptr(), None, None, 0 if v is None else v.data_ptr(), kind, 0)
        else:
            return None
    a.ncols, a.n = len(cols), cols[0].length
    a._keep = keep
    return a


def hash_columns(cols: List) -> torch.Tensor:
    """64-bit row hash over one or more key columns → int64 tensor (bit pattern of the uint64 hash)."""
    from ..engine.column import PrimColumn, StrColumn, materialize
    assert cols
    if any(is_decimal(c.dtype) for c in cols):
        cols = [p for c in cols for p in (decimal_key_parts(materialize(c)) if is_decimal(c.dtype) else [c])]
    n = cols[0].length
    device = cols[0].device
    if torch.device(device).type == "cuda":
        out = torch.empty(n, dtype=torch.int64, device=device)
        if n == 0:
            return out
        st = N.stream_handle(device)
        if 2 <= len(cols) <= MAX_KEY_COLS:
            kc = key_cols([materialize(c) for c in cols])
            if kc is not None:
                N.call("dxa_hash_multi", ctypes.byref(kc), N.ptr(out), st)     # every key column, one launch
                return out
        for j, c in enumerate(cols):
            c = materialize(c)
            comb = 1 if j else 0
            if isinstance(c, StrColumn):
                N.call("dxa_hash_str", N.ptr(c.arena), N.ptr(c.starts), N.ptr(c.lens), N.ptr(N.u8(c.valid)), n,
                       N.ptr(out), comb, st)
            elif isinstance(c, PrimColumn):
                d = c.data
                if d.dtype == torch.float64:
                    N.call("dxa_hash_f64", N.ptr(d), N.ptr(N.u8(c.valid)), n, N.ptr(out), comb, st)
                else:
                    if d.dtype != torch.int64:
                        d = d.to(torch.int64)
                    N.call("dxa_hash_i64", N.ptr(d), N.ptr(N.u8(c.valid)), n, N.ptr(out), comb, st)
            else:
                raise TypeError(f"cannot hash column {c!r}")
        return out
    acc = None
    for c in cols:
        h = _col_hash_np(c)
        acc = h if acc is None else _combine_np(acc, h)
    return torch.from_numpy(acc.view(np.int64).copy()).to(device)
