"""String-column operations: compaction/concatenation of arenas, literal predicates, CONCAT, casts, case mapping,
``stringToTimestamp``.  GPU → strings.hip kernels; CPU → straightforward torch/Python reference code.
"""
from __future__ import annotations

import ctypes
import datetime as _dt
import re
from typing import List, Optional, Sequence, Union

import numpy as np
import torch

from . import native as N

_CMP_OPS = {"=": 0, "!=": 1, "<": 2, "<=": 3, ">": 4, ">=": 5, "startswith": 6, "endswith": 7, "contains": 8}


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def _offsets(lens: torch.Tensor):
    """Exclusive scan of lengths → (offsets int64, total bytes)."""
    if lens.numel() == 0:
        return torch.zeros(0, dtype=torch.int64, device=lens.device), 0
    cs = torch.cumsum(lens.to(torch.int64), 0)
    total = int(cs[-1].item())
    return cs - lens.to(torch.int64), total


def _alloc_arena(total: int, device) -> torch.Tensor:
    a = torch.empty(total + 16, dtype=torch.uint8, device=device)
    a[total:].zero_()            # every byte below total is written by the producer; the pad feeds 16-B reads
    return a


def compact(col):
    """Densely repack the bytes a StrColumn references (drops the rest of its arena)."""
    off, total = _offsets(col.lens)
    dst = _alloc_arena(total, col.device)
    n = col.length
    if n and total:
        if _gpu(col.starts):
            N.call("dxa_str_gather", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n, N.ptr(off), N.ptr(dst),
                   N.stream_handle(col.device))
        else:
            src = col.arena
            idx = torch.repeat_interleave(col.starts - off, col.lens.to(torch.int64)) + torch.arange(
                total, dtype=torch.int64)
            dst[:total] = src[idx]
    out = type(col)(dst, off, col.lens.clone(), col.valid, col.dtype)
    out._compact = True
    if col.max_len is not None:
        out.max_len = col.max_len
    return out


def compact_known(col, total: int):
    """``compact`` when the caller already knows the column's total byte count (no host synchronisation)."""
    if not _gpu(col.starts):
        return compact(col)
    lens64 = col.lens.to(torch.int64)
    off = torch.cumsum(lens64, 0) - lens64
    dst = _alloc_arena(total, col.device)
    if col.length and total:
        N.call("dxa_str_gather", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), col.length, N.ptr(off),
               N.ptr(dst), N.stream_handle(col.device))
    out = type(col)(dst, off, col.lens.clone(), col.valid, col.dtype)
    out._compact = True
    return out


class _StrPart(ctypes.Structure):
    _fields_ = [("arena", ctypes.c_void_p), ("starts", ctypes.c_void_p), ("lens", ctypes.c_void_p),
                ("dst_off", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("row0", ctypes.c_int64),
                ("incl", ctypes.c_void_p), ("ex_out", ctypes.c_void_p)]


def _gather_parts(parts, device) -> None:
    """One ``dxa_str_gather_parts`` launch (per 32 parts) for many string gathers.  ``parts``: (StrColumn view,
    destination offsets tensor, destination arena) triples; offsets are per row of the part — or (StrColumn view,
    (inclusive byte scan, starts out), destination arena): the kernel derives each row's offset from the scan and
    stores it as the compacted column's starts."""
    parts = [p for p in parts if p[0].length]
    if not parts:
        return
    if N.lib().dxa_str_part_size() != ctypes.sizeof(_StrPart):
        raise N.NativeError("StrPart layout mismatch between strings.py and strings.hip")
    arr = (_StrPart * (len(parts) + 1))()
    row = 0
    for j, (c, off, dst) in enumerate(parts):
        if isinstance(off, tuple):
            incl, ex = off
            arr[j] = _StrPart(c.arena.data_ptr(), c.starts.data_ptr(), c.lens.data_ptr(), None, dst.data_ptr(), row,
                              incl.data_ptr(), ex.data_ptr())
        else:
            arr[j] = _StrPart(c.arena.data_ptr(), c.starts.data_ptr(), c.lens.data_ptr(), off.data_ptr(),
                              dst.data_ptr(), row, None, None)
        row += c.length
    arr[len(parts)].row0 = row                      # end sentinel
    N.call("dxa_str_gather_parts", ctypes.cast(arr, ctypes.c_void_p), len(parts), N.stream_handle(device))


def lens_concat(lens: Sequence[torch.Tensor]) -> torch.Tensor:
    """The rows' lengths of several string columns end to end (int32).  Columns parsed from one batch hold their
    lengths as consecutive full-width rows of the parser's length matrix: then this is a view of that block, not a
    copy (a 1 M-event batch's five string leaves: a 20 MB concatenation kernel per batch)."""
    if len(lens) > 1 and all(t.dtype == torch.int32 and t.dim() == 1 and t.is_contiguous() for t in lens):
        base = lens[0]
        step = base.shape[0] * 4
        p0 = base.data_ptr()
        st = base.untyped_storage()
        if all(t.shape[0] == base.shape[0] and t.data_ptr() == p0 + k * step and
               t.untyped_storage().data_ptr() == st.data_ptr() for k, t in enumerate(lens)):
            end = base.storage_offset() + len(lens) * base.shape[0]
            if end * 4 <= st.nbytes():
                return torch.as_strided(base, (len(lens) * base.shape[0],), (1,), base.storage_offset())
    return torch.cat(list(lens))


def compact_many(cols: Sequence, lens_all: Optional[torch.Tensor] = None, total: Optional[int] = None) -> list:
    """``compact`` of several string columns with ONE host synchronisation and one scan: every column's bytes are
    packed into one shared arena (column k's rows after column k-1's), offsets from a single scan over all the
    lengths, the bytes moved by one multi-part gather launch.  ``lens_all`` / ``total``: the columns' lengths
    already concatenated and their sum already read (then no synchronisation here)."""
    cols = list(cols)
    if not cols:
        return []
    if not _gpu(cols[0].starts) or len(cols) == 1:
        return [compact(c) for c in cols]
    device = cols[0].device
    total_rows = sum(c.length for c in cols)
    if total_rows == 0:
        return [compact(c) for c in cols]
    if lens_all is None:
        lens_all = lens_concat([c.lens for c in cols])
    cs = torch.cumsum(lens_all, 0, dtype=torch.int64)
    ex = torch.empty_like(cs)                      # the compacted starts: written by the gather (cs - lens)
    if total is None:
        total = int(cs[-1].item())
    dst = _alloc_arena(total, device)
    out, parts, r = [], [], 0
    for c in cols:
        off = ex[r:r + c.length]
        if c.length:
            parts.append((c, (cs[r:r + c.length], off), dst))
        r += c.length
        o = type(c)(dst, off, c.lens, c.valid, c.dtype)
        o._compact = True
        out.append(o)
    _gather_parts(parts, device)                   # every column's bytes in one launch
    return out


def concat_multi(groups: Sequence[Sequence]):
    """Several row-concatenations of device StrColumns at once (a table concatenation's string columns): one length
    concatenation, one scan, one host read and one multi-part gather for all of them; the outputs share one arena.
    Returns [(arena, starts, lens)] per group (validity is the caller's)."""
    device = groups[0][0].device
    flat = [c for g in groups for c in g]
    lens_all = torch.cat([c.lens.to(torch.int32) for c in flat])
    if lens_all.numel() == 0:
        return [(_alloc_arena(0, device), torch.zeros(0, dtype=torch.int64, device=device),
                 torch.zeros(0, dtype=torch.int32, device=device)) for _ in groups]
    cs = torch.cumsum(lens_all, 0, dtype=torch.int64)
    ex = cs - lens_all
    if all(c.length == 0 or getattr(c, "_compact", False) or c.max_len is not None for c in flat):
        # every part's bytes are bounded on the host — a compacted arena holds exactly its rows' bytes (window
        # panes), rows with a known length bound (a window dictionary's key slots) at most rows x bound, an empty
        # part none — so the batch thread does not wait for the scan
        total = sum(0 if c.length == 0 else int(c.arena.numel()) if getattr(c, "_compact", False)
                    else c.length * c.max_len for c in flat)
    else:
        total = int(cs[-1].item())
    dst = _alloc_arena(total, device)
    out, parts, pos = [], [], 0
    for g in groups:
        n = sum(c.length for c in g)
        for c in g:
            if c.length:
                parts.append((c, ex[pos:pos + c.length], dst))
            pos += c.length
        out.append((dst, ex[pos - n:pos], lens_all[pos - n:pos]))
    _gather_parts(parts, device)                    # every part of every column in one launch
    return out


def concat(cols: Sequence, valid: Optional[torch.Tensor]):
    """Row-concatenate StrColumns (may reference different arenas) into one compact column."""
    device = cols[0].device
    lens = torch.cat([c.lens for c in cols])
    off, total = _offsets(lens)
    dst = _alloc_arena(total, device)
    if _gpu(cols[0].starts):
        parts, pos = [], 0
        for c in cols:
            if c.length:
                parts.append((c, off[pos:pos + c.length], dst))
            pos += c.length
        _gather_parts(parts, device)                # all parts' bytes in one launch
        return type(cols[0])(dst, off, lens.to(torch.int32), valid, cols[0].dtype)
    pos = 0
    for c in cols:                                  # CPU reference path
        n = c.length
        if n:
            o = off[pos:pos + n].contiguous()
            tot = int(c.lens.to(torch.int64).sum().item())
            if tot:
                # destination positions are contiguous from o[0]
                srcpos = torch.repeat_interleave(c.starts, c.lens.to(torch.int64)) + (
                    torch.arange(tot) - torch.repeat_interleave(o - o[0], c.lens.to(torch.int64)))
                dst[int(o[0]):int(o[0]) + tot] = c.arena[srcpos]
        pos += n
    return type(cols[0])(dst, off, lens.to(torch.int32), valid, cols[0].dtype)


def cmp_literal(col, lit: str, op: str) -> torch.Tensor:
    """Byte-wise comparison of every string against a literal → bool mask (nulls handled by the caller)."""
    code = _CMP_OPS[op]
    lb = lit.encode("utf-8")
    n = col.length
    if _gpu(col.starts):
        out = torch.empty(n, dtype=torch.bool, device=col.device)
        if n:
            lt = torch.frombuffer(bytearray(lb + b"\0"), dtype=torch.uint8).to(col.device, non_blocking=True)
            N.call("dxa_str_cmp_lit", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n, N.ptr(lt), len(lb),
                   code, N.ptr(out.view(torch.uint8)), N.stream_handle(col.device))
        return out
    vals = _raw_bytes(col)
    f = {
        0: lambda s: s == lb, 1: lambda s: s != lb, 2: lambda s: s < lb, 3: lambda s: s <= lb,
        4: lambda s: s > lb, 5: lambda s: s >= lb, 6: lambda s: s.startswith(lb), 7: lambda s: s.endswith(lb),
        8: lambda s: lb in s,
    }[code]
    return torch.tensor([f(s) for s in vals], dtype=torch.bool)


def like(col, tokens: List[int]) -> torch.Tensor:
    """General LIKE on the device (tokens from expr._like_tokens) → bool mask."""
    n = col.length
    out = torch.empty(n, dtype=torch.bool, device=col.device)
    if n:
        tk = torch.tensor(tokens or [0], dtype=torch.int16).to(col.device, non_blocking=True)
        N.call("dxa_str_like", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n, N.ptr(tk), len(tokens),
               N.ptr(out.view(torch.uint8)), N.stream_handle(col.device))
    return out


def rlike(col, dfa) -> torch.Tensor:
    """RLIKE on the device through a regex_dfa.DFA → bool mask."""
    n = col.length
    out = torch.empty(n, dtype=torch.bool, device=col.device)
    if n:
        blobs = dfa.__dict__.setdefault("_dev", {})
        blob = blobs.get(col.device)
        if blob is None:
            blob = torch.tensor(dfa.classes + [t - 0x10000 if t & 0x8000 else t for t in dfa.table],
                                dtype=torch.int16).to(col.device)
            blobs[col.device] = blob
        N.call("dxa_str_rlike", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n, N.ptr(blob),
               int(blob.numel()), dfa.n_classes, dfa.start, N.ptr(out.view(torch.uint8)), N.stream_handle(col.device))
    return out


_DIGEST_WIDTH = {0: 32, 1: 40, 2: 64, 3: 56}


def digest(col, kind: int):
    """md5 (0) / sha1 (1) / sha256 (2) / sha224 (3) of every row on the device → lower-case hex StrColumn."""
    from ..engine.column import StrColumn
    n, w = col.length, _DIGEST_WIDTH[kind]
    dev = col.device
    out = _alloc_arena(n * w, dev)
    if n:
        N.call("dxa_str_digest", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n, kind, N.ptr(out),
               N.stream_handle(dev))
    starts = torch.arange(n, dtype=torch.int64, device=dev) * w
    return StrColumn(out, starts, torch.full((n,), w, dtype=torch.int32, device=dev), col.valid)


def crc32(col) -> torch.Tensor:
    """CRC-32 of every row's bytes on the device → int64 tensor."""
    out = torch.empty(col.length, dtype=torch.int64, device=col.device)
    if col.length:
        N.call("dxa_str_crc32", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), col.length, N.ptr(out),
               N.stream_handle(col.device))
    return out


def encode(col, mode: int):
    """hex (0: upper-case, 2 chars per byte) / base64 (1: padded) of every row on the device → StrColumn."""
    from ..engine.column import StrColumn
    n, dev = col.length, col.device
    l64 = col.lens.to(torch.int64)
    out_lens = l64 * 2 if mode == 0 else (l64 + 2) // 3 * 4
    off, total = _offsets(out_lens)
    out = _alloc_arena(total, dev)
    if n:
        N.call("dxa_str_encode", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n, mode, N.ptr(off),
               N.ptr(out), N.stream_handle(dev))
    return StrColumn(out, off, out_lens.to(torch.int32), col.valid)


def _prefilter(col, prog):
    """RLIKE mask from the pattern's DFA (rows that cannot match skip the backtracking search), or None."""
    from . import regex_dfa
    pat = getattr(prog, "pattern", None)
    if pat is None:
        return None
    try:
        dfa = regex_dfa.compile_rlike(pat)
    except regex_dfa.Unsupported:
        return None
    return rlike(col, dfa)


def _vm_tensors(prog, device):
    cache = prog.__dict__.setdefault("_dev", {})
    t = cache.get(device)
    if t is None:
        t = cache[device] = (N.h2d(prog.code, torch.int32, device), N.h2d(prog.sets, torch.int32, device))
    return t


def regex_extract(col, prog, group: int):
    """regexp_extract on the device: views into the source arena (no copy).  Returns (StrColumn, fallback mask)
    — rows whose match exceeded the kernel's backtracking budget are flagged for the host."""
    from ..engine.column import StrColumn
    n, dev = col.length, col.device
    code, sets = _vm_tensors(prog, dev)
    starts = torch.empty(n, dtype=torch.int64, device=dev)
    lens = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    if n:
        hit = _prefilter(col, prog)
        N.call("dxa_str_regex", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n, N.ptr(code),
               code.numel() // 4, N.ptr(sets), sets.numel() // 8, 0, group, 0, 0, N.ptr(starts), N.ptr(lens), 0, 0,
               N.ptr(status), N.ptr(hit), N.stream_handle(dev))
    return StrColumn(col.arena, starts, lens, col.valid), status.bool()


def regex_replace(col, prog, tokens: List[int]):
    """regexp_replace on the device (length pass, scan, write pass) → (StrColumn, fallback mask)."""
    from ..engine.column import StrColumn
    n, dev = col.length, col.device
    code, sets = _vm_tensors(prog, dev)
    rep = N.h2d(tokens or [0], torch.int32, dev)
    lens = torch.zeros(n, dtype=torch.int32, device=dev)
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    st = N.stream_handle(dev)
    args = (N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n, N.ptr(code), code.numel() // 4, N.ptr(sets),
            sets.numel() // 8)
    hit = _prefilter(col, prog) if n else None
    if n:
        N.call("dxa_str_regex", *args, 1, 0, N.ptr(rep), len(tokens), 0, N.ptr(lens), 0, 0, N.ptr(status),
               N.ptr(hit), st)
    off, total = _offsets(lens)
    out = _alloc_arena(total, dev)
    if n and total:
        N.call("dxa_str_regex", *args, 2, 0, N.ptr(rep), len(tokens), 0, 0, N.ptr(off), N.ptr(out), N.ptr(status),
               N.ptr(hit), st)
    return StrColumn(out, off, lens, col.valid), status.bool()


def _raw_bytes(col) -> List[bytes]:
    arena = col.arena.cpu().numpy().tobytes()
    return [arena[s:s + l] for s, l in zip(col.starts.cpu().tolist(), col.lens.cpu().tolist())]


def eq_columns(a, b) -> torch.Tensor:
    n = a.length
    if _gpu(a.starts):
        out = torch.empty(n, dtype=torch.bool, device=a.device)
        if n:
            N.call("dxa_str_eq_col", N.ptr(a.arena), N.ptr(a.starts), N.ptr(a.lens), N.ptr(b.arena), N.ptr(b.starts),
                   N.ptr(b.lens), n, N.ptr(out.view(torch.uint8)), N.stream_handle(a.device))
        return out
    return torch.tensor([x == y for x, y in zip(_raw_bytes(a), _raw_bytes(b))], dtype=torch.bool)


def compare_columns(a, b, op: str) -> torch.Tensor:
    """Row-wise string column comparison, byte-wise (UTF-8 code point) order; nulls are the caller's (their rows
    compare as empty strings here)."""
    if op in ("=", "!="):
        eq = eq_columns(a, b)
        return eq if op == "=" else ~eq
    if _gpu(a.starts):
        from .sort import _safe_lens
        n = a.length
        out = torch.empty(n, dtype=torch.bool, device=a.device)
        if n:
            al, bl = _safe_lens(a), _safe_lens(b)
            N.call("dxa_str_cmp_col", N.ptr(a.arena), N.ptr(a.starts.to(torch.int64).contiguous()), N.ptr(al),
                   N.ptr(b.arena), N.ptr(b.starts.to(torch.int64).contiguous()), N.ptr(bl), n, _CMP_OPS[op],
                   N.ptr(out.view(torch.uint8)), N.stream_handle(a.device))
        return out
    va, vb = _raw_bytes(a), _raw_bytes(b)
    f = {"<": lambda x, y: x < y, "<=": lambda x, y: x <= y, ">": lambda x, y: x > y, ">=": lambda x, y: x >= y}[op]
    return N.h2d([f(x, y) for x, y in zip(va, vb)], torch.bool, a.device)


class _ConcatPart(ctypes.Structure):
    _fields_ = [("arena", ctypes.c_void_p), ("starts", ctypes.c_void_p), ("lens", ctypes.c_void_p),
                ("valid", ctypes.c_void_p), ("lit", ctypes.c_void_p), ("lit_len", ctypes.c_int32),
                ("is_lit", ctypes.c_int32)]


def concat_strings(parts: List[Union[str, object]], n: int, device):
    """CONCAT over string columns and literals (Spark: any null input → null)."""
    from ..engine.column import StrColumn, and_valid
    device = torch.device(device)
    if device.type == "cuda":
        arr, keep, raw = _concat_parts(parts, device)
        lens = torch.empty(n, dtype=torch.int64, device=device)
        ok = torch.empty(n, dtype=torch.bool, device=device)
        st = N.stream_handle(device)
        N.call("dxa_concat_len", N.ptr(raw), len(parts), n, N.ptr(lens), N.ptr(ok.view(torch.uint8)), st)
        bound = _concat_bound(parts, n)
        if bound is not None:
            # every part has a known per-row maximum (literals, fixed-slot conversions): allocate that, no host read
            off = torch.cumsum(lens, 0) - lens if n else lens
            dst = _alloc_arena(bound, device)
        else:
            off, total = _offsets(lens)
            dst = _alloc_arena(total, device)
        N.call("dxa_concat_write", N.ptr(raw), len(parts), n, N.ptr(off), N.ptr(ok.view(torch.uint8)), N.ptr(dst), st)
        valid = None if all(isinstance(p, str) or p.valid is None for p in parts) else ok
        col = StrColumn(dst, off, lens.to(torch.int32), valid)
        col._keep = (keep, raw)
        return col
    cols = [None if isinstance(p, str) else p.to_pylist() for p in parts]
    out = []
    for i in range(n):
        s = []
        null = False
        for p, c in zip(parts, cols):
            if c is None:
                s.append(p)
            elif c[i] is None:
                null = True
                break
            else:
                s.append(c[i])
        out.append(None if null else "".join(s))
    from ..engine.column import strings_from_pylist
    return strings_from_pylist(out, device)


def _concat_parts(parts, device):
    """The part descriptors and every literal's bytes in ONE device buffer (one upload): descriptors first, then the
    literals, whose device addresses are known once the buffer is allocated."""
    arr = (_ConcatPart * len(parts))()
    head = ctypes.sizeof(arr)
    lits, pos = [], head
    for p in parts:
        if isinstance(p, str):
            b = p.encode("utf-8") + b"\0"
            lits.append((pos, b))
            pos += len(b)
    raw = torch.empty(pos, dtype=torch.uint8, device=device)
    base = raw.data_ptr()
    keep = []
    li = 0
    for i, p in enumerate(parts):
        if isinstance(p, str):
            off, b = lits[li]
            li += 1
            arr[i] = _ConcatPart(0, 0, 0, 0, base + off, len(b) - 1, 1)
        else:
            v = N.u8(p.valid)
            keep.append(v)
            arr[i] = _ConcatPart(p.arena.data_ptr(), p.starts.data_ptr(), p.lens.data_ptr(),
                                 0 if v is None else v.data_ptr(), 0, 0, 0)
    blob = bytearray(bytes(arr))
    for off, b in lits:
        blob += b
    raw.copy_(torch.frombuffer(blob, dtype=torch.uint8).pin_memory(), non_blocking=True)
    return arr, keep, raw


def _concat_bound(parts, n: int):
    """Upper bound of a CONCAT's total bytes when every column part carries ``_max_len`` (bytes per row)."""
    tot = 0
    for p in parts:
        if isinstance(p, str):
            tot += len(p.encode("utf-8"))
        else:
            m = getattr(p, "_max_len", None)
            if m is None:
                return None
            tot += m
    return tot * n


def concat_ws(sep: str, parts: List[Union[str, object]], n: int, device):
    """concat_ws on the device: null column parts are skipped (Spark), the separator joins what remains."""
    from ..engine.column import StrColumn
    device = torch.device(device)
    arr, keep, raw = _concat_parts(parts, device)
    sb = sep.encode("utf-8")
    st_ = N.h2d(sb + b"\0", torch.uint8, device)
    lens = torch.empty(n, dtype=torch.int64, device=device)
    st = N.stream_handle(device)
    N.call("dxa_concat_ws_len", N.ptr(raw), len(parts), n, len(sb), N.ptr(lens), st)
    off, total = _offsets(lens)
    dst = _alloc_arena(total, device)
    N.call("dxa_concat_ws_write", N.ptr(raw), len(parts), n, N.ptr(st_), len(sb), N.ptr(off), N.ptr(dst), st)
    col = StrColumn(dst, off, lens.to(torch.int32), None)
    col._keep = (keep, raw, st_)
    return col


def from_int64(data: torch.Tensor, valid):
    """CAST(long AS STRING)."""
    from ..engine.column import StrColumn, strings_from_pylist
    n = data.shape[0]
    if _gpu(data):
        # fixed 24-byte slots: one launch, no host read (a compact copy is made only if the column is retained)
        dev = data.device
        dst = torch.empty(n * 24 + 16, dtype=torch.uint8, device=dev)
        starts = torch.empty(n, dtype=torch.int64, device=dev)
        lens = torch.empty(n, dtype=torch.int32, device=dev)
        N.call("dxa_i64_to_str_slots", N.ptr(data.to(torch.int64).contiguous()), n, N.ptr(dst), N.ptr(starts),
               N.ptr(lens), N.stream_handle(dev))
        out = StrColumn(dst, starts, lens, valid)
        out._max_len = 20
        return out
    vals = data.tolist()
    v = valid.tolist() if valid is not None else [True] * n
    return strings_from_pylist([str(x) if ok else None for x, ok in zip(vals, v)], data.device)


def case_map(col, upper: bool):
    from ..engine.column import StrColumn, strings_from_pylist
    n = col.length
    if _gpu(col.starts):
        off, total = _offsets(col.lens)
        dst = _alloc_arena(total, col.device)
        N.call("dxa_case_map", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n, N.ptr(off), N.ptr(dst),
               1 if upper else 0, N.stream_handle(col.device))
        return StrColumn(dst, off, col.lens.clone(), col.valid)
    vals = col.to_pylist()
    return strings_from_pylist([None if v is None else (_ascii_upper(v) if upper else _ascii_lower(v))
                                for v in vals], col.device)


def _ascii_upper(s):
    return "".join(c.upper() if "a" <= c <= "z" else c for c in s)


def _ascii_lower(s):
    return "".join(c.lower() if "A" <= c <= "Z" else c for c in s)


_TS_A = re.compile(r"^(\d{4})-(\d{1,2})-(\d{1,2}) (\d{1,2}):(\d{1,2}):(\d{1,2})(?:\.(\d+))?$")
_TS_B = re.compile(r"^(\d{4})-(\d{1,2})-(\d{1,2})T(\d{1,2}):(\d{1,2}):(\d{1,2})Z$")
_TS_C = re.compile(r"^(\d{1,2})/(\d{1,2})/(\d{4}) (\d{1,2}):(\d{1,2}):(\d{1,2})$")


def py_string_to_timestamp_us(s: Optional[str]) -> Optional[int]:
    """Reference semantics of DataX's ``stringToTimestamp`` (ConcurrentDateFormat.scala:38-62), UTC."""
    if not s:
        return None
    frac = 0
    m = _TS_A.match(s)
    if m:
        y, mo, d, hh, mi, ss = (int(x) for x in m.groups()[:6])
        if m.group(7):
            frac = int((m.group(7) + "000000")[:6])
    else:
        m = _TS_B.match(s)
        if m:
            y, mo, d, hh, mi, ss = (int(x) for x in m.groups())
        else:
            m = _TS_C.match(s)
            if not m:
                return None
            mo, d, y, hh, mi, ss = (int(x) for x in m.groups())
    if not (1 <= mo <= 12 and 1 <= d <= 31 and hh <= 23 and mi <= 59 and ss <= 59):
        return None
    try:
        days = (_dt.date(y, mo, 1) - _dt.date(1970, 1, 1)).days + d - 1
    except ValueError:
        return None
    return (days * 86400 + hh * 3600 + mi * 60 + ss) * 1_000_000 + frac


def to_timestamp(col):
    from ..engine.column import PrimColumn
    n = col.length
    if _gpu(col.starts):
        out = torch.empty(n, dtype=torch.int64, device=col.device)
        ok = torch.empty(n, dtype=torch.bool, device=col.device)
        N.call("dxa_str_to_ts", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), N.ptr(N.u8(col.valid)), n,
               N.ptr(out), N.ptr(ok.view(torch.uint8)), N.stream_handle(col.device))
        return PrimColumn("timestamp", out, ok)
    vals = [py_string_to_timestamp_us(v) for v in col.to_pylist()]
    data = torch.tensor([0 if v is None else v for v in vals], dtype=torch.int64)
    return PrimColumn("timestamp", data, torch.tensor([v is not None for v in vals], dtype=torch.bool))
