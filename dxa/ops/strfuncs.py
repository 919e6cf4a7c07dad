"""Device paths of Spark string built-ins (dxa/ops/csrc/strfuncs.hip): lpad / rpad, reverse, repeat, translate,
initcap, ascii, substring_index, levenshtein.  Inputs are device ``StrColumn``s with constant extra arguments; every
function returns a column (or None when the kernel flagged rows it does not handle — the caller then takes the host
path for the whole column, which is the CPU evaluator's code and so the differential tests' oracle).

Small constant arguments (pad text, translate tables, delimiters) go up through pinned staging buffers with
non-blocking copies: a pageable host→device copy would stall the host behind the stream."""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import native as N
from .strings import _alloc_arena, _offsets

c_p, c_i32, c_i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
N.register_sigs({
    "dxa_pad_args_size": [],
    "dxa_str_pad": [c_p, c_p, c_p, c_p, c_p],
    "dxa_str_reverse": [c_p, c_p, c_p, c_i64, c_p, c_p, c_p],
    "dxa_str_repeat": [c_p, c_p, c_p, c_i64, c_i64, c_p, c_p, c_p],
    "dxa_str_translate": [c_p, c_p, c_p, c_i64, c_p, c_p, c_i32, c_p, c_p, c_p, c_p],
    "dxa_str_initcap": [c_p, c_p, c_p, c_i64, c_p, c_p, c_p, c_p],
    "dxa_str_substring_index": [c_p, c_p, c_p, c_i64, c_p, c_i32, c_i64, c_p, c_p, c_p],
    "dxa_str_levenshtein": [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_p],
})


def upload(data, dtype, device) -> torch.Tensor:
    """A small host array on the device without stalling the host: pinned staging (torch's caching host
    allocator keeps the block until the copy has run) + a non-blocking copy."""
    if isinstance(data, (bytes, bytearray)):
        h = torch.frombuffer(bytearray(data) if data else bytearray(1), dtype=torch.uint8)
    else:
        h = torch.tensor(list(data) if len(data) else [0], dtype=dtype)
    return h.pin_memory().to(device, non_blocking=True)


def _st(col):
    return N.stream_handle(col.device)


def _out_col(col, arena, off, lens):
    from ..engine.column import StrColumn
    return StrColumn(arena, off, lens.to(torch.int32), col.valid)


class _PadArgs(ctypes.Structure):
    _fields_ = [("arena", c_p), ("starts", c_p), ("lens", c_p), ("n", c_i64), ("target", c_i64), ("pad", c_p),
                ("pad_len", c_i32), ("pad_chars", c_i32), ("pad_off", c_p), ("left", c_i32), ("pad_", c_i32)]


def pad(col, target: int, pad_text: str, left: bool):
    """lpad / rpad (UTF8String.lpad / rpad): cut to ``target`` characters, or fill with ``pad_text`` repeated."""
    if N.lib().dxa_pad_args_size() != ctypes.sizeof(_PadArgs):
        raise N.NativeError("PadArgs layout mismatch between strfuncs.py and strfuncs.hip")
    dev = col.device
    pb = pad_text.encode("utf-8")
    offs = [0]
    for ch in pad_text:
        offs.append(offs[-1] + len(ch.encode("utf-8")))
    pbuf = upload(pb, torch.uint8, dev)
    poff = upload(offs, torch.int32, dev)
    a = _PadArgs(col.arena.data_ptr(), col.starts.data_ptr(), col.lens.data_ptr(), col.length, int(target),
                 pbuf.data_ptr(), len(pb), len(pad_text), poff.data_ptr(), 1 if left else 0, 0)
    lens = torch.empty(col.length, dtype=torch.int64, device=dev)
    N.call("dxa_str_pad", ctypes.byref(a), None, N.ptr(lens), None, _st(col))
    off, total = _offsets(lens)
    dst = _alloc_arena(total, dev)
    N.call("dxa_str_pad", ctypes.byref(a), N.ptr(off), None, N.ptr(dst), _st(col))
    out = _out_col(col, dst, off, lens)
    out._keep = (pbuf, poff)
    return out


def reverse(col):
    off, total = _offsets(col.lens)
    dst = _alloc_arena(total, col.device)
    N.call("dxa_str_reverse", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), col.length, N.ptr(off),
           N.ptr(dst), _st(col))
    return _out_col(col, dst, off, col.lens)


def repeat(col, times: int):
    times = max(0, int(times))
    lens = col.lens.to(torch.int64) * times
    off, total = _offsets(lens)
    dst = _alloc_arena(total, col.device)
    N.call("dxa_str_repeat", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), col.length, times, N.ptr(off),
           N.ptr(dst), _st(col))
    return _out_col(col, dst, off, lens)


def translate(col, matching: str, replace: str):
    """translate(src, matching, replace): the i-th character of ``matching`` becomes the i-th of ``replace``, or is
    deleted when ``replace`` is shorter; the first occurrence of a repeated character wins (Spark's map build)."""
    dev = col.device
    frm, to, seen = [], [], set()
    for i, ch in enumerate(matching):
        if ch in seen:
            continue
        seen.add(ch)
        frm.append(ord(ch))
        to.append(ord(replace[i]) if i < len(replace) else -1)
    tf = upload(frm, torch.int32, dev)
    tt = upload(to, torch.int32, dev)
    lens = torch.empty(col.length, dtype=torch.int64, device=dev)
    args = (N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), col.length, N.ptr(tf), N.ptr(tt), len(frm))
    N.call("dxa_str_translate", *args, None, N.ptr(lens), None, _st(col))
    off, total = _offsets(lens)
    dst = _alloc_arena(total, dev)
    N.call("dxa_str_translate", *args, N.ptr(off), None, N.ptr(dst), _st(col))
    out = _out_col(col, dst, off, lens)
    out._keep = (tf, tt)
    return out


def initcap(col):
    """None when a row holds non-ASCII bytes (Java's Unicode case mapping: host path)."""
    off, total = _offsets(col.lens)
    dst = _alloc_arena(total, col.device)
    bad = torch.zeros(1, dtype=torch.int32, device=col.device)
    N.call("dxa_str_initcap", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), col.length, N.ptr(off),
           N.ptr(dst), N.ptr(bad), _st(col))
    if int(bad.item()):
        return None
    return _out_col(col, dst, off, col.lens)


def ascii_code(col):
    """Spark 2.4 ``ascii``: the first BYTE of the UTF-8 encoding as a signed int (``getBytes()(0)``), 0 for ''."""
    from ..engine.column import PrimColumn
    n = col.length
    first = col.arena[col.starts.clamp(min=0, max=max(0, col.arena.shape[0] - 1))] if n else \
        torch.zeros(0, dtype=torch.uint8, device=col.device)
    v = first.view(torch.int8).to(torch.int32)
    return PrimColumn("int", torch.where(col.lens > 0, v, torch.zeros_like(v)), col.valid)


def substring_index(col, delim: str, count: int):
    from ..engine.column import StrColumn
    dev = col.device
    db = delim.encode("utf-8")
    dt = upload(db, torch.uint8, dev)
    st = torch.empty(col.length, dtype=torch.int64, device=dev)
    ln = torch.empty(col.length, dtype=torch.int32, device=dev)
    N.call("dxa_str_substring_index", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), col.length, N.ptr(dt),
           len(db), int(count), N.ptr(st), N.ptr(ln), _st(col))
    out = StrColumn(col.arena, st, ln, col.valid)
    out._keep = dt
    return out


def levenshtein(a, b) -> Optional[object]:
    """None when a row is non-ASCII or longer than the kernel's 128-character DP rows (host path)."""
    from ..engine.column import PrimColumn, and_valid
    out = torch.empty(a.length, dtype=torch.int32, device=a.device)
    bad = torch.zeros(1, dtype=torch.int32, device=a.device)
    N.call("dxa_str_levenshtein", N.ptr(a.arena), N.ptr(a.starts), N.ptr(a.lens), N.ptr(b.arena), N.ptr(b.starts),
           N.ptr(b.lens), a.length, N.ptr(out), N.ptr(bad), _st(a))
    if int(bad.item()):
        return None
    return PrimColumn("int", out, and_valid(a.valid, b.valid))


# ---- number ↔ text and codecs (dxa/ops/csrc/strconv.hip) ----------------------------------------------------------

N.register_sigs({
    "dxa_format_number": [c_p, c_i32, c_p, c_i64, c_i32, c_p, c_p, c_p, c_p, c_p],
    "dxa_conv": [c_p, c_p, c_p, c_p, c_i64, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p],
    "dxa_bin": [c_p, c_i64, c_p, c_p, c_p, c_p],
    "dxa_soundex": [c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_p],
    "dxa_str_decode": [c_p, c_p, c_p, c_p, c_i64, c_i32, c_p, c_p, c_p, c_p, c_p, c_p],
    "dxa_split_part": [c_p, c_p, c_p, c_i64, c_p, c_i32, c_i64, c_p, c_p, c_p],
    "dxa_utf8_clean": [c_p, c_p, c_p, c_i64, c_p, c_p, c_p, c_p, c_p],
})
FMT_SLOT, CONV_SLOT = 64, 66


def _slots(n, width, dev):
    return (torch.empty(n * width + 16, dtype=torch.uint8, device=dev),
            torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int32, device=dev))


def format_number(col, d: int):
    """format_number(x, d) over a device double / integral column; None when a row needs the host (|x| ≥ 10^18,
    NaN / ±Inf) — one 4-byte flag read."""
    from ..engine.column import StrColumn
    dev, n = col.device, col.length
    if d < 0 or d > 38:
        return None
    f64 = col.data.dtype in (torch.float64, torch.float32)
    data = col.data.to(torch.float64 if f64 else torch.int64).contiguous()
    arena, starts, lens = _slots(n, FMT_SLOT, dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    N.call("dxa_format_number", N.ptr(data), 1 if f64 else 0, N.ptr(N.u8(col.valid)), n, int(d), N.ptr(arena),
           N.ptr(starts), N.ptr(lens), N.ptr(bad), N.stream_handle(dev))
    if int(bad.item()):
        return None
    return StrColumn(arena, starts, lens, col.valid)


def conv(col, from_base: int, to_base: int):
    from ..engine.column import StrColumn
    dev, n = col.device, col.length
    out, starts, lens = _slots(n, CONV_SLOT, dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    N.call("dxa_conv", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), N.ptr(N.u8(col.valid)), n,
           int(from_base), int(to_base), N.ptr(out), N.ptr(starts), N.ptr(lens), N.ptr(ok), _st(col))
    return StrColumn(out, starts, lens, ok.view(torch.bool))


def bin_text(col):
    from ..engine.column import StrColumn
    dev, n = col.device, col.length
    out, starts, lens = _slots(n, CONV_SLOT, dev)
    N.call("dxa_bin", N.ptr(col.data.to(torch.int64).contiguous()), n, N.ptr(out), N.ptr(starts), N.ptr(lens),
           N.stream_handle(dev))
    return StrColumn(out, starts, lens, col.valid)


def soundex(col):
    """None when some row's first byte is not an ASCII letter (Spark returns those inputs unchanged)."""
    from ..engine.column import StrColumn
    dev, n = col.device, col.length
    out, starts, lens = _slots(n, 4, dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    N.call("dxa_soundex", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), N.ptr(N.u8(col.valid)), n,
           N.ptr(out), N.ptr(starts), N.ptr(lens), N.ptr(bad), _st(col))
    if int(bad.item()):
        return None
    return StrColumn(out, starts, lens, col.valid)


def decode(col, mode: int):
    """unhex (mode 0) / unbase64 (mode 1): the decoded bytes as text (ill-formed UTF-8 → U+FFFD, utf8_clean)."""
    from ..engine.column import StrColumn
    dev, n = col.device, col.length
    lens = torch.empty(n, dtype=torch.int64, device=dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    args = (N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), N.ptr(N.u8(col.valid)), n, mode)
    N.call("dxa_str_decode", *args, None, None, N.ptr(lens), N.ptr(ok), N.ptr(bad), _st(col))
    off, total = _offsets(lens)
    dst = _alloc_arena(total, dev)
    N.call("dxa_str_decode", *args, N.ptr(off), N.ptr(dst), N.ptr(lens), N.ptr(ok), N.ptr(bad), _st(col))
    return utf8_clean(StrColumn(dst, off, lens.to(torch.int32), ok.view(torch.bool)))


def utf8_clean(col):
    """Bytes → text as Python's ``bytes.decode("utf-8", errors="replace")`` renders them: the column itself when it is
    already well-formed UTF-8 (one read of the changed-row count), else a rewritten copy."""
    from ..engine.column import StrColumn
    dev, n = col.device, col.length
    if n == 0:
        return col
    lens = torch.empty(n, dtype=torch.int64, device=dev)
    changed = torch.zeros(1, dtype=torch.int32, device=dev)
    a = (N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n)
    N.call("dxa_utf8_clean", *a, None, None, N.ptr(lens), N.ptr(changed), _st(col))
    cs = torch.cumsum(lens, 0)
    total, nchanged = torch.stack([cs[-1], changed[0].to(torch.int64)]).tolist()
    if not nchanged:
        return col
    off = cs - lens
    dst = _alloc_arena(int(total), dev)
    N.call("dxa_utf8_clean", *a, N.ptr(off), N.ptr(dst), None, None, _st(col))
    return StrColumn(dst, off, lens.to(torch.int32), col.valid)


def split_part(col, delim: str, k: int):
    from ..engine.column import StrColumn
    if k == 0:
        raise ValueError("split_part: the field index must not be 0")
    dev, n = col.device, col.length
    db = delim.encode("utf-8")
    dl = upload(db, torch.uint8, dev)
    st = torch.empty(n, dtype=torch.int64, device=dev)
    ln = torch.empty(n, dtype=torch.int32, device=dev)
    N.call("dxa_split_part", N.ptr(col.arena), N.ptr(col.starts), N.ptr(col.lens), n, N.ptr(dl), len(db), int(k),
           N.ptr(st), N.ptr(ln), _st(col))
    out = StrColumn(col.arena, st, ln, col.valid)
    out._keep = dl
    return out
