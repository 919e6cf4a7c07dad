"""Sorting on the device (kernel K14): stable LSD radix argsort over multi-word uint64 keys
(``radix_sort.hip``), order keys for SQL types, and dense ranks of string columns.

The SQL layer (ORDER BY, window functions, string comparisons in sorts) reduces every sort to
``argsort_words(words)``: ``words[0]`` is the least significant 64-bit word, each word an int64 tensor holding the
bits of an *unsigned* key.  One byte histogram of every word (a single read, one host synchronisation for all words)
tells the driver which bytes are constant over the input; only the others get a radix pass.  On the CPU the same
contract is served by successive stable ``torch.argsort`` calls (the reference implementation the GPU tests compare
against).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from . import native as N

N.register_sigs({
    "dxa_rs_tile": [],
    "dxa_rs_byte_hist": [N.c_p, N.c_i64, N.c_p, N.c_p],
    "dxa_rs_pass": [N.c_p, N.c_p, N.c_i64, N.c_i32, N.c_p, N.c_p, N.c_p, N.c_p, N.c_p, N.c_p],
    "dxa_order_key": [N.c_p, N.c_i64, N.c_i32, N.c_i32, N.c_p, N.c_p],
    "dxa_str_chunk": [N.c_p, N.c_p, N.c_p, N.c_p, N.c_i64, N.c_i32, N.c_p, N.c_p],
})

_TILE = 4096
_SIGN = -(1 << 63)           # int64 with only the top bit set


def _as_signed_order(w: torch.Tensor) -> torch.Tensor:
    """uint64 bits in an int64 tensor → int64 values with the same order (flip the top bit)."""
    return w ^ _SIGN


def argsort_words(words: Sequence[torch.Tensor]) -> torch.Tensor:
    """Stable argsort by the unsigned multi-word key ``(words[-1], ..., words[0])`` (``words[0]`` least significant)
    → int64 permutation."""
    words = [w.contiguous().view(torch.int64) if w.dtype != torch.int64 else w.contiguous() for w in words]
    if not words:
        raise ValueError("argsort_words needs at least one key word")
    n = int(words[0].shape[0])
    dev = words[0].device
    if dev.type != "cuda":
        perm = torch.arange(n, dtype=torch.int64)
        for w in words:
            perm = perm[torch.argsort(_as_signed_order(w[perm]), stable=True)]
        return perm
    if n <= 1:
        return torch.arange(n, dtype=torch.int64, device=dev)
    st = N.stream_handle(dev)
    # which bytes vary: one histogram kernel per word, one read-back for all of them
    hists = torch.empty((len(words), 8, 256), dtype=torch.int64, device=dev)
    for j, w in enumerate(words):
        N.call("dxa_rs_byte_hist", N.ptr(w), n, N.ptr(hists[j]), st)
    varying = (hists.amax(dim=2) < n).tolist()
    ntiles = (n + _TILE - 1) // _TILE
    m = ntiles * 256
    counts = torch.empty(m, dtype=torch.int32, device=dev)
    offsets = torch.empty(m, dtype=torch.int64, device=dev)
    sums = torch.empty((m + 4095) // 4096, dtype=torch.int64, device=dev)
    kb = torch.empty(n, dtype=torch.int64, device=dev)
    vb = torch.empty(n, dtype=torch.int64, device=dev)
    perm: Optional[torch.Tensor] = None
    for w, vary in zip(words, varying):
        if not any(vary):
            continue
        key = w if perm is None else w[perm]
        if perm is None:
            ka, va = key.clone(), None
        else:
            ka, va = key, perm
        for b in range(8):
            if not vary[b]:
                continue
            N.call("dxa_rs_pass", N.ptr(ka), N.ptr(va) if va is not None else None, n, 8 * b, N.ptr(counts),
                   N.ptr(offsets), N.ptr(sums), N.ptr(kb), N.ptr(vb), st)
            # ping-pong: the pass output becomes the next input
            if va is None:
                va = vb
                vb = torch.empty(n, dtype=torch.int64, device=dev)
            else:
                va, vb = vb, va
            ka, kb = kb, ka
        perm = va
    return perm if perm is not None else torch.arange(n, dtype=torch.int64, device=dev)


# -- order keys ----------------------------------------------------------------------------------------------------

def order_key(data: torch.Tensor, kind: str, descending: bool = False) -> torch.Tensor:
    """uint64 order key (as int64 bits) of a primitive column: ``kind`` ``"int"`` (two's complement integers,
    booleans, timestamps, dates), ``"float"`` (IEEE doubles; NaN largest, -0.0 == 0.0 as in Spark)."""
    if data.dtype == torch.bool or data.dtype in (torch.int8, torch.int16, torch.int32, torch.uint8):
        data = data.to(torch.int64)
    elif data.dtype == torch.float32:
        data = data.to(torch.float64)
    bits = data.contiguous().view(torch.int64)
    code = 1 if kind == "float" else 0
    if bits.device.type == "cuda":
        out = torch.empty_like(bits)
        if bits.numel():
            N.call("dxa_order_key", N.ptr(bits), bits.numel(), code, 1 if descending else 0, N.ptr(out),
                   N.stream_handle(bits.device))
        return out
    return _order_key_cpu(bits, code, descending)


def _order_key_cpu(bits: torch.Tensor, code: int, descending: bool) -> torch.Tensor:
    v = bits.clone()
    if code == 0:
        v ^= _SIGN
    else:
        mag = v & 0x7fffffffffffffff
        nan = mag > 0x7ff0000000000000
        v = torch.where(nan, torch.full_like(v, 0x7ff8000000000000), v)
        v = torch.where(v == _SIGN, torch.zeros_like(v), v)          # -0.0 → 0.0
        neg = v < 0
        v = torch.where(neg, ~v, v | _SIGN)
    return ~v if descending else v


# -- strings -------------------------------------------------------------------------------------------------------

def _safe_lens(col) -> torch.Tensor:
    """int32 lengths with null rows as empty strings (a null slot's start/length are not meaningful)."""
    lens = col.lens.to(torch.int32)
    if col.valid is not None:
        lens = torch.where(col.valid, lens, torch.zeros_like(lens))
    return lens.contiguous()


def string_chunk(col, chunk: int, rows: Optional[torch.Tensor] = None,
                 lens: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Big-endian 8-byte chunk ``chunk`` of every string (zero-padded past its end) as uint64 bits; ``rows`` picks
    the rows (default: all), ``lens`` overrides the column's lengths (``_safe_lens``)."""
    lens = _safe_lens(col) if lens is None else lens
    n = int(rows.shape[0]) if rows is not None else col.length
    starts = col.starts.to(torch.int64).contiguous()
    if starts.device.type == "cuda":
        out = torch.empty(n, dtype=torch.int64, device=col.device)
        if n:
            N.call("dxa_str_chunk", N.ptr(col.arena), N.ptr(starts), N.ptr(lens),
                   N.ptr(rows.contiguous()) if rows is not None else None, n, chunk, N.ptr(out),
                   N.stream_handle(col.device))
        return out
    arena = col.arena
    idx = rows if rows is not None else torch.arange(n, dtype=torch.int64)
    st, ln = starts[idx], lens[idx].to(torch.int64)
    v = torch.zeros(n, dtype=torch.int64)
    for b in range(8):
        pos = chunk * 8 + b
        inside = pos < ln
        at = torch.where(inside, st + pos, torch.zeros_like(st))
        byte = torch.where(inside, arena[at].to(torch.int64), torch.zeros_like(st))
        v |= byte << (56 - 8 * b)
    return v


def string_ranks(col) -> torch.Tensor:
    """Dense rank of every string in byte-wise (UTF-8 code point) order: equal strings share a rank, rank order =
    string order.  Rows are ordered by their first 8 bytes with one radix sort; then only rows still tied with a
    neighbour are refined by their next 8 bytes (sorting (rank, chunk) pairs), until no tie has bytes left; the
    remaining ties (one string is the other plus NUL bytes) are broken by length.  Null rows get an arbitrary rank."""
    n = col.length
    dev = col.device
    if n == 0:
        return torch.zeros(0, dtype=torch.int64, device=dev)
    safe = _safe_lens(col)
    lens = safe.to(torch.int64)
    perm = argsort_words([string_chunk(col, 0, lens=safe)])
    key_sorted = string_chunk(col, 0, perm, safe)
    boundary = torch.ones(n, dtype=torch.bool, device=dev)
    boundary[1:] = key_sorted[1:] != key_sorted[:-1]
    chunk = 1
    lens_sorted = lens[perm]
    while True:
        rank_sorted = torch.cumsum(boundary.to(torch.int64), 0)
        tied = ~boundary.clone()
        tied[:-1] |= ~boundary[1:]                   # first row of a tied run
        need = tied & (lens_sorted > 8 * chunk)
        # a run needs refining if any member still has bytes beyond the chunks compared so far
        run_need = torch.zeros(n + 1, dtype=torch.int64, device=dev).index_add_(
            0, rank_sorted, need.to(torch.int64))[rank_sorted] > 0
        active = torch.nonzero(tied & run_need).flatten()
        if active.numel() == 0:
            break
        rows = perm[active]
        ck = string_chunk(col, chunk, rows, safe)
        sub = argsort_words([ck, rank_sorted[active]])
        perm[active] = rows[sub]
        ck = ck[sub]
        ra = rank_sorted[active][sub]
        nb = torch.zeros(active.numel(), dtype=torch.bool, device=dev)
        nb[1:] = (ck[1:] != ck[:-1]) | (ra[1:] != ra[:-1])
        nb[0] = boundary[active[0]]
        boundary[active] = nb | boundary[active]
        lens_sorted = lens[perm]
        chunk += 1
    # ties left: equal chunks everywhere; a shorter string (a prefix padded with NULs) sorts first
    rank_sorted = torch.cumsum(boundary.to(torch.int64), 0)
    tied = ~boundary.clone()
    tied[:-1] |= ~boundary[1:]
    active = torch.nonzero(tied).flatten()
    if active.numel():
        la = lens_sorted[active]
        ra = rank_sorted[active]
        sub = argsort_words([la, ra])
        perm[active] = perm[active][sub]
        la, ra = la[sub], ra[sub]
        nb = torch.zeros(active.numel(), dtype=torch.bool, device=dev)
        nb[1:] = (la[1:] != la[:-1]) | (ra[1:] != ra[:-1])
        nb[0] = boundary[active[0]]
        boundary[active] = nb | boundary[active]
        rank_sorted = torch.cumsum(boundary.to(torch.int64), 0)
    ranks = torch.empty(n, dtype=torch.int64, device=dev)
    ranks[perm] = rank_sorted - 1
    return ranks


# -- SQL sort specs ------------------------------------------------------------------------------------------------

def column_order_key(col, descending: bool = False):
    """(uint64 order key as int64 bits, valid bool) of a materialised column; null rows get key 0 (so they keep
    their relative order from more significant keys)."""
    from ..engine.column import PrimColumn, StrColumn
    if isinstance(col, StrColumn):
        key = order_key(string_ranks(col), "int", descending)
    elif isinstance(col, PrimColumn) and col.data.dim() == 2:
        # wide decimal(p > 18): dense ranks of the signed 128-bit values — (hi, lo ^ sign) sorts lexicographically
        # as signed words in exactly the 128-bit order
        hl = torch.stack([col.data[:, 1], col.data[:, 0] ^ (-(1 << 63))], 1)
        ranks = torch.unique(hl, dim=0, return_inverse=True)[1].to(torch.int64)
        key = order_key(ranks, "int", descending)
    elif isinstance(col, PrimColumn):
        kind = "float" if col.data.dtype in (torch.float64, torch.float32) else "int"
        key = order_key(col.data, kind, descending)
    else:
        raise TypeError(f"cannot sort by {col.dtype}")
    valid = col.valid_mask()
    if col.valid is not None:
        key = torch.where(valid, key, torch.zeros_like(key))
    return key, valid


def _expand_struct_specs(specs):
    """A struct sort key is its fields, left to right (Spark's struct ordering): the struct's own null placement
    first (a flag column that is null where the struct is), then every field — nested structs recursively — with
    the struct's direction and ascending-nulls-first field ordering (reversed as a whole for DESC)."""
    from ..engine.column import ConstColumn, PrimColumn, StructColumn
    out = []
    for col, ascending, nulls_first in specs:
        if isinstance(col, ConstColumn):
            col = col.materialize()
        if not isinstance(col, StructColumn):
            out.append((col, ascending, nulls_first))
            continue
        if col.valid is not None:
            out.append((PrimColumn("int", torch.zeros(col.length, dtype=torch.int64, device=col.valid.device),
                                   col.valid), ascending, nulls_first))
        out += _expand_struct_specs([(c, ascending, ascending) for c in col.children])
    return out


def sort_spec_words(specs) -> List[torch.Tensor]:
    """``specs``: [(column, ascending, nulls_first)] most significant first → key words, least significant first:
    every item contributes its order key and, above it, a null-placement flag word.  Struct columns order by their
    fields (``_expand_struct_specs``)."""
    words: List[torch.Tensor] = []
    for col, ascending, nulls_first in reversed(_expand_struct_specs(list(specs))):
        key, valid = column_order_key(col, not ascending)
        words.append(key)
        if col.valid is not None:
            flag = valid if nulls_first else ~valid          # 0 sorts first
            words.append(flag.to(torch.int64))
    return words
