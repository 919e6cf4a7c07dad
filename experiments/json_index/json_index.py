"""Stage-1 structural index of a JSON-lines batch (prototype, ``csrc/json_index.hip``): per segment of records, the
number of structural characters (``{ } [ ] : ,``) outside strings, and optionally the per-64-byte structural
bitmaps.  It measures the bulk pass of a two-stage (simdjson-style) parser on MI355X; the engine's parser is still
``json_parse_kernel``."""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from . import native as N

N.register_sigs({"dxa_json_index": [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]})


def structural_index(buf: torch.Tensor, offs: torch.Tensor, per_seg: int = 64, bits: bool = False
                     ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """(counts per segment of ``per_seg`` records, structural bitmap words or None) for records
    ``buf[offs[i]:offs[i+1]]`` (back to back)."""
    n = int(offs.shape[0]) - 1
    segs = max(1, (n + per_seg - 1) // per_seg)
    counts = torch.zeros(segs, dtype=torch.int64, device=buf.device)
    words = torch.zeros((buf.numel() + 63) // 64, dtype=torch.int64, device=buf.device) if bits else None
    if n > 0:
        N.call("dxa_json_index", N.ptr(buf), int(buf.numel()), N.ptr(offs), n, per_seg, N.ptr(counts),
               None if words is None else N.ptr(words), N.stream_handle(buf.device))
    return counts, words


def host_counts(data: bytes, offs, per_seg: int = 64):
    """Reference: the same counts by a byte-at-a-time scan (strings, backslash escapes)."""
    n = len(offs) - 1
    out = []
    for s in range(0, n, per_seg):
        lo, hi = offs[s], offs[min(s + per_seg, n)]
        cnt, in_str, esc = 0, False, False
        for b in data[lo:hi]:
            if in_str:
                if esc:
                    esc = False
                elif b == 0x5C:
                    esc = True
                elif b == 0x22:
                    in_str = False
            elif b == 0x22:
                in_str = True
            elif b in b"{}[]:,":
                cnt += 1
        out.append(cnt)
    return out
