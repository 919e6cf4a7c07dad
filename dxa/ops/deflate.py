"""gzip on the device (deflate.hip): fixed-size chunks → independent gzip members, concatenated.

Used by blob sinks (``compressiontype`` gzip, the default — the reference's GZipHelper, BlobSinker.scala) so that
the rendered JSON crosses PCIe compressed and no host thread spends ~1 s per 1 M events in zlib.  The result is an
RFC 1952 multi-member stream that gunzip, zlib (``wbits=47``) and Python's ``gzip`` read as the original bytes.
"""
from __future__ import annotations

import os

import torch

from . import native as N

CHUNK = int(os.environ.get("DXA_GZIP_CHUNK", "8192"))
# dynamic Huffman tables per member (a counting pass whose parse the coding pass reuses), the default: on the
# passthrough output 3.18x vs 2.53x with the fixed code, 54.7 vs 91.9 GB/s, and the blob-sink flow at 40.8 vs
# 43.3 M events/s (profiles/round5/blob/README.md).  ``dynamic=False`` (the fixed code) stays for tests.
DYNAMIC = True


def slot_bytes(chunk: int) -> int:
    """Per-chunk scratch slot (mirrors dxa_gzip_slot_bytes): header + worst-case fixed-Huffman output + trailer."""
    return (12 + (chunk * 9 + 7) // 8 + 32 + 15) & ~15


def gzip_device(buf: torch.Tensor, n: int, chunk: int = CHUNK, dynamic: bool = DYNAMIC) -> torch.Tensor:
    """Multi-member gzip of ``buf[:n]`` (uint8, on the GPU) on the current stream → uint8 device tensor."""
    dev = buf.device
    if n <= 0:
        return torch.empty(0, dtype=torch.uint8, device=dev)
    if not 64 <= chunk <= 32768 or chunk % 64:
        raise ValueError("gzip chunk must be a multiple of 64 in [64, 32768]")
    if buf.data_ptr() % 16:
        buf = buf[:n].clone()                   # the kernel stages 16-byte aligned chunks
    nch = (n + chunk - 1) // chunk
    slots = torch.empty(nch * slot_bytes(chunk), dtype=torch.uint8, device=dev)
    out_len = torch.empty(nch, dtype=torch.int32, device=dev)
    st = N.stream_handle(dev)
    # dynamic: the counting pass's parse (one word per input byte), read back by the coding pass
    toks = torch.empty(nch * chunk, dtype=torch.int32, device=dev) if dynamic else None
    N.call("dxa_gzip_chunks", N.ptr(buf), n, chunk, N.ptr(slots), N.ptr(out_len), int(dynamic),
           N.ptr(toks) if dynamic else None, st)
    ends = torch.cumsum(out_len.to(torch.int64), 0)
    offs = ends - out_len
    total = int(ends[-1].item())
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    N.call("dxa_gzip_pack", N.ptr(slots), chunk, N.ptr(out_len), N.ptr(offs), nch, N.ptr(out), st)
    return out
