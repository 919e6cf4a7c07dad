"""Reference data loading (CSV / TSV → device string table).  Reference: DataProcessing/datax-host/src/main/scala/
datax/handler/ReferenceDataHandler.scala:16-61 and datax-utility/.../CSVUtil.scala:15-41 — Spark reads the file
with the given delimiter and header options and no schema inference, so every column is a string; stream–static
joins cast as needed.

MI355X path (``load_csv`` on a GPU):
* rank 0 reads the file once (local, mounted or ``wasbs://``; gzip-aware), copies the bytes to HBM and, with
  several ranks, broadcasts that device buffer over RCCL — ONE collective of the compact text, never W copies of
  parsed columns, and the receivers' copies land straight in HBM (no host staging on ranks > 0);
* every rank frames lines with the newline kernels and tokenizes one line per lane
  (``csv.hip``): each cell is a [start, len) view into the resident byte arena, so a 100 M-row table is one pass over
  its bytes and stays in HBM for the life of the job (sized for 288 GB); joins against it reuse one cached hash
  table (``Catalog.cached_build``).
The CPU path applies the same Spark semantics in Python (``tokenize_line``) — the differential-test oracle.

``schema`` (a DDL string, optional, e.g. ``"refKey long, zone long, tier string"``) is this engine's extension (the
DataFrameReader ``.schema(...)`` option): the named columns are cast on the device once at load.
"""
from __future__ import annotations

import time
from typing import List, Optional, Tuple

import torch

from ..engine.column import StrColumn, Table, strings_from_pylist
from . import fs


def tokenize_line(line: str, delim: str = ",", quote: str = '"', escape: str = "\\") -> List[Optional[str]]:
    """One CSV line → fields with the device kernel's (Spark 2.4 PERMISSIVE) semantics: empty unquoted → None,
    quoted → unescaped content (escape + quote/escape, or a doubled quote, is one literal char), junk between a
    closing quote and the delimiter dropped."""
    out: List[Optional[str]] = []
    p, n = 0, len(line)
    while True:
        if p < n and line[p] == quote:
            q = p + 1
            buf = []
            while q < n:
                c = line[q]
                if c == escape and escape != quote and q + 1 < n and line[q + 1] in (quote, escape):
                    buf.append(line[q + 1])
                    q += 2
                    continue
                if c == quote:
                    if q + 1 < n and line[q + 1] == quote:
                        buf.append(quote)
                        q += 2
                        continue
                    break
                buf.append(c)
                q += 1
            out.append("".join(buf))
            while q < n and line[q] != delim:
                q += 1
        else:
            q = p
            while q < n and line[q] != delim:
                q += 1
            out.append(line[p:q] if q > p else None)
        if q >= n:
            return out
        p = q + 1


def _split_lines(text: str) -> List[str]:
    return [l.rstrip("\r\n") for l in text.split("\n") if l.rstrip("\r\n")]


def read_shared(path: str, device) -> bytes:
    """The file's bytes on every rank: rank 0 reads, then one broadcast (RCCL over xGMI on GPUs)."""
    from .. import parallel as P
    if not P.active():
        return fs.read_bytes(path)
    data = fs.read_bytes(path) if P.rank() == 0 else b""
    return P.broadcast_bytes(data, src=0)


def read_shared_device(path: str, device) -> Tuple[torch.Tensor, int, bool]:
    """The file's bytes in HBM on every rank → (buffer with 64 zero bytes of padding, length, host_staged).  Rank 0
    reads the file and copies it to the device once; other ranks receive the RCCL broadcast straight into their own
    HBM (``host_staged`` is False there: the payload never touched their host memory)."""
    from .. import parallel as P
    if P.active():
        data = fs.read_bytes(path) if P.rank() == 0 else None
        buf, length = P.broadcast_device_bytes(data, 0, device)
        return buf, length, P.rank() == 0
    data = fs.read_bytes(path)
    length = len(data)
    host = torch.empty(length + 64, dtype=torch.uint8, pin_memory=True)
    host[length:].zero_()
    if length:
        host[:length] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    buf = host.to(device, non_blocking=True)
    buf.record_stream(torch.cuda.current_stream(device))
    return buf, length, True


def load_csv(path: str, delimiter: str = ",", header: bool = True, device="cpu", schema: Optional[str] = None,
             quote: str = '"', escape: str = "\\", stats: Optional[dict] = None) -> Table:
    device = torch.device(device)
    t0 = time.perf_counter()
    staged = True
    if device.type == "cuda":
        buf, length, staged = read_shared_device(path, device)
        t_read = time.perf_counter() - t0
        table = _load_device(buf, length, delimiter, header, device, quote, escape)
    else:
        data = read_shared(path, device)
        if data.startswith(b"\xef\xbb\xbf"):               # UTF-8 BOM (files saved by Excel / .NET)
            data = data[3:]
        length = len(data)
        t_read = time.perf_counter() - t0
        table = _load_host(data.decode("utf-8"), delimiter, header, device, quote, escape)
    if schema:
        table = _apply_schema(table, schema)
    if stats is not None:
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        stats.update(bytes=length, rows=table.length, read_s=t_read, total_s=time.perf_counter() - t0,
                     host_staged=staged)
    return table


def _header_names(first: str, delimiter: str, quote: str, escape: str, ncols: Optional[int] = None):
    f = tokenize_line(first, delimiter, quote, escape)
    return [(c or f"_c{i}").strip() for i, c in enumerate(f)]


def _load_host(text: str, delimiter, header, device, quote, escape) -> Table:
    lines = _split_lines(text)
    if not lines:
        return Table([], [], 0, device)
    if header:
        names, lines = _header_names(lines[0], delimiter, quote, escape), lines[1:]
    else:
        names = [f"_c{i}" for i in range(len(tokenize_line(lines[0], delimiter, quote, escape)))]
    rows = [tokenize_line(l, delimiter, quote, escape) for l in lines]
    cols = [strings_from_pylist([r[j] if j < len(r) else None for r in rows], device) for j in range(len(names))]
    return Table(names, cols, len(rows), device)


def _head(buf: torch.Tensor, length: int, need_newline: bool = True) -> bytes:
    """The first bytes of a device buffer, up to and including the first non-empty line (a small D2H read)."""
    k = min(length, 1 << 16)
    while True:
        head = buf[:k].cpu().numpy().tobytes()
        if k >= length or any(l.strip(b"\r") for l in head.split(b"\n")[:-1]):
            return head
        k = min(length, k * 4)


def _load_device(buf: torch.Tensor, length: int, delimiter, header, device, quote, escape) -> Table:
    """CSV bytes already in HBM (``buf``: ``length`` bytes + ≥ 64 zero bytes) → device string table."""
    from ..ops import native as N
    from ..ops.jsonparse import frame_lines_gpu
    if len(delimiter) != 1 or len(quote) != 1 or len(escape) != 1:
        raise ValueError("CSV delimiter, quote and escape must be single characters")
    data = _head(buf, length)
    if data.startswith(b"\xef\xbb\xbf"):                   # UTF-8 BOM (files saved by Excel / .NET): re-base the
        nb = torch.zeros(length - 3 + 64, dtype=torch.uint8, device=device)   # bytes (kernels want an aligned start)
        nb[:length - 3] = buf[3:length]
        buf, length, data = nb, length - 3, data[3:]
    # header / column count from the first non-empty line (host: a few bytes)
    first_end = 0
    first = ""
    while first_end < len(data):
        nl = data.find(b"\n", first_end)
        nl = len(data) if nl < 0 else nl
        first = data[first_end:nl].decode("utf-8").rstrip("\r")
        if first:
            break
        first_end = nl + 1
    if not first:
        return Table([], [], 0, device)
    names = _header_names(first, delimiter, quote, escape) if header else \
        [f"_c{i}" for i in range(len(tokenize_line(first, delimiter, quote, escape)))]
    ncols = len(names)
    offs = frame_lines_gpu(buf, length)                 # non-empty lines (one host read of the line count)
    if header:
        offs = offs[1:]                                 # the first non-empty line is the header
    n = int(offs.shape[0]) - 1
    if n <= 0:
        return Table(names, [strings_from_pylist([], device) for _ in names], 0, device)
    starts = torch.empty((ncols, n), dtype=torch.int64, device=device)
    lens = torch.empty((ncols, n), dtype=torch.int32, device=device)
    valid = torch.empty((ncols, n), dtype=torch.uint8, device=device)
    row_ok = torch.empty(n, dtype=torch.uint8, device=device)
    N.call("dxa_csv_tokenize", N.ptr(buf), N.ptr(offs), n, ncols, ord(delimiter), ord(quote), ord(escape),
           N.ptr(starts), N.ptr(lens), N.ptr(valid), N.ptr(row_ok), N.stream_handle(device))
    keep = None
    if not bool(row_ok.all()):                           # whitespace-only lines (CRLF blanks): drop them
        keep = torch.nonzero(row_ok).flatten()
        n = int(keep.shape[0])
    cols = []
    for j in range(ncols):
        s, l, v = starts[j], lens[j], valid[j].to(torch.bool)
        if keep is not None:
            s, l, v = s[keep], l[keep], v[keep]
        cols.append(StrColumn(buf, s, l, v))
    return Table(names, cols, n, device)


def _apply_schema(table: Table, ddl: str) -> Table:
    from ..engine.expr import cast_column
    from ..engine.types import parse_ddl_schema
    sch = parse_ddl_schema(ddl)
    want = {f.name.lower(): f.dtype for f in sch.fields}
    cols = []
    for name, c in zip(table.names, table.columns):
        t = want.get(name.lower())
        cols.append(cast_column(c, t) if t is not None and t != "string" else c)
    return Table(table.names, cols, table.length, table.device)
