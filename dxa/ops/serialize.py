"""Binding for the native row serialiser (``libdxa_host.so`` / host_serialize.cpp).

Columns are brought to host memory once (one D2H copy per buffer), described as a flat ``SerNode`` tree and rendered
by worker threads; the result is one newline-separated JSON blob that sinks can write without per-row Python work.
"""
from __future__ import annotations

import ctypes
import json
import os
import threading
from typing import List, Optional, Tuple

import numpy as np
import torch

from .build import HOST_LIB

_LIB = None
_lock = threading.Lock()

K_I64, K_F64, K_BOOL, K_STR, K_TS, K_DATE, K_CONST, K_STRUCT, K_MAP, K_ARRAY, K_RAW, K_NULL = range(12)


class SerNode(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("nchildren", ctypes.c_int32), ("child0", ctypes.c_int32),
                ("drop_nulls", ctypes.c_int32), ("name", ctypes.c_char_p), ("name_len", ctypes.c_int32),
                ("pad", ctypes.c_int32), ("data", ctypes.c_void_p), ("valid", ctypes.c_void_p),
                ("arena", ctypes.c_void_p), ("starts", ctypes.c_void_p), ("lens", ctypes.c_void_p),
                ("const_text", ctypes.c_char_p), ("const_len", ctypes.c_int32), ("pad2", ctypes.c_int32)]


def lib():
    global _LIB
    if _LIB is None:
        with _lock:
            if _LIB is None:
                if not HOST_LIB.exists():
                    from .build import build
                    build()
                L = ctypes.CDLL(str(HOST_LIB))
                L.dxa_serialize_rows.restype = ctypes.c_void_p
                L.dxa_serialize_rows.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                                 ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
                L.dxa_host_free.argtypes = [ctypes.c_void_p]
                L.dxa_java_double.argtypes = [ctypes.c_double, ctypes.c_char_p, ctypes.c_int]
                if L.dxa_sernode_size() != ctypes.sizeof(SerNode):
                    raise RuntimeError("SerNode layout mismatch")
                _LIB = L
    return _LIB


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def _quoted(name: str) -> bytes:
    return json.dumps(name, ensure_ascii=False).encode("utf-8")


class _Builder:
    """Describes a table as a SerNode tree over *host* buffers.  Device buffers are copied with non-blocking D2H
    copies into pinned memory on the current stream; ``event`` marks their completion, so the rendering can run on
    a host worker while the GPU already works on the next batch."""

    def __init__(self):
        self.nodes: List[dict] = []
        self.keep = []
        self.device_copies = False

    def _host(self, t: Optional[torch.Tensor]):
        if t is None:
            return 0
        h = t.detach()
        if h.is_cuda:
            src = h.contiguous()
            h = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
            h.copy_(src, non_blocking=True)
            self.keep.append(src)            # the source must outlive the async copy
            self.device_copies = True
        h = h.contiguous()
        self.keep.append(h)
        return h.data_ptr()

    def add(self, col, name: Optional[str]) -> int:
        from ..engine.column import (ArrayColumn, ConstColumn, JsonColumn, PrimColumn, StrColumn, StructColumn)
        from ..engine.serialize import _scalar_text
        from ..engine.decimal import is_decimal, to_text_column as decimal_text
        col = _canon_array(col)
        idx = len(self.nodes)
        nd = {"kind": K_NULL, "nchildren": 0, "child0": 0, "drop_nulls": 0, "name": _quoted(name) if name else b"",
              "data": 0, "valid": 0, "arena": 0, "starts": 0, "lens": 0, "const": b""}
        self.nodes.append(nd)
        if isinstance(col, ConstColumn):
            if col.value is None:
                nd["kind"] = K_NULL
            else:
                nd["kind"] = K_CONST
                nd["const"] = _scalar_text(col.value, col.dtype).encode("utf-8")
            return idx
        if isinstance(col, PrimColumn) and is_decimal(col.dtype):
            col = decimal_text(col, raw=True)       # exact digits at the column's scale, a raw JSON number
        nd["valid"] = self._host(col.valid.view(torch.uint8) if col.valid is not None else None)
        if isinstance(col, StrColumn):
            nd["kind"] = K_RAW if isinstance(col, JsonColumn) else K_STR
            if col.arena.numel() > 4 * col.length * 64 + 4096 and not getattr(col, "_compact", False):
                # views into a large arena (e.g. the batch's raw input buffer): gather only the referenced bytes
                # on the device before the D2H copy
                col = col.compact()
            nd["arena"] = self._host(col.arena)
            nd["starts"] = self._host(col.starts)
            nd["lens"] = self._host(col.lens)
            return idx
        if isinstance(col, PrimColumn):
            dt = col.dtype
            d = col.data
            if dt == "boolean":
                nd["kind"] = K_BOOL
                d = d.to(torch.uint8) if d.dtype == torch.bool else (d != 0).to(torch.uint8)
            elif dt in ("byte", "short", "int", "long"):
                nd["kind"] = K_I64
            elif dt == "timestamp":
                nd["kind"] = K_TS
            elif dt == "date":
                nd["kind"] = K_DATE
            else:
                nd["kind"] = K_F64
                d = d.to(torch.float64)
            nd["data"] = self._host(d)
            return idx
        if isinstance(col, (StructColumn, ArrayColumn)):
            kids = list(zip(col.names, col.children)) if isinstance(col, StructColumn) else \
                [(None, e) for e in col.elements]
            nd["kind"] = (K_MAP if col.is_map else K_STRUCT) if isinstance(col, StructColumn) else K_ARRAY
            nd["drop_nulls"] = 1 if isinstance(col, ArrayColumn) and col.drop_nulls else 0
            nd["nchildren"] = len(kids)
            # children must be contiguous: reserve slots first, then fill recursively
            first = len(self.nodes)
            nd["child0"] = first
            placeholders = []
            for nm, _ in kids:
                self.nodes.append(None)
                placeholders.append(nm)
            for j, (nm, c) in enumerate(kids):
                sub = _Builder()
                sub.keep = self.keep
                sub.nodes = self.nodes
                # build child in place: append at end, then move into its reserved slot
                k = sub.add(c, nm if isinstance(col, StructColumn) else None)
                self.nodes[first + j] = self.nodes[k]
                self.nodes[k] = {"kind": K_NULL, "nchildren": 0, "child0": 0, "drop_nulls": 0, "name": b"",
                                 "data": 0, "valid": 0, "arena": 0, "starts": 0, "lens": 0, "const": b""}
            return idx
        raise TypeError(f"cannot serialise {col!r}")


def _canon_array(col):
    """Arrays with a per-row ``present`` mask as the serializer's node kinds express them: a drop-nulls array, or —
    when a present slot holds a real null — the rows rendered on the host as raw JSON text."""
    from ..engine.column import ArrayColumn, JsonColumn, column_from_pylist
    if not isinstance(col, ArrayColumn) or col.present is None:
        return col
    canon = col.canonical()
    if canon is not None:
        return canon
    from ..engine.serialize import _frag_values
    sc = column_from_pylist(_frag_values(col), "string", col.device)
    return JsonColumn(sc.arena, sc.starts, sc.lens, sc.valid, "string")


class DevNode(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("nchildren", ctypes.c_int32), ("child0", ctypes.c_int32),
                ("drop_nulls", ctypes.c_int32), ("name_off", ctypes.c_int32), ("name_len", ctypes.c_int32),
                ("const_off", ctypes.c_int32), ("const_len", ctypes.c_int32), ("data", ctypes.c_void_p),
                ("valid", ctypes.c_void_p), ("arena", ctypes.c_void_p), ("starts", ctypes.c_void_p),
                ("lens", ctypes.c_void_p)]


class _DevBuilder:
    """SerNode tree over *device* buffers for the GPU serializer (json_serialize.hip); names and constant values go
    into one text pool."""

    def __init__(self):
        self.nodes: List[dict] = []
        self.text = bytearray()
        self.keep = []

    def _t(self, b: bytes):
        """Text starts 8-B aligned with zero padding before it: the device emits it as 8-B words."""
        self.text += b"\0" * (-len(self.text) % 8)
        off = len(self.text)
        self.text += b
        return off, len(b)

    def _dev(self, t: Optional[torch.Tensor]):
        if t is None:
            return 0
        t = t.contiguous()
        self.keep.append(t)
        return t.data_ptr()

    def _blank(self):
        return {"kind": K_NULL, "nchildren": 0, "child0": 0, "drop_nulls": 0, "name": (0, 0), "const": (0, 0),
                "data": 0, "valid": 0, "arena": 0, "starts": 0, "lens": 0}

    def add(self, col, name: Optional[str]) -> int:
        from ..engine.column import (ArrayColumn, ConstColumn, JsonColumn, PrimColumn, StrColumn, StructColumn)
        from ..engine.serialize import _scalar_text
        from ..engine.decimal import is_decimal, to_text_column as decimal_text
        col = _canon_array(col)
        idx = len(self.nodes)
        nd = self._blank()
        if name:
            nd["name"] = self._t(_quoted(name) + b":")
        self.nodes.append(nd)
        if isinstance(col, ConstColumn):
            if col.value is not None:
                nd["kind"] = K_CONST
                nd["const"] = self._t(_scalar_text(col.value, col.dtype).encode("utf-8"))
            return idx
        if isinstance(col, PrimColumn) and is_decimal(col.dtype):
            col = decimal_text(col, raw=True)       # exact digits at the column's scale, a raw JSON number
        if col.valid is not None:
            nd["valid"] = self._dev(col.valid.view(torch.uint8) if col.valid.dtype == torch.bool else col.valid)
        if isinstance(col, StrColumn):
            nd["kind"] = K_RAW if isinstance(col, JsonColumn) else K_STR
            nd["arena"] = self._dev(col.arena)
            nd["starts"] = self._dev(col.starts.to(torch.int64))
            nd["lens"] = self._dev(col.lens.to(torch.int32))
            return idx
        if isinstance(col, PrimColumn):
            dt, d = col.dtype, col.data
            if dt == "boolean":
                nd["kind"] = K_BOOL
                d = d.to(torch.uint8)
            elif dt in ("byte", "short", "int", "long"):
                nd["kind"] = K_I64
                d = d.to(torch.int64)
            elif dt == "timestamp":
                nd["kind"] = K_TS
            elif dt == "date":
                nd["kind"] = K_DATE
                d = d.to(torch.int64)
            else:
                nd["kind"] = K_F64
                d = d.to(torch.float64)
            nd["data"] = self._dev(d)
            return idx
        if isinstance(col, (StructColumn, ArrayColumn)):
            kids = list(zip(col.names, col.children)) if isinstance(col, StructColumn) else \
                [(None, e) for e in col.elements]
            nd["kind"] = (K_MAP if col.is_map else K_STRUCT) if isinstance(col, StructColumn) else K_ARRAY
            nd["drop_nulls"] = 1 if isinstance(col, ArrayColumn) and col.drop_nulls else 0
            nd["nchildren"] = len(kids)
            first = len(self.nodes)
            nd["child0"] = first
            for _ in kids:
                self.nodes.append(None)
            for j, (nm, c) in enumerate(kids):
                k = self.add(c, nm if isinstance(col, StructColumn) else None)
                self.nodes[first + j] = self.nodes[k]
                self.nodes[k] = self._blank()
            return idx
        raise TypeError(f"cannot serialise {col!r}")

    def program(self, top: List[int]) -> List[int]:
        """Flat render program for json_serialize.hip: preorder FIELD ops (code 0, node, depth, mode | skip << 8) with
        a CLOSE op (code 1) after each container's children; `skip` = ops to jump when the field is omitted/null.
        Modes: 0 struct member, 1 map member, 2 array element, 3 filterNull array element."""
        ops: List[List[int]] = []
        for t in top:
            self._emit(ops, t, 0, 0)
        return [v for op in ops for v in op]

    def _emit(self, ops: List[List[int]], idx: int, depth: int, mode: int):
        # a method, not a nested recursive function: that would be a reference cycle pinning this plan (and the
        # column tensors it keeps alive) until the cyclic collector ran
        if depth > 30:
            raise ValueError("JSON nesting deeper than 30 levels")
        pos = len(ops)
        ops.append([0, idx, depth, mode])
        nd = self.nodes[idx]
        if nd["kind"] in (K_STRUCT, K_MAP, K_ARRAY):
            cm = {K_STRUCT: 0, K_MAP: 1}.get(nd["kind"], 3 if nd["drop_nulls"] else 2)
            for j in range(nd["nchildren"]):
                self._emit(ops, nd["child0"] + j, depth + 1, cm)
            ops.append([1, idx, depth, 0])
        ops[pos][3] = mode | ((len(ops) - pos - 1) << 8)

    def tables_blob(self, prog: List[int]) -> bytes:
        """Node array, render program (padded to 8 B) and text pool as ONE buffer, the layout dxa_serialize_rows
        expects: a single upload per rendered batch."""
        arr = (DevNode * max(1, len(self.nodes)))()
        for i, nd in enumerate(self.nodes):
            arr[i] = DevNode(nd["kind"], nd["nchildren"], nd["child0"], nd["drop_nulls"], nd["name"][0],
                             nd["name"][1], nd["const"][0], nd["const"][1], nd["data"], nd["valid"], nd["arena"],
                             nd["starts"], nd["lens"])
        p = (ctypes.c_int32 * max(2, len(prog) + len(prog) % 2))(*prog)
        text = bytes(self.text) + b"\0" * (-len(self.text) % 8 + 8)
        return bytes(arr)[:ctypes.sizeof(DevNode) * len(self.nodes)] + bytes(p)[:((len(prog) * 4 + 7) // 8) * 8] + text


class _SerSegs(ctypes.Structure):
    _fields_ = [("nseg", ctypes.c_int32), ("pad", ctypes.c_int32), ("row", ctypes.c_int64 * 17),
                ("pc", ctypes.c_int32 * 17), ("block", ctypes.c_int32 * 17)]


MAX_SEGMENTS = 16
_LDS_LIMIT = 64 * 1024
STATS = {"rendered_bytes": 0, "d2h_bytes": 0, "d2h_s": 0.0, "launch_pairs": 0}


def _render_members(members: List["Staged"]) -> None:
    """Render every GPU-staged table of ``members`` with ONE length launch, one scan, one write launch, one upload
    of the render tables and one D2H each for the lengths and the text (a segment per table); each member's
    ``JsonLines`` is a slice of the shared pinned blob.  A gzip member is rendered alone (its compressed stream is
    what crosses PCIe)."""
    from . import native as N
    dev = members[0].device
    side = _side_stream(dev)
    with torch.inference_mode(), torch.cuda.stream(side):
        for m in members:
            side.wait_event(m.event)
        plan, keep = _plan_of(members)
        blob, nnodes, nprog, tw, pcs = plan
        segs = _SerSegs()
        segs.nseg = len(members)
        r = 0
        for k, m in enumerate(members):
            segs.row[k], segs.pc[k] = r, pcs[k]
            r += m.n
        segs.row[len(members)], segs.pc[len(members)] = r, pcs[len(members)]
        n = r
        lens_h = torch.empty(n, dtype=torch.int64, pin_memory=True)
        if n:
            tables = N.h2d(blob, torch.uint8, dev)
            st = N.stream_handle(dev)
            lens = torch.empty(n, dtype=torch.int64, device=dev)
            N.call("dxa_serialize_rows", 0, N.ptr(tables), nnodes, nprog, tw, ctypes.addressof(segs), N.ptr(lens),
                   None, None, st)
            ends = torch.cumsum(lens, 0)
            lens_h.copy_(lens, non_blocking=True)
            side.synchronize()
        lens_np = lens_h.numpy()
        total = int(lens_np.sum())
        STATS["rendered_bytes"] += total
        STATS["launch_pairs"] += 1
        if n:
            out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
            N.call("dxa_serialize_rows", 1, N.ptr(tables), nnodes, nprog, tw, ctypes.addressof(segs), N.ptr(lens),
                   N.ptr(ends), N.ptr(out), st)
        if len(members) == 1 and members[0].compress and total > 1:
            # gzip of the newline-joined documents (no trailing newline: what a blob sink writes), on the GPU;
            # only the compressed stream crosses PCIe
            from .deflate import gzip_device
            gz = gzip_device(out, total - 1)
            host = torch.empty(gz.numel(), dtype=torch.uint8, pin_memory=True)
            side.synchronize()
            d2h(host, gz, gz.numel(), side)
            members[0]._done(JsonLines(None, lens_np - 1, gz=host.numpy()))
            return
        host = torch.empty(total, dtype=torch.uint8, pin_memory=True)
        side.synchronize()
        d2h(host, out if n else host, total, side)
    blob_np = host.numpy()                              # the pinned buffer itself, no copy
    r = off = 0
    for m in members:
        ln = lens_np[r:r + m.n]
        size = int(ln.sum())
        m._done(JsonLines(blob_np[off:off + size], ln - 1))
        r += m.n
        off += size


def _build_plan(members: List["Staged"]):
    """The render tables of ``members`` through ``_DevBuilder``: (blob, nodes, program ops, text words, per-member
    program starts + total), and the converted tensors the blob points at (alive until the kernels ran)."""
    b = _DevBuilder()
    progs = []
    for m in members:
        top = [b.add(c, nm) for nm, c in zip(m.table.names, m.table.columns)]
        progs.append(b.program(top))
    prog = [v for p in progs for v in p]
    blob = b.tables_blob(prog)
    tw = (len(blob) - ctypes.sizeof(DevNode) * len(b.nodes) - ((len(prog) * 4 + 7) // 8) * 8) // 8
    pcs, pc = [], 0
    for p in progs:
        pcs.append(pc)
        pc += len(p) // 4
    pcs.append(pc)
    return (blob, len(b.nodes), len(prog) // 4, tw, pcs), b.keep


# Render plans of flat tables (one node per column) by their shape — names, column kinds, constants' types: the
# node array, program and text pool are the same every batch; only the five buffer pointers of each node change, and
# a constant whose text differs from the template's (a batch time in an alert row) gets its text appended to the
# pool.  A batch's outputs then cost a signature and the pointer reads instead of a walk of the builder per column.
_PLANS: dict = {}
_PLAN_MAX = 64
_PTR_COLS = 5                        # DevNode's pointer fields (data, valid, arena, starts, lens): its last 5 words
_INT_KINDS = {"byte": K_I64, "short": K_I64, "int": K_I64, "long": K_I64, "date": K_DATE}


def _flat_signature(members: List["Staged"], consts: Optional[list] = None):
    """The plan-cache key of ``members`` (None: not flat); ``consts`` collects (node index, value, type) of every
    constant column."""
    from ..engine.column import ConstColumn, JsonColumn, PrimColumn, StrColumn
    from ..engine.decimal import is_decimal
    sig = []
    k = 0
    for m in members:
        for nm, c in zip(m.table.names, m.table.columns):
            tc = type(c)
            if tc is PrimColumn:
                if is_decimal(c.dtype):
                    return None
                sig.append((nm, c.dtype))
            elif tc is StrColumn or tc is JsonColumn:
                sig.append((nm, tc))
            elif tc is ConstColumn:
                v = c.value
                if v is not None and type(v) not in (str, int, float, bool):
                    return None
                sig.append((nm, c.dtype, type(v)))
                if consts is not None and v is not None:
                    consts.append((k, v, c.dtype))
            else:
                return None
            k += 1
        sig.append(len(m.table.columns))
    return tuple(sig)


_CONST_TEXT: dict = {}


def _const_text(v, dtype) -> bytes:
    """A constant's rendered text (``_DevBuilder.add``'s), memoised: alert rows carry a new batch time each batch."""
    key = (type(v), v, str(dtype))
    t = _CONST_TEXT.get(key)
    if t is None:
        from ..engine.serialize import _scalar_text
        if len(_CONST_TEXT) >= 4096:
            _CONST_TEXT.clear()
        t = _CONST_TEXT[key] = _scalar_text(v, dtype).encode("utf-8")
    return t


def _flat_pointers(members: List["Staged"], keep: list) -> List[int]:
    """(data, valid, arena, starts, lens) of every column, converted as ``_DevBuilder.add`` converts them."""
    from ..engine.column import ConstColumn, PrimColumn
    out = []
    for m in members:
        for c in m.table.columns:
            if type(c) is ConstColumn:
                out += (0, 0, 0, 0, 0)
                continue
            v = c.valid
            if v is not None:
                v = (v.view(torch.uint8) if v.dtype == torch.bool else v).contiguous()
                keep.append(v)
            vp = 0 if v is None else v.data_ptr()
            if type(c) is PrimColumn:
                dt, d = c.dtype, c.data
                if dt == "boolean":
                    d = d.to(torch.uint8)
                elif dt in _INT_KINDS:
                    d = d.to(torch.int64)
                elif dt != "timestamp":
                    d = d.to(torch.float64)
                d = d.contiguous()
                keep.append(d)
                out += (d.data_ptr(), vp, 0, 0, 0)
            else:
                a, st, ln = c.arena.contiguous(), c.starts.to(torch.int64).contiguous(), c.lens.to(torch.int32).contiguous()
                keep += (a, st, ln)
                out += (0, vp, a.data_ptr(), st.data_ptr(), ln.data_ptr())
    return out


def _plan_of(members: List["Staged"]):
    """The render plan of ``members`` (``_build_plan``'s tuple, the blob with this batch's pointers) and the tensors
    to keep alive; flat shapes reuse a cached template."""
    consts: list = []
    sig = _flat_signature(members, consts)
    if sig is None:
        return _build_plan(members)
    tmpl = _PLANS.get(sig)
    if tmpl is None:
        plan, keep = _build_plan(members)
        blob, nnodes = plan[0], plan[1]
        t = np.frombuffer(blob, dtype=np.uint8).copy()
        words = t[:ctypes.sizeof(DevNode) * nnodes].view(np.uint64).reshape(nnodes, -1)
        words[:, -_PTR_COLS:] = 0
        if len(_PLANS) >= _PLAN_MAX:
            _PLANS.clear()
        _PLANS[sig] = (t, plan, [(k, _const_text(v, dt)) for k, v, dt in consts])
        return plan, keep
    t, plan, texts = tmpl
    nnodes, tw = plan[1], plan[3]
    keep: list = []
    ptrs = _flat_pointers(members, keep)
    extra, patches = bytearray(), []
    for (k, v, dt), (_, old) in zip(consts, texts):
        txt = _const_text(v, dt)
        if txt != old:
            patches.append((k, tw * 8 + len(extra), len(txt)))
            extra += txt + b"\0" * (-len(txt) % 8)
    if patches:
        extra += b"\0" * 8                      # the zero word the text pool ends with
        if len(t) + len(extra) > _LDS_LIMIT:    # the kernels stage the tables in 64 KiB of LDS
            return _build_plan(members)
        buf = np.concatenate([t, np.frombuffer(bytes(extra), dtype=np.uint8)])
        tw += len(extra) // 8
    else:
        buf = t.copy()
    nb = ctypes.sizeof(DevNode) * nnodes
    buf[:nb].view(np.uint64).reshape(nnodes, -1)[:, -_PTR_COLS:] = np.array(ptrs, dtype=np.uint64).reshape(nnodes,
                                                                                                           _PTR_COLS)
    if patches:
        ints = buf[:nb].view(np.int32).reshape(nnodes, -1)
        for k, off, ln in patches:
            ints[k, 6], ints[k, 7] = off, ln           # DevNode.const_off / const_len
    return (torch.from_numpy(buf), nnodes, plan[2], tw, plan[4]), keep


class RenderGroup:
    """GPU-staged tables of one batch (every output's payloads) rendered together by whichever sink thread asks
    first (``_render_members``); the others wait on the lock and take their slice."""

    def __init__(self, members: List["Staged"]):
        self.members = members
        self.lock = threading.Lock()

    def ensure(self) -> None:
        with self.lock:
            if any(m._result is None for m in self.members):
                _render_members(self.members)


def link_render_groups(staged: List["Staged"]) -> None:
    """Group the GPU-staged, uncompressed, non-empty tables of a batch (same device, at most MAX_SEGMENTS per group,
    render tables within the 64 KiB the kernels stage in LDS) so each group renders with one launch pair."""
    seen, by_dev = set(), {}
    for s in staged:
        if not isinstance(s, Staged) or not s.gpu or s.compress or s.n == 0 or id(s) in seen or s.group is not None:
            continue
        seen.add(id(s))
        by_dev.setdefault(s.device, []).append(s)
    for ms in by_dev.values():
        cur, size = [], 0
        for m in ms:
            est = m.lds_estimate()
            if cur and (len(cur) == MAX_SEGMENTS or size + est > _LDS_LIMIT):
                _close_group(cur)
                cur, size = [], 0
            cur.append(m)
            size += est
        _close_group(cur)


def _close_group(ms: List["Staged"]) -> None:
    if len(ms) > 1:
        g = RenderGroup(ms)
        for m in ms:
            m.group = g


_SDMA = True                 # SDMA engine for the rendered-output D2H; off for good after a failed copy


def d2h(host: torch.Tensor, dev: torch.Tensor, nbytes: int, stream) -> None:
    """Copy the first ``nbytes`` of ``dev`` into pinned ``host`` and wait.  The producing work must be complete.
    Runs on an SDMA engine (``dxa_copy_sdma``): a hipMemcpy D2H into pinned memory is a blit kernel that holds CUs
    for the whole PCIe transfer.  Falls back to the stream copy if the runtime refuses the pointers."""
    global _SDMA
    if nbytes <= 0:
        return
    import time
    t0 = time.perf_counter()
    try:
        if _SDMA:
            from . import native as N
            rc = N.lib().dxa_copy_sdma(host.data_ptr(), dev.data_ptr(), nbytes)
            if rc == 0:
                return
            _SDMA = False
        with torch.cuda.stream(stream):
            host[:nbytes].copy_(dev[:nbytes], non_blocking=True)
        stream.synchronize()
    finally:
        STATS["d2h_bytes"] += nbytes
        STATS["d2h_s"] += time.perf_counter() - t0


_side_streams = {}
_side_lock = threading.Lock()


def _side_stream(device):
    """The output stream, at normal priority (a high-priority render stream measured within run-to-run noise on
    Latency-Process and throughput, profiles/gc/README.md)."""
    with _side_lock:
        s = _side_streams.get(device)
        if s is None:
            s = _side_streams[device] = torch.cuda.Stream(device)
        return s


def gpu_serializer_enabled(device) -> bool:
    if device.type != "cuda":
        return False
    try:
        from . import native
        native.lib()
        return True
    except Exception:  # noqa: BLE001
        return False


class Staged:
    """A table captured for serialization.  On the GPU the rows are rendered by the device serializer on a side
    stream (ordered after the producing work by an event) and the blob comes back with one D2H copy; otherwise the
    columns are copied to pinned host memory (async) and rendered by the native host serializer.  ``render`` may
    run on any host thread."""

    def __init__(self, table, compress: bool = False):
        self.n = table.length
        self.event = None
        self.gpu = gpu_serializer_enabled(table.device)
        self.compress = compress and self.gpu
        self.group = None
        self._result = None
        if self.gpu:
            self.table = table
            self.device = table.device
            self.event = torch.cuda.Event()
            self.event.record(torch.cuda.current_stream(table.device))
            return
        b = _Builder()
        self.top = [b.add(c, n) for n, c in zip(table.names, table.columns)]
        self.builder = b
        if b.device_copies:
            self.event = torch.cuda.Event()
            self.event.record(torch.cuda.current_stream(table.device))

    def _done(self, jl: "JsonLines") -> None:
        self._result = jl
        self.table = None

    def lds_estimate(self) -> int:
        """Upper bound of this table's share of the render tables (nodes + program + names) in LDS."""
        def walk(c, name):
            kids = getattr(c, "children", None) or getattr(c, "elements", None) or []
            names = getattr(c, "names", None) or [None] * len(kids)
            const = len(str(getattr(c, "value", "") or "")) if type(c).__name__ == "ConstColumn" else 0
            return (ctypes.sizeof(DevNode) + 32 + len(name or "") + 16 + const +
                    sum(walk(k, nm) for nm, k in zip(names, kids)))
        return sum(walk(c, nm) for nm, c in zip(self.table.names, self.table.columns))

    def _render_gpu(self) -> "JsonLines":
        if self._result is None:
            if self.group is not None:
                self.group.ensure()
            else:
                _render_members([self])
        return self._result

    def render(self, nthreads: Optional[int] = None) -> "JsonLines":
        if self.gpu:
            return self._render_gpu()
        if self.event is not None:
            self.event.synchronize()
        L = lib()
        b = self.builder
        arr = (SerNode * max(1, len(b.nodes)))()
        for i, nd in enumerate(b.nodes):
            arr[i] = SerNode(nd["kind"], nd["nchildren"], nd["child0"], nd["drop_nulls"], nd["name"],
                             len(nd["name"]), 0, nd["data"], nd["valid"], nd["arena"], nd["starts"], nd["lens"],
                             nd["const"], len(nd["const"]), 0)
        tops = (ctypes.c_int32 * max(1, len(self.top)))(*self.top)
        n = self.n
        line_len = np.zeros(max(1, n), dtype=np.int64)
        out_len = ctypes.c_int64(0)
        threads = nthreads or min(16, os.cpu_count() or 4)
        ptr = L.dxa_serialize_rows(ctypes.addressof(arr), len(b.nodes), ctypes.addressof(tops), len(self.top), n,
                                   threads, line_len.ctypes.data, ctypes.addressof(out_len))
        try:
            blob = ctypes.string_at(ptr, out_len.value)
        finally:
            L.dxa_host_free(ptr)
        self.builder = None                 # release pinned buffers
        return JsonLines(blob, line_len[:n])


class JsonLines:
    """Newline-terminated JSON lines held as one buffer (what sinks write) + per-line lengths.  The buffer may be
    ``bytes`` or a uint8 numpy array (e.g. the pinned D2H target of the device serializer — no extra host copy);
    behaves as a read-only sequence of ``str`` (decoded lazily) for sinks that want individual documents."""

    def __init__(self, blob, lens, gz=None):
        self.gz = gz                        # gzip of data(), when the device compressed it (then blob may be None)
        self._buf = blob
        self._bytes = blob if isinstance(blob, (bytes, bytearray)) else None
        self.lens = np.asarray(lens, dtype=np.int64)
        self._starts = None

    def _text_buf(self):
        if self._buf is None:               # compressed-only payload: the text is inflated on first use
            import gzip as _gzip
            self._buf = self._bytes = _gzip.decompress(bytes(self.gz)) + b"\n"
        return self._buf

    @property
    def blob(self) -> bytes:
        self._text_buf()
        if self._bytes is None:
            self._bytes = np.asarray(self._buf).tobytes()
        return self._bytes

    def nbytes(self) -> int:
        return len(self._text_buf())

    def view(self) -> memoryview:
        """Zero-copy view of the whole newline-terminated buffer."""
        self._text_buf()
        return memoryview(self._buf if self._bytes is None else self._bytes).cast("B")

    def __len__(self):
        return int(self.lens.shape[0])

    def _offsets(self):
        if self._starts is None:
            self._starts = np.concatenate([[0], np.cumsum(self.lens + 1)[:-1]]) if len(self) else \
                np.zeros(0, dtype=np.int64)
        return self._starts

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        s = int(self._offsets()[i])
        return bytes(self.view()[s:s + int(self.lens[i])]).decode("utf-8")

    def __iter__(self):
        b = self.blob
        if b.count(b"\n") == len(self):              # no raw newlines inside documents: split in one pass
            return iter(b.decode("utf-8").split("\n")[:len(self)])
        return (self[i] for i in range(len(self)))

    def text(self) -> str:
        """All lines joined by newlines (no trailing newline) — ``"\\n".join(lines)`` without per-line objects."""
        return bytes(self.data()).decode("utf-8")

    def data(self):
        """Newline-joined documents without the trailing newline, as a zero-copy buffer."""
        n = self.nbytes()
        return self.view()[:n - 1] if n else memoryview(b"")

    def __eq__(self, other):
        return list(self) == list(other)

    def __repr__(self):
        return f"JsonLines(n={len(self)}, bytes={self.nbytes()})"


def stage_table(table, compress: bool = False) -> Staged:
    return Staged(table, compress)


def serialize_table(table, nthreads: Optional[int] = None) -> Tuple[bytes, List[int]]:
    """Render every row → (blob of newline-terminated JSON lines, per-line lengths)."""
    jl = Staged(table).render(nthreads)
    return jl.blob, jl.lens.tolist()


def table_lines(table) -> List[str]:
    return list(Staged(table).render())


def java_double(d: float) -> str:
    buf = ctypes.create_string_buffer(64)
    n = lib().dxa_java_double(d, buf, 64)
    return buf.raw[:n].decode()
