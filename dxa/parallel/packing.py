"""Packed wire format of a columnar table for the RCCL collectives (all-to-all shuffles, all-gathers, broadcasts).

A table is flattened into leaves (prim columns, string columns, validity-only leaves of structs / arrays) and sent
as (a) one [rows × C] int64 matrix — row layout ``[prim data | string lengths | string offsets | mask words]``,
doubles bit-cast, narrower integers / booleans widened, validity folded into 63-bit mask words — and (b) one byte
arena per string leaf.  A string's offset column holds its position inside the bytes its DESTINATION receives, so
a receiver turns it into a view of the received arena without any scan.

Two implementations of the same layout:

* device (``exchange.hip``): ``dxa_xchg_plan`` (LDS histogram per block of rows + one-workgroup scan → the
  [W × (1+S)] send sizes), then — after the size exchange, the one host read-back — ``dxa_xchg_scatter`` writes
  every row at its destination-ordered position straight into the send matrix and its string bytes into the send
  arenas; ``dxa_xchg_unpack`` rebuilds every received leaf in one launch.  Three launches on the send side, one
  on the receive side, whatever the column count;
* torch (CPU, and the oracle the GPU tests compare the buffers against): a stable argsort by destination, gathers,
  cumsums.

Rows keep their relative order within a destination in both (stable), so the two produce identical buffers.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import torch

K8, K4, K1, K2 = 0, 1, 2, 3
_KIND = {8: K8, 4: K4, 1: K1, 2: K2}


class Leaf:
    __slots__ = ("kind", "dtype", "col", "mcol", "sidx", "vbit", "torch_dtype", "str_type")

    def __init__(self, kind, dtype, col=None):
        self.kind, self.dtype, self.col = kind, dtype, col
        self.mcol = -1
        self.sidx = -1
        self.vbit = -1
        self.torch_dtype = None
        self.str_type = None


class _Presence:
    """A slot-presence mask in the shape of a validity-only leaf."""
    dtype = "boolean"

    def __init__(self, mask):
        self.valid = mask


def flatten(col, leaves: List[Leaf], spec: list):
    """Walk a column tree; record data-bearing leaves and a rebuild spec."""
    from ..engine.column import ArrayColumn, ConstColumn, PrimColumn, StrColumn, StructColumn
    if isinstance(col, ConstColumn):
        spec.append(("const", col.value, col.dtype))
        return
    if isinstance(col, StructColumn):
        # the validity leaf exists whether or not this rank's column has nulls: every rank must flatten a table to
        # the same leaves (which of them carry validity is agreed separately, see Layout.assign)
        vleaf = len(leaves)
        leaves.append(Leaf("valid_only", "boolean", col))
        sub = []
        for c in col.children:
            flatten(c, leaves, sub)
        spec.append(("struct", col.names, col.is_map, col.dtype, vleaf, sub))
        return
    if isinstance(col, ArrayColumn):
        vleaf = len(leaves)
        leaves.append(Leaf("valid_only", "boolean", col))
        # one presence leaf per slot, on every rank (a rank without a ``present`` mask sends all-ones)
        pleaves = []
        for j in range(len(col.elements)):
            pleaves.append(len(leaves))
            leaves.append(Leaf("valid_only", "boolean", _Presence(col.slot_present(j))))
        sub = []
        for c in col.elements:
            flatten(c, leaves, sub)
        spec.append(("array", col.drop_nulls, vleaf, sub, pleaves))
        return
    if isinstance(col, StrColumn):
        spec.append(("str", len(leaves)))
        lf = Leaf("str", col.dtype, col)
        lf.str_type = type(col)
        leaves.append(lf)
        return
    if isinstance(col, PrimColumn) and col.data.dim() == 2:
        # a wide decimal(p > 18, s): its (lo, hi) words travel as two int64 leaves
        lo = PrimColumn("long", col.data[:, 0].contiguous(), col.valid)
        hi = PrimColumn("long", col.data[:, 1].contiguous(), None)
        spec.append(("wide", len(leaves), len(leaves) + 1, col.dtype))
        for part in (lo, hi):
            lf = Leaf("prim", "long", part)
            lf.torch_dtype = torch.int64
            leaves.append(lf)
        return
    if isinstance(col, PrimColumn):
        spec.append(("prim", len(leaves)))
        lf = Leaf("prim", col.dtype, col)
        lf.torch_dtype = col.data.dtype
        leaves.append(lf)
        return
    raise TypeError(f"cannot exchange column {col!r}")


def rebuild(spec_item, leaves_out, n, device):
    from ..engine.column import ArrayColumn, ConstColumn, StructColumn
    kind = spec_item[0]
    if kind == "const":
        return ConstColumn(spec_item[1], spec_item[2], n, device)
    if kind in ("prim", "str"):
        return leaves_out[spec_item[1]]
    if kind == "wide":
        from ..engine.column import PrimColumn
        lo, hi = leaves_out[spec_item[1]], leaves_out[spec_item[2]]
        return PrimColumn(spec_item[3], torch.stack([lo.data, hi.data], 1), lo.valid)
    if kind == "struct":
        _, names, is_map, dtype, vleaf, sub = spec_item
        kids = [rebuild(s, leaves_out, n, device) for s in sub]
        return StructColumn(names, kids, n, leaves_out[vleaf] if vleaf is not None else None, is_map, dtype, device)
    if kind == "array":
        _, drop, vleaf, sub, pleaves = spec_item
        els = [rebuild(s, leaves_out, n, device) for s in sub]
        pm = [leaves_out.get(p) for p in pleaves]
        present = None
        if any(p is not None for p in pm):
            ones = torch.ones(n, dtype=torch.bool, device=device)
            present = torch.stack([ones if p is None else p for p in pm], 1)
        return ArrayColumn(els, n, leaves_out[vleaf] if vleaf is not None else None, drop, device, present=present)
    raise ValueError(kind)


class Layout:
    """Leaves of a table and their matrix columns.

    Which leaves carry a validity bit must be the same on every rank of a collective, but a rank whose share of a
    column has no nulls may hold it without a validity vector.  ``flags()`` are this rank's per-leaf "has validity"
    bits; the ranks OR them (they ride along with the send sizes of a shuffle / all-gather, so agreeing costs no extra
    collective) and ``assign`` lays the matrix out for the agreed set — a leaf without local validity then sends
    all-ones."""

    def __init__(self, table):
        self.names = list(table.names)
        self.n = table.length
        self.device = table.device
        self.leaves: List[Leaf] = []
        self.spec: list = []
        for c in table.columns:
            flatten(c, self.leaves, self.spec)
        prims = [lf for lf in self.leaves if lf.kind == "prim"]
        strs = [lf for lf in self.leaves if lf.kind == "str"]
        for j, lf in enumerate(prims):
            lf.mcol = j
        for j, lf in enumerate(strs):
            lf.sidx = j
            lf.mcol = len(prims) + j
        self.P, self.S = len(prims), len(strs)
        self.prims, self.strs = prims, strs
        self.local_valid = [lf.col.valid is not None for lf in self.leaves]
        self.assign(self.local_valid)

    NFLAG_BITS = 62

    def flags(self) -> List[int]:
        """``local_valid`` as int64 words (62 bits each: exact as floats, positive)."""
        nw = max(1, (len(self.leaves) + self.NFLAG_BITS - 1) // self.NFLAG_BITS)
        out = [0] * nw
        for i, v in enumerate(self.local_valid):
            if v:
                out[i // self.NFLAG_BITS] |= 1 << (i % self.NFLAG_BITS)
        return out

    def assign_flags(self, words: List[int]) -> None:
        self.assign([bool((words[i // self.NFLAG_BITS] >> (i % self.NFLAG_BITS)) & 1)
                     for i in range(len(self.leaves))])

    def assign(self, has_valid: List[bool]) -> None:
        nv = 0
        for lf, hv in zip(self.leaves, has_valid):
            lf.vbit = nv if hv else -1
            nv += 1 if hv else 0
        self.V = nv
        self.nmask = (nv + 62) // 63
        self.C = self.P + 2 * self.S + self.nmask

    def meta(self):
        """Picklable per-leaf layout (what a receiver needs to rebuild columns it has never seen)."""
        return [(lf.kind, lf.dtype, lf.mcol, lf.sidx, lf.vbit, lf.torch_dtype, lf.str_type,
                 getattr(lf.col, "dtype", None)) for lf in self.leaves]


# ---------------------------------------------------------------------------------------------------------------
# torch reference
# ---------------------------------------------------------------------------------------------------------------

def _as_i64(d: torch.Tensor) -> torch.Tensor:
    if d.dtype == torch.float64:
        return d.view(torch.int64)
    if d.dtype == torch.float32:
        return d.view(torch.int32).to(torch.int64)
    return d if d.dtype == torch.int64 else d.to(torch.int64)


def plan_torch(lay: Layout, dest: Optional[torch.Tensor], W: int):
    """Send sizes [W, 1+S] (rows, then bytes of every string leaf, per destination) and the stable order."""
    n, dev = lay.n, lay.device
    if dest is None:
        dest = torch.zeros(n, dtype=torch.int64, device=dev)
    order = torch.argsort(dest, stable=True)
    cols = [torch.bincount(dest, minlength=W).to(torch.int64)]
    for lf in lay.strs:
        by = torch.zeros(W, dtype=torch.int64, device=dev)
        if n:
            by.index_add_(0, dest, lf.col.lens.to(torch.int64).clamp(min=0))
        cols.append(by)
    return torch.stack(cols, 1).contiguous(), (dest, order)


def scatter_torch(lay: Layout, state, send_rows: List[int], send_bytes: List[List[int]]):
    """(matrix [n, C] in destination order, [arena per string leaf])."""
    from ..ops import strings as sops
    dest, order = state
    n, dev = lay.n, lay.device
    sdest = dest[order]
    cols = []
    for lf in lay.prims:
        cols.append(_as_i64(lf.col.data[order]))
    offs_cols, arenas = [], []
    for lf in lay.strs:
        lens = lf.col.lens[order].to(torch.int64)
        cols.append(lens)
        lens_c = lens.clamp(min=0)
        excl = torch.cumsum(lens_c, 0) - lens_c
        by = _h2d(send_bytes[lf.sidx], torch.int64, dev)
        dstart = torch.cumsum(by, 0) - by
        offs_cols.append(excl - dstart[sdest] if n else excl)
        total = int(sum(send_bytes[lf.sidx]))
        sc = lf.col.take(order)
        arenas.append(sops.compact_known(sc, total).arena[:total].contiguous() if n and total else
                      torch.empty(0, dtype=torch.uint8, device=dev))
    cols += offs_cols
    masks = [torch.zeros(n, dtype=torch.int64, device=dev) for _ in range(lay.nmask)]
    for lf in lay.leaves:
        if lf.vbit >= 0:
            w, b = divmod(lf.vbit, 63)
            if lf.col.valid is None:
                masks[w] |= 1 << b
            else:
                masks[w] |= lf.col.valid[order].to(torch.int64) << b
    cols += masks
    mat = torch.stack(cols, 1).contiguous() if (cols and n) else \
        torch.empty((n, lay.C), dtype=torch.int64, device=dev)
    return mat, arenas


def unpack_torch(names, spec, meta, mat, arenas, row_prefix, src_base, byte_base, n_out, device):
    """Leaves from a received matrix: row r comes from source rank k (row_prefix), at matrix row
    ``src_base[k] + r - row_prefix[k]``; a string starts at ``byte_base[s][k]`` + its offset column."""
    from ..engine.column import PrimColumn, Table
    W = len(src_base)
    nstr = sum(1 for m in meta if m[0] == "str")
    nprim = sum(1 for m in meta if m[0] == "prim")
    dev = device
    r = torch.arange(n_out, dtype=torch.int64, device=dev)
    rp = _h2d(row_prefix, torch.int64, dev)
    k = (torch.searchsorted(rp[1:W], r, right=True) if W > 1 else torch.zeros_like(r))
    src = _h2d(src_base, torch.int64, dev)[k] + r - rp[k]
    rows = mat[src] if n_out else torch.empty((0, mat.shape[1]), dtype=torch.int64, device=dev)
    mask0 = nprim + 2 * nstr
    out = {}
    for li, (kind, dtype, mcol, sidx, vbit, tdt, stype, cdt) in enumerate(meta):
        valid = None
        if vbit >= 0:
            w, b = divmod(vbit, 63)
            valid = ((rows[:, mask0 + w] >> b) & 1).to(torch.bool)
        if kind == "prim":
            d = rows[:, mcol].contiguous()
            if tdt == torch.float64:
                d = d.view(torch.float64)
            elif tdt == torch.float32:
                d = d.to(torch.int32).view(torch.float32)
            elif tdt is not None and tdt != torch.int64:
                d = d.to(tdt)
            out[li] = PrimColumn(dtype, d, valid)
        elif kind == "str":
            bb = _h2d(byte_base[sidx], torch.int64, dev)[k]
            starts = bb + rows[:, nprim + nstr + sidx]
            out[li] = stype(arenas[sidx], starts, rows[:, mcol].to(torch.int32), valid, cdt)
        else:
            out[li] = valid
    return Table(names, [rebuild(sp, out, n_out, device) for sp in spec], n_out, device)


# ---------------------------------------------------------------------------------------------------------------
# device (exchange.hip)
# ---------------------------------------------------------------------------------------------------------------

_LIMITS = None


def _limits():
    global _LIMITS
    if _LIMITS is None:
        from ..ops import native as N
        N.register_sigs({"dxa_xchg_limits": [ctypes.c_void_p], "dxa_xchg_plan": [ctypes.c_void_p, ctypes.c_void_p],
                         "dxa_xchg_scatter": [ctypes.c_void_p, ctypes.c_void_p],
                         "dxa_xchg_unpack": [ctypes.c_void_p, ctypes.c_void_p]})
        arr = (ctypes.c_int32 * 9)()
        N.call("dxa_xchg_limits", ctypes.cast(arr, ctypes.c_void_p))
        _LIMITS = list(arr)
    return _LIMITS


class _XCol(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("kind", ctypes.c_int32), ("pad", ctypes.c_int32)]


class _XValid(ctypes.Structure):
    _fields_ = [("valid", ctypes.c_void_p), ("word", ctypes.c_int32), ("bit", ctypes.c_int32)]


class _XStr(ctypes.Structure):
    _fields_ = [("arena", ctypes.c_void_p), ("starts", ctypes.c_void_p), ("lens", ctypes.c_void_p),
                ("dst", ctypes.c_void_p)]


def _pack_args_type(L):
    maxc, maxv, maxs = L[1], L[2], L[3]

    class PackArgs(ctypes.Structure):
        _fields_ = [("dest", ctypes.c_void_p), ("n", ctypes.c_int64), ("W", ctypes.c_int32),
                    ("nblocks", ctypes.c_int32), ("ncols", ctypes.c_int32), ("nvalid", ctypes.c_int32),
                    ("nstr", ctypes.c_int32), ("C", ctypes.c_int32), ("hist", ctypes.c_void_p),
                    ("sizes", ctypes.c_void_p), ("mat", ctypes.c_void_p), ("cols", _XCol * maxc),
                    ("valids", _XValid * maxv), ("strs", _XStr * maxs), ("sizes_stride", ctypes.c_int32),
                    ("nextra", ctypes.c_int32), ("extra", ctypes.c_int64 * L[8]), ("coalesce", ctypes.c_int32),
                    ("pad1", ctypes.c_int32)]
    return PackArgs


class _UCol(ctypes.Structure):
    _fields_ = [("out", ctypes.c_void_p), ("valid", ctypes.c_void_p), ("kind", ctypes.c_int32),
                ("mcol", ctypes.c_int32), ("sidx", ctypes.c_int32), ("vword", ctypes.c_int32),
                ("vbit", ctypes.c_int32), ("pad", ctypes.c_int32), ("starts", ctypes.c_void_p)]


def _unpack_args_type(L):
    class UnpackArgs(ctypes.Structure):
        _fields_ = [("mat", ctypes.c_void_p), ("n", ctypes.c_int64), ("W", ctypes.c_int32),
                    ("nleaf", ctypes.c_int32), ("C", ctypes.c_int32), ("off_col0", ctypes.c_int32),
                    ("nstr", ctypes.c_int32), ("mask_col0", ctypes.c_int32), ("meta", ctypes.c_void_p),
                    ("leaves", _UCol * L[4])]
    return UnpackArgs


def device_ok(lay: Layout, W: int) -> bool:
    """The device kernels handle this layout (within their by-value argument limits)."""
    if lay.device.type != "cuda":
        return False
    L = _limits()
    if W > L[0] or lay.P > L[1] or len(lay.leaves) > L[2] or lay.S > L[3] or len(lay.leaves) > L[4]:
        return False
    for lf in lay.prims:
        if lf.col.data.element_size() not in _KIND:
            return False
    return True


class DevicePlan:
    """State between ``plan_device`` and ``scatter_device`` (keeps the argument block and its tensors alive)."""

    def __init__(self, args, keep, hist):
        self.args, self.keep, self.hist = args, keep, hist


def plan_device(lay: Layout, dest: Optional[torch.Tensor], W: int, extra=()):
    from ..ops import native as N
    L = _limits()
    n, dev = lay.n, lay.device
    PackArgs = _pack_args_type(L)
    a = PackArgs()
    keep = []
    if dest is not None:
        dest = dest.to(torch.int64).contiguous()
        keep.append(dest)
        a.dest = dest.data_ptr()
    a.n, a.W = n, W
    a.nblocks = max(1, (n + L[5] - 1) // L[5])
    a.ncols, a.nvalid, a.nstr, a.C = lay.P, lay.V, lay.S, lay.C
    for j, lf in enumerate(lay.prims):
        d = lf.col.data.contiguous()
        keep.append(d)
        a.cols[j] = _XCol(d.data_ptr(), _KIND[d.element_size()], 0)
    for lf in lay.strs:
        c = lf.col
        st, ln = c.starts.contiguous(), c.lens.contiguous()
        if ln.dtype != torch.int32:
            ln = ln.to(torch.int32)
        if st.dtype != torch.int64:
            st = st.to(torch.int64)
        keep += [st, ln, c.arena]
        a.strs[lf.sidx] = _XStr(c.arena.data_ptr(), st.data_ptr(), ln.data_ptr(), 0)
    hist = torch.empty((1 + lay.S) * W * a.nblocks, dtype=torch.int64, device=dev)
    sizes = torch.empty((W, 1 + lay.S + len(extra)), dtype=torch.int64, device=dev)
    a.hist, a.sizes = hist.data_ptr(), sizes.data_ptr()
    keep.append(sizes)                 # the scatter kernel reads it again (coalesced string bytes)
    a.sizes_stride, a.nextra = sizes.shape[1], len(extra)
    for i, x in enumerate(extra):
        a.extra[i] = int(x)
    N.call("dxa_xchg_plan", ctypes.byref(a), N.stream_handle(dev))
    return sizes, DevicePlan(a, keep, hist)


def scatter_device(lay: Layout, plan: DevicePlan, send_rows: List[int], send_bytes: List[List[int]],
                   rows_alloc: Optional[int] = None, bytes_alloc: Optional[List[int]] = None,
                   coalesce: bool = False):
    """Send matrix + arenas; ``rows_alloc`` / ``bytes_alloc`` over-allocate (padding for all-gathers).  With
    ``coalesce`` the arenas are ONE buffer, destination-major (``coalesced_bytes``), and ``bytes_alloc`` is its
    one-element capacity."""
    from ..ops import native as N
    a = plan.args
    n, dev = lay.n, lay.device
    # validity bits of the agreed layout (Layout.assign): a null pointer sends all-ones
    a.nvalid, a.C = lay.V, lay.C
    v = 0
    for lf in lay.leaves:
        if lf.vbit >= 0:
            w, b = divmod(lf.vbit, 63)
            ptr = 0
            if lf.col.valid is not None:
                vv = lf.col.valid.contiguous()
                if vv.dtype != torch.bool and vv.dtype != torch.uint8:
                    vv = vv.to(torch.bool)
                plan.keep.append(vv)
                ptr = vv.data_ptr()
            a.valids[v] = _XValid(ptr, w, b)
            v += 1
    R = max(n, rows_alloc or 0)
    mat = torch.empty((R, lay.C), dtype=torch.int64, device=dev)
    if R > n:
        mat[n:].zero_()
    a.mat = mat.data_ptr()
    if coalesce:
        total = sum(int(x) for b in send_bytes for x in b)
        cap = max(total, (bytes_alloc or [0])[0])
        ar = torch.empty(cap + 16, dtype=torch.uint8, device=dev)
        for lf in lay.strs:
            a.strs[lf.sidx].dst = ar.data_ptr()
        a.coalesce = 1
        N.call("dxa_xchg_scatter", ctypes.byref(a), N.stream_handle(dev))
        a.coalesce = 0
        return mat, [ar[:cap]]
    arenas = []
    for lf in lay.strs:
        total = int(sum(send_bytes[lf.sidx]))
        cap = max(total, (bytes_alloc or [0] * lay.S)[lf.sidx])
        ar = torch.empty(cap + 16, dtype=torch.uint8, device=dev)
        arenas.append(ar)
        a.strs[lf.sidx].dst = ar.data_ptr()
    N.call("dxa_xchg_scatter", ctypes.byref(a), N.stream_handle(dev))
    return mat, [ar[:max(int(sum(send_bytes[lf.sidx])), (bytes_alloc or [0] * lay.S)[lf.sidx])]
                 for ar, lf in zip(arenas, lay.strs)]


def unpack_device(names, spec, meta, mat, arenas, row_prefix, src_base, byte_base, n_out, device):
    from ..engine.column import PrimColumn, Table
    from ..ops import native as N
    L = _limits()
    W = len(src_base)
    nstr = sum(1 for m in meta if m[0] == "str")
    nprim = sum(1 for m in meta if m[0] == "prim")
    UnpackArgs = _unpack_args_type(L)
    a = UnpackArgs()
    mat = mat.contiguous()
    a.mat, a.n, a.W, a.nleaf, a.C = mat.data_ptr(), n_out, W, len(meta), int(mat.shape[1])
    a.off_col0, a.nstr, a.mask_col0 = nprim + nstr, nstr, nprim + 2 * nstr
    host_meta = list(row_prefix) + list(src_base) + [x for s in range(nstr) for x in byte_base[s]]
    m = torch.tensor(host_meta, dtype=torch.int64).pin_memory().to(device, non_blocking=True)
    a.meta = m.data_ptr()
    # every output carved from one allocation (8-byte aligned slots)
    sizes = []
    for kind, dtype, mcol, sidx, vbit, tdt, stype, cdt in meta:
        s = 0
        if kind == "prim":
            s += n_out * torch.empty(0, dtype=tdt).element_size()
        elif kind == "str":
            s += n_out * 8 + n_out * 4
        if vbit >= 0:
            s += n_out
        sizes.append((s + 7) // 8 * 8)
    pool = torch.empty(max(8, sum(sizes)), dtype=torch.uint8, device=device)
    out, pos = {}, 0
    for li, ((kind, dtype, mcol, sidx, vbit, tdt, stype, cdt), sz) in enumerate(zip(meta, sizes)):
        u = a.leaves[li]
        u.mcol, u.sidx = mcol, sidx
        u.vword, u.vbit = (vbit // 63, vbit % 63) if vbit >= 0 else (-1, 0)
        p = pos
        valid = None
        if kind == "prim":
            es = torch.empty(0, dtype=tdt).element_size()
            d = pool[p:p + n_out * es].view(tdt) if n_out else torch.empty(0, dtype=tdt, device=device)
            p += n_out * es
            u.kind, u.out = _KIND[es], (d.data_ptr() if n_out else 0)
        elif kind == "str":
            starts = pool[p:p + n_out * 8].view(torch.int64) if n_out else torch.empty(0, dtype=torch.int64,
                                                                                        device=device)
            p += n_out * 8
            lens = pool[p:p + n_out * 4].view(torch.int32) if n_out else torch.empty(0, dtype=torch.int32,
                                                                                      device=device)
            p += n_out * 4
            u.kind, u.out, u.starts = -1, (lens.data_ptr() if n_out else 0), (starts.data_ptr() if n_out else 0)
        else:
            u.kind, u.out = K8, 0
        if vbit >= 0:
            valid = pool[p:p + n_out].view(torch.bool) if n_out else torch.empty(0, dtype=torch.bool, device=device)
            u.valid = valid.data_ptr() if n_out else 0
        else:
            u.valid = 0
        if kind == "prim":
            out[li] = PrimColumn(dtype, d, valid)
        elif kind == "str":
            out[li] = stype(arenas[sidx], starts, lens, valid, cdt)
        else:
            out[li] = valid
        pos += sz
    if n_out:
        N.call("dxa_xchg_unpack", ctypes.byref(a), N.stream_handle(device))
    m.record_stream(torch.cuda.current_stream(device))
    return Table(names, [rebuild(sp, out, n_out, device) for sp in spec], n_out, device)


# ---------------------------------------------------------------------------------------------------------------
# dispatch
# ---------------------------------------------------------------------------------------------------------------

def plan(lay: Layout, dest: Optional[torch.Tensor], W: int, force_torch: bool = False, extra=()):
    """Send sizes [W, 1+S (+ len(extra))]: rows and bytes per string leaf for every destination, then ``extra``
    words repeated on every row (the device path writes them from its scan kernel: no upload, no concatenation)."""
    if not force_torch and device_ok(lay, W) and len(extra) <= _limits()[8]:
        sizes, st = plan_device(lay, dest, W, extra)
        return sizes, ("device", st)
    sizes, st = plan_torch(lay, dest, W)
    if extra:
        x = _h2d(list(extra), torch.int64, sizes.device).expand(W, -1)
        sizes = torch.cat([sizes, x], 1).contiguous()
    return sizes, ("torch", st)


def coalesced_bytes(sizes: List[List[int]]) -> Tuple[List[int], List[List[int]]]:
    """Layout of ONE destination-major byte buffer holding every string leaf: ``sizes[s][d]`` bytes of leaf s for
    rank d are at ``[d0: leaf 0 | leaf 1 | …][d1: …]`` → (bytes per rank, start of leaf s's block of rank d).
    Used for both sides of a collective: send splits / leaf bases, or received sizes per source rank."""
    S = len(sizes)
    W = len(sizes[0]) if S else 0
    per_rank, base, pos = [], [[0] * W for _ in range(S)], 0
    for d in range(W):
        start = pos
        for s in range(S):
            base[s][d] = pos
            pos += int(sizes[s][d])
        per_rank.append(pos - start)
    return per_rank, base


def scatter(lay: Layout, state, send_rows, send_bytes, rows_alloc=None, bytes_alloc=None, coalesce=False):
    """Send matrix and string bytes.  ``coalesce``: the bytes as ONE buffer laid out by ``coalesced_bytes`` (one
    collective moves every string leaf); ``bytes_alloc`` is then ``[capacity]``."""
    kind, st = state
    if kind == "device":
        return scatter_device(lay, st, send_rows, send_bytes, rows_alloc, bytes_alloc, coalesce)
    mat, arenas = scatter_torch(lay, st, send_rows, send_bytes)
    if rows_alloc and rows_alloc > mat.shape[0]:
        mat = torch.cat([mat, torch.zeros((rows_alloc - mat.shape[0], lay.C), dtype=torch.int64,
                                          device=mat.device)])
    if coalesce:
        dev = lay.device
        parts = []
        W = len(send_rows)
        for d in range(W):
            for s in range(lay.S):
                lo = sum(int(x) for x in send_bytes[s][:d])
                parts.append(arenas[s][lo:lo + int(send_bytes[s][d])])
        buf = torch.cat(parts) if parts else torch.empty(0, dtype=torch.uint8, device=dev)
        cap = (bytes_alloc or [0])[0]
        if cap > buf.shape[0]:
            buf = torch.cat([buf, torch.zeros(cap - buf.shape[0], dtype=torch.uint8, device=dev)])
        return mat, [buf]
    if bytes_alloc:
        arenas = [torch.cat([ar, torch.zeros(bytes_alloc[j] - ar.shape[0], dtype=torch.uint8, device=ar.device)])
                  if bytes_alloc[j] > ar.shape[0] else ar for j, ar in enumerate(arenas)]
    return mat, arenas


def unpack(names, spec, meta, mat, arenas, row_prefix, src_base, byte_base, n_out, device, force_torch=False):
    """``arenas`` must carry 16 readable bytes past their data (the string kernels' unaligned reads): the
    collectives receive into buffers allocated that way."""
    if not force_torch and torch.device(device).type == "cuda" and len(meta) <= _limits()[4]:
        return unpack_device(names, spec, meta, mat, arenas, row_prefix, src_base, byte_base, n_out, device)
    return unpack_torch(names, spec, meta, mat, arenas, row_prefix, src_base, byte_base, n_out, device)


def _h2d(data, dtype, device):
    from ..ops.native import h2d
    return h2d(data, dtype, device)
