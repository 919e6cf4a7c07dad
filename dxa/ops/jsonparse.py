"""Schema-directed JSON parsing of a batch of raw events into a nested ``StructColumn`` (the reference's
``from_json(Raw, rawSchema)``, DataProcessing/datax-host/src/main/scala/datax/processor/CommonProcessorFactory.scala:93).

A ``ParsePlan`` flattens the Spark schema into nodes (structs and leaves) and an open-addressed
(parent, FNV-1a(key)) lookup table consumed by the ``dxa_json_parse`` kernel.  Leaves can be pruned: fields no query
references are left out of the table, so the kernel skips their values without writing a column.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Set, Tuple

import numpy as np
import torch

from . import native as N
from decimal import Decimal as _Decimal

from ..engine.decimal import from_text as decimal_from_text, is_decimal, quantize as decimal_quantize
from ..engine.types import ArrayType, MapType, StructField, StructType

FT = {"struct": 0, "boolean": 1, "long": 2, "double": 3, "float": 3, "decimal": 3, "string": 4, "raw": 5,
      "timestamp": 6, "int": 7, "date": 8, "decimal_exact": 9,
      "short": 7, "byte": 7}      # smallint / tinyint: parsed as int, then range-checked (``_narrow``)
FT_DECIMAL = 9          # decimal(p,s): the kernel keeps the number token's text; decimal.hip converts it exactly
FT_SKIP = 10            # a field no statement reads (column pruning): its key still matches in schema order, its value
#                         is skipped unstored — dropping the node instead would make every such key a failed
#                         speculation plus a full-key hash (measured: -2.4 % on the groupby flow)

FNV_BASIS = 0xcbf29ce484222325
FNV_PRIME = 0x100000001b3
M64 = (1 << 64) - 1
GOLD = 0x9E3779B97F4A7C15


def _fnv1a(b: bytes) -> int:
    h = FNV_BASIS
    for c in b:
        h = ((h ^ c) * FNV_PRIME) & M64
    return h


def _fmix64(x: int) -> int:
    x ^= x >> 33
    x = (x * 0xff51afd7ed558ccd) & M64
    x ^= x >> 33
    x = (x * 0xc4ceb9fe1a85ec53) & M64
    x ^= x >> 33
    return x


def _to_i64(x: int) -> int:
    return x - (1 << 64) if x >= (1 << 63) else x


@dataclass
class Node:
    path: Tuple[str, ...]
    parent: int
    name: str
    dtype: object
    code: int
    val_slot: int = -1
    len_slot: int = -1
    dropped: bool = False      # parsed (typed), but not part of the assembled struct: a column no statement reads
    shadow: int = 0            # string leaf: index of its timestamp-shadow node (stringToTimestamp parsed in place)
    shadow_of: int = -1        # a timestamp-shadow node: the string leaf it belongs to (no key, no struct position)
    order: int = 0             # position in the schema walk (sibling order for key speculation)


class ParsePlan:
    """The parser's node table for a schema.  ``keep`` (column pruning): the raw paths statements can read; the
    other fields are either parsed as usual and dropped when the struct is assembled (the default — on MI355X the
    typed scanners beat the skipper: the groupby flow's 23 unread leaves parse in 1.57 ms per 2 M events parsed,
    1.81 ms skipped, and the headline runs 3 % faster, profiles/round5/parser/README.md), or, with
    ``skip_unread``, matched by key and skipped unstored (FT_SKIP nodes)."""

    def __init__(self, schema: StructType, keep: Optional[Set[Tuple[str, ...]]] = None, skip_unread: bool = False,
                 ts_shadow: Optional[Set[Tuple[str, ...]]] = None):
        self.schema = schema
        self.nodes: List[Node] = [Node((), -1, "", schema, 0)]
        self.keep = keep
        self.skip_unread = skip_unread
        self._build(schema, 0, ())
        # timestamp shadows: string leaves a projection feeds to stringToTimestamp get a timestamp value slot the
        # kernel fills from the same bytes (dxa_ts.h); the column carries it as `_parsed_ts`
        for path in sorted(ts_shadow or ()):
            low = tuple(p.lower() for p in path)
            for idx, nd in enumerate(self.nodes[1:], start=1):
                if tuple(p.lower() for p in nd.path) == low and nd.code == FT["string"] and not nd.shadow:
                    self.nodes.append(Node(nd.path + ("#ts",), -1, "", "timestamp", FT["timestamp"], shadow_of=idx))
                    nd.shadow = len(self.nodes) - 1
                    break
        self._kept_first()
        nv = nl = 0
        for nd in self.nodes[1:]:
            if nd.code not in (0, FT_SKIP):
                nd.val_slot = nv
                nv += 1
                if nd.code in (4, 5, FT_DECIMAL):
                    nd.len_slot = nl
                    nl += 1
        self.nval, self.nlen = nv, nl
        # output rows of the assembled columns come first (value / length slots, nodes): the kernel writes them to
        # one set of buffers and the dropped fields' rows to another, so kept columns pin only kept rows
        self.nkv = sum(1 for nd in self.nodes[:self.nkn] if nd.val_slot >= 0)
        self.nkl = sum(1 for nd in self.nodes[:self.nkn] if nd.len_slot >= 0)
        self.max_depth = max((len(nd.path) for nd in self.nodes if nd.code == 0), default=0)
        cap = 1 << max(4, math.ceil(math.log2(max(2, 2 * len(self.nodes)))))
        keys = [0] * cap
        node_of = [-1] * cap
        for idx, nd in enumerate(self.nodes[1:], start=1):
            if nd.shadow_of >= 0:
                continue
            k = _fmix64(_fnv1a(nd.name.encode("utf-8")) ^ (((nd.parent + 1) * GOLD) & M64))
            if k == 0:
                k = 1
            s = k & (cap - 1)
            while keys[s] != 0:
                s = (s + 1) & (cap - 1)
            keys[s] = k
            node_of[s] = idx
        self.lut_keys = [_to_i64(k) for k in keys]
        self.lut_node = node_of
        self.cap = cap
        # key-order speculation tables: children in schema order, key texts as zero-padded 8-byte words
        nn = len(self.nodes)
        self.first_child = [-1] * nn
        self.next_sib = [-1] * nn
        last = {}
        for idx in sorted(range(1, nn), key=lambda i: self.nodes[i].order):       # schema order
            nd = self.nodes[idx]
            if nd.shadow_of >= 0:
                continue
            if nd.parent in last:
                self.next_sib[last[nd.parent]] = idx
            else:
                self.first_child[nd.parent] = idx
            last[nd.parent] = idx
        words, self.key_word, self.key_len = [], [0] * nn, [0] * nn
        for idx, nd in enumerate(self.nodes):
            b = nd.name.encode("utf-8")
            self.key_word[idx], self.key_len[idx] = len(words), len(b)
            b += b"\0" * (-len(b) % 8)
            words += [int.from_bytes(b[i:i + 8], "little") for i in range(0, len(b), 8)]
        self.key_words = [_to_i64(w) for w in words] or [0]
        self._dev: Dict[str, Tuple[torch.Tensor, ...]] = {}

    def _kept_first(self):
        """Renumber the nodes: the root, then every assembled node (kept fields, their structs, timestamp shadows),
        then the parsed-but-dropped and FT_SKIP ones — each group in schema order.  ``order`` keeps the schema walk
        for the sibling chains."""
        for i, nd in enumerate(self.nodes):
            nd.order = i
        kept = lambda nd: not nd.dropped and nd.code != FT_SKIP           # noqa: E731
        new = [0] + [i for i in range(1, len(self.nodes)) if kept(self.nodes[i])] + \
            [i for i in range(1, len(self.nodes)) if not kept(self.nodes[i])]
        remap = {old: k for k, old in enumerate(new)}
        nodes = [self.nodes[i] for i in new]
        for nd in nodes:
            if nd.parent >= 0:
                nd.parent = remap[nd.parent]
            if nd.shadow:
                nd.shadow = remap[nd.shadow]
            if nd.shadow_of >= 0:
                nd.shadow_of = remap[nd.shadow_of]
        self.nodes = nodes
        self.nkn = 1 + sum(1 for nd in nodes[1:] if kept(nd))

    def _wanted(self, path) -> bool:
        if self.keep is None:
            return True
        return any(k[:len(path)] == path or path[:len(k)] == k for k in self.keep)

    def _build(self, st: StructType, parent: int, prefix, dropped: bool = False):
        for f in st.fields:
            path = prefix + (f.name,)
            drop = dropped or not self._wanted(path)
            if drop and self.skip_unread:
                # unread; a pruned struct keeps its schema children as FT_SKIP nodes, so the kernel walks it with
                # key speculation instead of the generic skipper (the CPU reference never visits them)
                self.nodes.append(Node(path, parent, f.name, f.dtype, FT_SKIP))
                if isinstance(f.dtype, StructType):
                    self._build_skipped(f.dtype, len(self.nodes) - 1, path)
                continue
            if isinstance(f.dtype, StructType):
                self.nodes.append(Node(path, parent, f.name, f.dtype, 0, dropped=drop))
                self._build(f.dtype, len(self.nodes) - 1, path, drop)
            elif isinstance(f.dtype, (MapType, ArrayType)):
                self.nodes.append(Node(path, parent, f.name, f.dtype, FT["raw"], dropped=drop))
            else:
                code = FT_DECIMAL if is_decimal(f.dtype) else FT.get(f.dtype, FT["string"])
                self.nodes.append(Node(path, parent, f.name, f.dtype, code, dropped=drop))

    def _build_skipped(self, st: StructType, parent: int, prefix):
        for f in st.fields:
            self.nodes.append(Node(prefix + (f.name,), parent, f.name, f.dtype, FT_SKIP))
            if isinstance(f.dtype, StructType):
                self._build_skipped(f.dtype, len(self.nodes) - 1, prefix + (f.name,))

    def string_slot_pairs(self, device) -> Optional[torch.Tensor]:
        """(value slot, length slot) of every assembled string-like field (string, raw JSON, decimal text), as a
        device int32 tensor: the kernel zeroes them per row before parsing it."""
        key = ("zslots", str(device))
        if key not in self._dev:
            pairs = [(nd.val_slot, nd.len_slot) for nd in self.nodes[1:self.nkn] if nd.code in (4, 5, FT_DECIMAL)]
            self._dev[key] = torch.tensor([v for p in pairs for v in p], dtype=torch.int32, device=device) \
                if pairs else None
        return self._dev[key]

    def device_tables(self, device):
        key = str(device)
        t = self._dev.get(key)
        if t is None:
            t = (torch.tensor(self.lut_keys, dtype=torch.int64, device=device),
                 torch.tensor(self.lut_node, dtype=torch.int32, device=device),
                 # raw-JSON leaves: bit 8 marks an array type (the value must be '[…]'; maps take '{…}')
                 torch.tensor([n.code | (0x100 if n.code == FT["raw"] and isinstance(n.dtype, ArrayType) else 0)
                               | (n.shadow << 16) for n in self.nodes], dtype=torch.int32, device=device),
                 torch.tensor([n.val_slot for n in self.nodes], dtype=torch.int32, device=device),
                 torch.tensor([n.len_slot for n in self.nodes], dtype=torch.int32, device=device),
                 torch.tensor(self.first_child, dtype=torch.int32, device=device),
                 torch.tensor(self.next_sib, dtype=torch.int32, device=device),
                 torch.tensor(self.key_word, dtype=torch.int32, device=device),
                 torch.tensor(self.key_len, dtype=torch.int32, device=device),
                 torch.tensor(self.key_words, dtype=torch.int64, device=device))
            self._dev[key] = t
        return t


def frame_records(records: Sequence[bytes], device="cpu", pin: bool = False):
    """Pack raw event payloads into one padded byte buffer + offsets (host-side framing)."""
    lens = np.fromiter((len(r) for r in records), dtype=np.int64, count=len(records))
    offs = np.zeros(len(records) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    blob = b"".join(records) + b"\0" * 16
    buf = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    o = torch.from_numpy(offs)
    if pin:
        buf, o = buf.pin_memory(), o.pin_memory()
    if torch.device(device).type != "cpu":
        buf, o = buf.to(device, non_blocking=True), o.to(device, non_blocking=True)
    return buf, o


def frame_lines_gpu(buf: torch.Tensor, length: int, expected: Optional[int] = None,
                    mismatches: Optional[list] = None) -> torch.Tensor:
    """Record offsets for '\\n'-delimited data already on the device (newline framing kernels).

    With ``expected`` (the producer's record count, e.g. from a batch header) there is no host synchronisation: every
    record must end with a newline and offsets are ``[0, nl_0 + 1, nl_1 + 1, ...]``.  The count is still verified on
    the device: if the text holds fewer newlines than ``expected`` the missing offsets are set to ``length`` (empty
    records, never uninitialised memory), and if it holds more, the extra records are not framed.  Either way a
    0-d bool device tensor "count differed" is appended to ``mismatches`` when given, for the caller to check at its
    next synchronisation point (``check_framing``).  Without ``expected`` the count is read back and empty lines are
    dropped."""
    seg = 1 << 16
    nseg = (length + seg - 1) // seg
    dev = buf.device
    if buf.data_ptr() % 16:
        buf = buf.clone()
    counts = torch.empty(max(nseg, 1), dtype=torch.int64, device=dev)
    # the count pass also keeps a 1-bit-per-byte newline mask, so the write pass reads 1/8 of the text's bytes
    bits = torch.empty(max((length + 15) // 16, 1), dtype=torch.int16, device=dev)
    st = N.stream_handle(dev)
    if length:
        N.call("dxa_count_newlines", N.ptr(buf), length, seg, N.ptr(counts), N.ptr(bits), st)
    counts = counts[:nseg]
    base = torch.cumsum(counts, 0) - counts
    total = expected if expected is not None else (int(counts.sum().item()) if nseg else 0)
    if expected is not None:
        offs = torch.empty(total + 1, dtype=torch.int64, device=dev)
        offs[:1].zero_()            # a kernel: `offs[0] = 0` is a host-synchronous scalar copy on this stack
        if length:                  # record i+1 starts after newline i
            N.call("dxa_write_newlines_bits", N.ptr(bits), length, seg, N.ptr(base), N.ptr(offs[1:]), total, 1, st)
            found = counts.sum()
            # offsets past the last newline found: empty records at the end of the text
            offs[1:].masked_fill_(torch.arange(1, total + 1, device=dev) > found, length)
            if mismatches is not None:
                mismatches.append(found != total)
        else:
            offs[1:].fill_(0)
            if mismatches is not None:
                mismatches.append(torch.full((), bool(total != 0), dtype=torch.bool, device=dev))
        return offs
    pos = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
    if length:
        N.call("dxa_write_newlines_bits", N.ptr(bits), length, seg, N.ptr(base), N.ptr(pos), total, 0, st)
    pos = pos[:total]
    ends = torch.cat([pos + 1, N.h2d([length], torch.int64, dev)])
    starts = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), pos + 1])
    keep = (ends - starts) > 1  # drop empty lines
    starts, ends = starts[keep], ends[keep]
    # contiguous offsets: record i = [offs[i], offs[i+1]); dropped empty lines only hold whitespace
    return torch.cat([starts, ends[-1:]]) if starts.numel() else torch.zeros(1, dtype=torch.int64, device=dev)


def check_framing(mismatches: list):
    """Raise if any ``frame_lines_gpu(..., expected=..., mismatches=...)`` call saw a record count other than the
    producer's (one host synchronisation for all of them)."""
    if mismatches:
        bad = int(torch.stack([m.reshape(()) for m in mismatches]).sum().item())
        mismatches.clear()
        if bad:
            raise ValueError(f"{bad} framed batch(es) held a different record count than their producer declared")


def parse(buf: torch.Tensor, offs: torch.Tensor, plan: ParsePlan, ends: Optional[torch.Tensor] = None):
    """Parse records ``buf[offs[i]:offs[i+1]]`` (or ``buf[offs[i]:ends[i]]`` when the records are not back to
    back, e.g. Kafka record values) → (Raw StructColumn, row_ok bool tensor)."""
    return parse_async(buf, offs, plan, ends).result()


class PendingParse:
    """A parse whose kernels are queued: ``result()`` waits only for its per-field null counts (a few bytes copied
    to pinned memory behind the kernels), then assembles the columns.  ``Processor.prepare`` starts batch t+1's
    parse while batch t is still being planned, so the wait is normally already over."""

    def __init__(self, done=None, plan=None, arena=None, parts=None, n=0, counts=None, event=None, stream=None):
        self._done = done
        self.plan, self.arena, self.parts, self.n = plan, arena, parts, n
        self.counts, self.event, self.stream = counts, event, stream

    def result(self):
        if self._done is None:
            if self.event is not None:
                self.event.synchronize()
            nulls = self.counts.tolist() if self.counts is not None else [1] * len(self.plan.nodes)
            vals, lens, valid, row_ok = self.parts
            if self.stream is not None and self.arena is not None:
                cur = torch.cuda.current_stream(self.arena.device)
                if cur != self.stream:
                    # parsed on a side stream (Processor.prepare): the host already waited for it, so the consumer
                    # stream needs no device wait, but the caching allocator must not hand these blocks back to the
                    # parse stream while the consumer's kernels may still read them
                    for t in (vals, lens, valid, row_ok, self.arena):
                        t.record_stream(cur)
            ps = getattr(self, "pane_stats", None)
            if ps is not None:
                from ..engine.windows import register_pane_stats
                for (slot, _row), st in zip(ps[0], ps[1].tolist()):
                    register_pane_stats(vals[slot].data_ptr(), self.n, st, self.arena.data_ptr())
            self._done = (_assemble(self.plan, self.arena, vals, lens, valid, self.n, nulls), row_ok)
            self.parts = self.arena = self.counts = self.event = self.stream = None
        return self._done


def parse_async(buf: torch.Tensor, offs: torch.Tensor, plan: ParsePlan,
                ends: Optional[torch.Tensor] = None) -> PendingParse:
    n = int(offs.shape[0]) - 1
    if buf.device.type == "cuda" and plan.max_depth < GPU_MAX_DEPTH:
        return _parse_gpu_async(buf, offs, n, plan, ends)
    if buf.device.type == "cuda":
        # schemas nested deeper than the kernel's register stack parse on the host (same semantics)
        col, ok = _parse_cpu(buf.cpu(), offs.cpu(), n, plan, None if ends is None else ends.cpu())
        return PendingParse(done=(col.to(buf.device), ok.to(buf.device)))
    return PendingParse(done=_parse_cpu(buf, offs, n, plan, ends))


GPU_MAX_DEPTH = 8      # json_parse.hip kMaxDepth: struct nesting tracked in registers


def _parse_gpu(buf, offs, n, plan: ParsePlan, ends=None):
    return _parse_gpu_async(buf, offs, n, plan, ends).result()


def _parse_gpu_async(buf, offs, n, plan: ParsePlan, ends=None) -> PendingParse:
    lut_k, lut_n, types, vslot, lslot, fchild, nsib, kword, klen, kwords = plan.device_tables(buf.device)
    nn = len(plan.nodes)
    m = max(n, 1)
    vals = torch.empty((max(1, plan.nkv), m), dtype=torch.int64, device=buf.device)
    # a null string must still be a valid (empty) view for the kernels that copy / hash / split every row of a
    # column without looking at validity: the kernel zeroes every assembled string's start and length per row
    lens = torch.empty((max(1, plan.nkl), m), dtype=torch.int32, device=buf.device)
    valid = torch.empty((plan.nkn, m), dtype=torch.uint8, device=buf.device)
    # rows of parsed-but-dropped fields (column pruning): written by the kernel, never assembled, freed with this
    # frame (their block goes back to this stream's pool behind the kernel)
    vals2 = torch.empty((max(1, plan.nval - plan.nkv), m), dtype=torch.int64, device=buf.device)
    lens2 = torch.empty((max(1, plan.nlen - plan.nkl), m), dtype=torch.int32, device=buf.device)
    valid2 = torch.empty((max(1, nn - plan.nkn), m), dtype=torch.uint8, device=buf.device)
    row_ok = torch.empty(max(n, 1), dtype=torch.uint8, device=buf.device)
    zs = plan.string_slot_pairs(buf.device)
    counts = event = pane_stats = None
    if n:
        st = N.stream_handle(buf.device)
        N.call("dxa_json_parse", N.ptr(buf), N.ptr(offs), n, N.ptr(lut_k), N.ptr(lut_n), plan.cap, N.ptr(types),
               N.ptr(vslot), N.ptr(lslot), nn, N.ptr(vals), N.ptr(lens), N.ptr(valid), N.ptr(row_ok),
               N.ptr(fchild), N.ptr(nsib), N.ptr(kword), N.ptr(klen), N.ptr(kwords), int(kwords.numel()),
               None if ends is None else N.ptr(ends), N.ptr(vals2), N.ptr(lens2), N.ptr(valid2), plan.nkv,
               plan.nkl, plan.nkn, N.ptr(zs), 0 if zs is None else zs.numel() // 2, st)
        nk = plan.nkn
        cnt = torch.empty(nk, dtype=torch.int64, device=buf.device)
        N.call("dxa_null_counts", N.ptr(valid), n, nk, N.ptr(cnt), st)      # the assembled nodes only
        counts = torch.empty(nk, dtype=torch.int64, pin_memory=True)
        counts.copy_(cnt, non_blocking=True)     # a few bytes behind the kernels; read in result()
        shadows = [(plan.nodes[i].val_slot, i) for i in range(1, plan.nkn) if plan.nodes[i].shadow_of >= 0]
        if shadows:
            # a window pane's statistics of every timestamp shadow, queued here with the parse (windows.py)
            from ..engine.windows import queue_pane_stats
            pst = queue_pane_stats(vals, valid, lens[:plan.nkl] if plan.nkl else lens[:0], n, shadows)
            pane_stats = (shadows, torch.empty(pst.shape, dtype=torch.int64, pin_memory=True))
            pane_stats[1].copy_(pst, non_blocking=True)
        event = torch.cuda.Event()
        event.record(torch.cuda.current_stream(buf.device))
    parts = (vals[:, :n], lens[:, :n], valid[:, :n].view(torch.bool), row_ok[:n].view(torch.bool))
    pp = PendingParse(plan=plan, arena=buf, parts=parts, n=n, counts=counts, event=event,
                      stream=torch.cuda.current_stream(buf.device))
    pp.pane_stats = pane_stats
    return pp


def _assemble(plan: ParsePlan, arena, vals, lens, valid, n, nulls=None):
    from ..engine.column import PrimColumn, StrColumn, JsonColumn, StructColumn
    device = arena.device
    cols: Dict[int, object] = {}
    for idx in range(len(plan.nodes) - 1, 0, -1):
        nd = plan.nodes[idx]
        if nd.code == FT_SKIP or nd.dropped or nd.shadow_of >= 0:
            continue
        v = valid[idx] if (nulls is None or nulls[idx]) else None   # complete columns carry no mask
        if nd.code == 0:
            kids = [(plan.nodes[j].name, cols[j]) for j in range(len(plan.nodes))
                    if plan.nodes[j].parent == idx and j in cols]
            cols[idx] = StructColumn([k for k, _ in kids], [c for _, c in kids], n, v, False, None, device)
            continue
        raw = vals[nd.val_slot]
        if nd.code == FT["string"]:
            cols[idx] = StrColumn(arena, raw, lens[nd.len_slot], v)
            if nd.shadow:
                sh = nd.shadow
                cols[idx]._parsed_ts = PrimColumn("timestamp", vals[plan.nodes[sh].val_slot],
                                                  valid[sh] if (nulls is None or nulls[sh]) else None)
        elif nd.code == FT["raw"]:
            cols[idx] = JsonColumn(arena, raw, lens[nd.len_slot], v, nd.dtype)
        elif nd.code == FT_DECIMAL:
            cols[idx] = decimal_from_text(StrColumn(arena, raw, lens[nd.len_slot], v), nd.dtype, trim=False)
        elif nd.code == FT["double"]:
            cols[idx] = PrimColumn(nd.dtype if nd.dtype in ("double", "float", "decimal") else "double",
                                   raw.view(torch.float64), v)
        elif nd.code == FT["boolean"]:
            cols[idx] = PrimColumn("boolean", raw != 0, v)
        elif nd.dtype in ("short", "byte"):
            # the kernel range-checks as int; a smallint / tinyint outside its own range is null, as in the
            # host parser (_convert)
            from ..engine.types import INT_RANGE
            lo, hi = INT_RANGE[nd.dtype]
            inr = (raw >= lo) & (raw <= hi)
            cols[idx] = PrimColumn(nd.dtype, raw, inr if v is None else v & inr)
        else:
            cols[idx] = PrimColumn(nd.dtype, raw, v)
    kids = [(plan.nodes[j].name, cols[j]) for j in range(1, len(plan.nodes)) if plan.nodes[j].parent == 0 and j in cols]
    root_valid = valid[0] if (nulls is None or nulls[0]) else None
    return StructColumn([k for k, _ in kids], [c for _, c in kids], n, root_valid, False, None, device)


# ------------------------------------------------------------------------------------------------------------------
# CPU reference (Python json) — same null/mismatch semantics as the kernel
# ------------------------------------------------------------------------------------------------------------------
def _iso_to_us(s: str) -> Optional[int]:
    import re
    import datetime as dt
    m = re.match(r"^(\d{4})-(\d{2})-(\d{2})(?:[T ](\d{2}):(\d{2})(?::(\d{2}))?(?:\.(\d+))?(Z|[+-]\d{2}:?(?:\d{2})?)?)?$",
                 s)
    if not m:
        return None
    y, mo, d = int(m.group(1)), int(m.group(2)), int(m.group(3))
    hh = int(m.group(4) or 0)
    mi = int(m.group(5) or 0)
    ss = int(m.group(6) or 0)
    frac = int(((m.group(7) or "") + "000000")[:6])
    tz = m.group(8)
    if not (1 <= mo <= 12 and 1 <= d <= 31 and hh <= 23 and mi <= 59 and ss <= 60):
        return None
    days = (dt.date(y, mo, 1) - dt.date(1970, 1, 1)).days + d - 1
    us = (days * 86400 + hh * 3600 + mi * 60 + ss) * 1_000_000 + frac
    if tz and tz != "Z":
        sign = -1 if tz[0] == "-" else 1
        digits = tz[1:].replace(":", "")
        th = int(digits[:2])
        tm = int(digits[2:4] or 0)
        us -= sign * (th * 3600 + tm * 60) * 1_000_000
    return us


def _floats(v):
    """JSON fractions were parsed as exact decimals; everything but decimal fields sees them as doubles."""
    if isinstance(v, _Decimal):
        return float(v)
    if isinstance(v, dict):
        return {k: _floats(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_floats(x) for x in v]
    return v


def _convert(v, dtype):
    """Python JSON value → storage value for a leaf, or None (null / mismatch)."""
    if v is None:
        return None
    if dtype in ("long", "int", "short", "byte"):
        if isinstance(v, bool) or not isinstance(v, int):
            return None
        from ..engine.types import INT_RANGE
        if not (INT_RANGE[dtype][0] <= v <= INT_RANGE[dtype][1]):
            return None
        if not (-2**63 <= v < 2**63):
            return None
        return v
    if is_decimal(dtype):
        if isinstance(v, bool) or not isinstance(v, (int, _Decimal)):
            return None
        return decimal_quantize(v, dtype)
    if dtype in ("double", "float", "decimal"):
        if isinstance(v, bool) or not isinstance(v, (int, float, _Decimal)):
            return None
        return float(v)
    if dtype == "string" and isinstance(v, _Decimal):
        return str(v)                                  # the number token's own text
    v = _floats(v)
    if dtype == "boolean":
        return v if isinstance(v, bool) else None
    if dtype == "string":
        if isinstance(v, str):
            return v
        return json.dumps(v, separators=(",", ":")) if not isinstance(v, bool) else ("true" if v else "false")
    if dtype == "timestamp":
        if isinstance(v, bool):
            return None
        if isinstance(v, int):
            if not (-2**63 <= v < 2**63):
                return None
            return ((v * 1_000_000 + 2**63) % 2**64) - 2**63      # seconds → µs, wrapping like Spark's long math
        if isinstance(v, str):
            return _iso_to_us(v)
        return None
    if dtype == "date":
        if isinstance(v, str):
            us = _iso_to_us(v)
            return None if us is None else us // 86_400_000_000
        return None
    if isinstance(dtype, (MapType, ArrayType)):
        if isinstance(dtype, MapType) and isinstance(v, dict):
            return json.dumps(v, separators=(",", ":"))
        if isinstance(dtype, ArrayType) and isinstance(v, list):
            return json.dumps(v, separators=(",", ":"))
        return None
    return None


def _parse_cpu(buf, offs, n, plan: ParsePlan, ends=None):
    from ..engine.column import column_from_pylist, strings_from_pylist, PrimColumn, StructColumn, JsonColumn
    data = buf.cpu().numpy().tobytes()
    o = offs.cpu().tolist()
    e = ends.cpu().tolist() if ends is not None else o[1:]
    recs = []
    ok = []
    for i in range(n):
        try:
            d = json.loads(data[o[i]:e[i]].decode("utf-8"), parse_float=_Decimal)
            if not isinstance(d, dict):
                raise ValueError
            recs.append(d)
            ok.append(True)
        except Exception:
            recs.append(None)
            ok.append(False)

    def build(idx, getters):
        kids = [j for j in range(1, len(plan.nodes))
                if plan.nodes[j].parent == idx and plan.nodes[j].code != FT_SKIP and not plan.nodes[j].dropped]
        names, cols = [], []
        for j in kids:
            nd = plan.nodes[j]
            vals = [None if g is None else g.get(nd.name) for g in getters]
            if nd.code == 0:
                sub = [v if isinstance(v, dict) else None for v in vals]
                col = build(j, sub)
                valid = torch.tensor([v is not None for v in sub], dtype=torch.bool)
                col = col.with_valid(valid)
            else:
                conv = [_convert(v, nd.dtype) for v in vals]
                if nd.code == FT["raw"]:
                    col = strings_from_pylist(conv, "cpu", nd.dtype)
                elif is_decimal(nd.dtype):
                    col = column_from_pylist(conv, nd.dtype, "cpu")
                elif nd.dtype in ("float", "decimal"):
                    col = column_from_pylist(conv, "double", "cpu")
                    col.dtype = nd.dtype
                else:
                    col = column_from_pylist(conv, nd.dtype, "cpu")
                if col.valid is None:
                    col.valid = torch.ones(n, dtype=torch.bool)
            names.append(nd.name)
            cols.append(col)
        return StructColumn(names, cols, n, None, False, None, "cpu")

    root = build(0, recs)
    row_ok = torch.tensor(ok, dtype=torch.bool)
    root.valid = row_ok
    return root, row_ok
