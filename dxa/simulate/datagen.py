"""Schema-driven synthetic event generation (SimulatedData / DataGenerator compatible schemas) on the GPU.

Two schema dialects are accepted:
* SimulatedData ``DataSchema`` fields (Services/DataX.SimulatedData/DataX.SimulatedData.DataGenService/Model/
  DataSchema.cs; rendered as in DataGen.cs:115-227): ``int|long`` with ``minRange/maxRange``, ``double|decimal``,
  ``string`` with ``valueList``, ``dateTime`` with ``datetimeStringFormat``/``utcAddSeconds``, ``struct``,
  ``array`` of doubles, constant ``value``, ``castAsString``;
* Spark ``StructType`` JSON with DataGenerator metadata (DataProcessing/datax-utility/src/main/scala/datax/utility/
  DataGenerator.scala:20-167): ``minValue/maxValue/allowedValues/maxLength/useCurrentTimeMillis``, 10 % nulls on
  nullable fields.

``compile_*`` produce an op program for ``datagen.hip``; ``generate`` renders N events straight into device memory
(length pass → scan → render pass) and returns (buf, offs) ready for the parser.  ``generate_cpu`` is the bit-exact
host reference of the same program.
"""
from __future__ import annotations

import ctypes
import json
import struct
import time
from dataclasses import dataclass, field
from typing import Any, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..engine.types import ArrayType, MapType, StructType, from_json_obj
from ..ops import native as N

OP_LIT, OP_INT, OP_DBL, OP_CHOICE, OP_TS_MS, OP_TS_STR, OP_BOOL, OP_ALNUM, OP_NULLP = range(9)

N.register_sigs({
    "dxa_datagen_op_size": [],
    "dxa_datagen_lengths": [N.c_p, N.c_i32, N.c_p, N.c_i32, N.c_p, N.c_i32, ctypes.c_uint64, N.c_i64, N.c_i64,
                            N.c_i64, N.c_i64, N.c_p, N.c_p],
    "dxa_datagen_write": [N.c_p, N.c_i32, N.c_p, N.c_i32, N.c_p, N.c_i32, ctypes.c_uint64, N.c_i64, N.c_i64, N.c_i64,
                          N.c_i64, N.c_p, N.c_p, N.c_p],
    "dxa_datagen_slotted": [N.c_p, N.c_i32, N.c_p, N.c_i32, N.c_p, N.c_i32, ctypes.c_uint64, N.c_i64, N.c_i64,
                            N.c_i64, N.c_i64, N.c_i64, N.c_p, N.c_p, N.c_p, N.c_p],
})


@dataclass
class GenProgram:
    ops: List[Tuple[int, int, int, int, int]] = field(default_factory=list)   # code, a, b, x, y
    pool: bytearray = field(default_factory=bytearray)
    table: List[Tuple[int, int]] = field(default_factory=list)

    def _align(self):
        """Text starts 8-B aligned with zero padding before it: the device reads literals as 8-B words."""
        self.pool += b"\0" * (-len(self.pool) % 8)

    def lit(self, s: str | bytes):
        b = s.encode() if isinstance(s, str) else s
        if self.ops and self.ops[-1][0] == OP_LIT and self.ops[-1][1] + self.ops[-1][2] == len(self.pool):
            c, a, ln, x, y = self.ops[-1]
            self.pool += b
            self.ops[-1] = (c, a, ln + len(b), x, y)
            return
        self._align()
        self.ops.append((OP_LIT, len(self.pool), len(b), 0, 0))
        self.pool += b

    def choice(self, rendered: Sequence[str]):
        start = len(self.table)
        for r in rendered:
            b = r.encode()
            self._align()
            self.table.append((len(self.pool), len(b)))
            self.pool += b
        self.ops.append((OP_CHOICE, start, len(rendered), 0, 0))

    def op(self, code, a=0, b=0, x=0, y=0):
        self.ops.append((code, a, b, x, y))

    def max_len(self) -> int:
        """Upper bound of one rendered event's length: every op at its longest text (a NULLP op may only shorten
        the ops it skips, so it adds its own 4 bytes).  Sizes the slots of ``generate_slotted``."""
        import math
        total = 0
        for code, a, b, x, y in self.ops:
            if code == OP_LIT:
                total += b
            elif code == OP_INT:
                total += max(len(str(x)), len(str(y))) if x <= y else 21
            elif code == OP_DBL:
                lo = struct.unpack("<d", struct.pack("<q", x))[0]
                hi = struct.unpack("<d", struct.pack("<q", y))[0]
                m = max(abs(lo), abs(hi))
                ip = len(str(int(m) + 1)) if math.isfinite(m) and m < 1e18 else 20
                total += 1 + ip + 1 + a                 # sign, integer part (+1 for rounding up), '.', decimals
            elif code == OP_CHOICE:
                total += max((ln for _, ln in self.table[a:a + b]), default=0)
            elif code == OP_TS_MS:
                total += 20
            elif code == OP_TS_STR:
                total += 40
            elif code == OP_BOOL:
                total += 5
            elif code == OP_ALNUM:
                total += a + 2
            elif code == OP_NULLP:
                total += 4
        return total

    # -- device upload --------------------------------------------------------------------------------------------
    def device(self, device):
        key = str(device)
        cache = getattr(self, "_dev", {})
        if key in cache:
            return cache[key]
        raw = b"".join(struct.pack("<iiiiqq", c, a, b, 0, x, y) for c, a, b, x, y in self.ops)
        ops = N.h2d(raw or b"\0" * 32, torch.uint8, device)
        pad = b"\0" * (-len(self.pool) % 8 + 16)
        pool = N.h2d(bytes(self.pool) + pad, torch.uint8, device)
        tab = N.h2d([v for p in self.table for v in p] or [0, 0], torch.int32, device)
        cache[key] = (ops, pool, tab)
        self._dev = cache
        return cache[key]


def _dbl_bits(v: float) -> int:
    return struct.unpack("<q", struct.pack("<d", float(v)))[0]


def _num_text(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return repr(v)
    return str(v)


# ----------------------------------------------------------------------------------------------------------------
# compilers
# ----------------------------------------------------------------------------------------------------------------

_TS_FORMATS = {"MM/dd/yyyy HH:mm:ss": 0, "yyyy-MM-ddTHH:mm:ssZ": 1, "yyyy-MM-dd'T'HH:mm:ss'Z'": 1,
               "yyyy-MM-dd HH:mm:ss": 2, "o": 1, "s": 1}


def compile_simulated(fields: List[dict], prog: Optional[GenProgram] = None) -> GenProgram:
    """SimulatedData DataSchema ``fields`` → program (one JSON object)."""
    prog = prog or GenProgram()
    prog.lit("{")
    for i, f in enumerate(fields):
        prog.lit(("," if i else "") + json.dumps(f["name"]) + ":")
        t = str(f.get("type", "string")).lower()
        cas = bool(f.get("castAsString"))
        if t == "struct":
            compile_simulated(f.get("properties", []), prog)
            continue
        if f.get("value") not in (None, ""):
            v = f["value"]
            prog.lit(str(v) if t in ("long", "int", "double") else json.dumps(str(v)))
            continue
        if f.get("minRange") not in (None, "") and f.get("maxRange") not in (None, ""):
            lo, hi = f["minRange"], f["maxRange"]
            if t == "array":
                prog.lit("[")
                for k in range(int(f.get("length", 1))):
                    if k:
                        prog.lit(",")
                    if cas:
                        prog.lit('"')
                    prog.op(OP_DBL, 4, 0, _dbl_bits(float(lo)), _dbl_bits(float(hi)))
                    if cas:
                        prog.lit('"')
                prog.lit("]")
                continue
            if cas:
                prog.lit('"')
            if t in ("long", "int"):
                prog.op(OP_INT, 0, 0, int(lo), int(hi))
            elif t in ("double", "decimal"):
                prog.op(OP_DBL, 4, 0, _dbl_bits(float(lo)), _dbl_bits(float(hi)))
            else:
                raise ValueError(f"Unknown type of data being requested on {f['name']}")
            if cas:
                prog.lit('"')
            continue
        if t == "datetime":
            fmt = _TS_FORMATS.get(f.get("datetimeStringFormat", "yyyy-MM-ddTHH:mm:ssZ"), 1)
            prog.op(OP_TS_STR, fmt, 0, int(f.get("utcAddSeconds") or 0), 0)
            continue
        if f.get("valueList"):
            prog.choice([json.dumps(str(v)) for v in f["valueList"]])
            continue
        prog.lit("null")
    prog.lit("}")
    return prog


def compile_spark(schema: StructType, prog: Optional[GenProgram] = None, null_permille: int = 100) -> GenProgram:
    """Spark StructType with DataGenerator metadata → program."""
    prog = prog or GenProgram()
    prog.lit("{")
    for i, f in enumerate(schema.fields):
        prog.lit(("," if i else "") + json.dumps(f.name) + ":")
        md = f.metadata or {}
        nested = 0
        if f.nullable and null_permille:
            prog.op(OP_NULLP, null_permille, 1)   # placeholder b fixed below
            nested = len(prog.ops) - 1
        start = len(prog.ops)
        _compile_value(prog, f.dtype, md, null_permille)
        if f.nullable and null_permille:
            code, a, _, x, y = prog.ops[nested]
            prog.ops[nested] = (code, a, len(prog.ops) - start, x, y)
    prog.lit("}")
    return prog


def _compile_value(prog: GenProgram, t, md: dict, null_permille: int):
    if isinstance(t, StructType):
        compile_spark(t, prog, null_permille)
        return
    if isinstance(t, ArrayType):
        n = int(md.get("maxLength", 3))
        prog.lit("[")
        for k in range(max(1, n)):
            if k:
                prog.lit(",")
            _compile_value(prog, t.element, {}, 0)
        prog.lit("]")
        return
    if isinstance(t, MapType):
        prog.lit('{"k":')
        _compile_value(prog, t.value, {}, 0)
        prog.lit("}")
        return
    if md.get("allowedValues") is not None:
        vals = md["allowedValues"]
        prog.choice([json.dumps(str(v)) if t == "string" else _num_text(v) for v in vals])
        return
    if t == "string" and md.get("datetimeStringFormat"):
        prog.op(OP_TS_STR, _TS_FORMATS.get(md["datetimeStringFormat"], 1), 0, int(md.get("utcAddSeconds") or 0), 0)
    elif t == "string":
        prog.op(OP_ALNUM, int(md.get("maxLength", 10)))
    elif t in ("long", "int"):
        if md.get("useCurrentTimeMillis"):
            prog.op(OP_TS_MS)
        else:
            lo = int(md.get("minValue", 0 if t == "long" else -2**31))
            hi = int(md.get("maxValue", 2**31 - 1))
            prog.op(OP_INT, 0, 0, lo, hi)
    elif t in ("double", "float", "decimal"):
        lo, hi = float(md.get("minValue", 0.0)), float(md.get("maxValue", 1.0))
        prog.op(OP_DBL, int(md.get("decimals", 4)), 0, _dbl_bits(lo), _dbl_bits(hi))
    elif t == "boolean":
        prog.op(OP_BOOL)
    elif t == "timestamp":
        prog.op(OP_TS_STR, 1)
    else:
        prog.lit("null")


# ----------------------------------------------------------------------------------------------------------------
# generation
# ----------------------------------------------------------------------------------------------------------------

def generate(prog: GenProgram, n: int, device, seed: int = 1, row0: int = 0, base_ms: Optional[int] = None,
             step_us: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Render n events into device memory → (buf uint8 [bytes+16], offs int64 [n+1])."""
    device = torch.device(device)
    base_ms = int(time.time() * 1000) if base_ms is None else base_ms
    if device.type != "cuda":
        return generate_cpu(prog, n, seed, row0, base_ms, step_us)
    return generate_finish(generate_begin(prog, n, device, seed, row0, base_ms, step_us))


@dataclass
class PendingGen:
    """A device generation whose length pass is queued (``generate_begin``); ``generate_finish`` reads the total
    size, allocates and renders.  Splitting the two lets a source queue batch t+1's length pass one step before it
    needs the bytes, so reading the size never waits behind the kernels running on the GPU."""
    prog: "GenProgram"
    n: int
    device: torch.device
    seed: int
    row0: int
    base_ms: int
    step_us: int
    offs: torch.Tensor
    total: torch.Tensor                  # offs[-1] copied to pinned host memory
    ready: Any                           # torch.cuda.Event after that copy


def generate_begin(prog: GenProgram, n: int, device, seed: int = 1, row0: int = 0, base_ms: Optional[int] = None,
                   step_us: int = 0) -> PendingGen:
    device = torch.device(device)
    base_ms = int(time.time() * 1000) if base_ms is None else base_ms
    ops, pool, tab = prog.device(device)
    st = N.stream_handle(device)
    lens = torch.empty(n, dtype=torch.int64, device=device)
    pw, ti = pool.numel() // 8, tab.numel()
    N.call("dxa_datagen_lengths", N.ptr(ops), len(prog.ops), N.ptr(pool), pw, N.ptr(tab), ti, seed & (2**64 - 1),
           row0, n, base_ms, step_us, N.ptr(lens), st)
    offs = torch.empty(n + 1, dtype=torch.int64, device=device)
    offs[:1].zero_()             # only the leading 0: the scan writes the rest (no 8 MB fill per 1 M events)
    torch.cumsum(lens, 0, out=offs[1:])
    total = torch.empty(1, dtype=torch.int64, pin_memory=True)
    total.copy_(offs[-1:], non_blocking=True)
    ready = torch.cuda.Event()
    ready.record(torch.cuda.current_stream(device))
    lens.record_stream(torch.cuda.current_stream(device))
    return PendingGen(prog, n, device, seed, row0, base_ms, step_us, offs, total, ready)


def generate_finish(p: PendingGen) -> Tuple[torch.Tensor, torch.Tensor]:
    p.ready.synchronize()
    total = int(p.total[0])
    ops, pool, tab = p.prog.device(p.device)
    pw, ti = pool.numel() // 8, tab.numel()
    buf = torch.empty(total + 16, dtype=torch.uint8, device=p.device)
    buf[total:].zero_()          # the parser's 16-B read window needs zero padding; the rest is fully written
    N.call("dxa_datagen_write", N.ptr(ops), len(p.prog.ops), N.ptr(pool), pw, N.ptr(tab), ti,
           p.seed & (2**64 - 1), p.row0, p.n, p.base_ms, p.step_us, N.ptr(p.offs), N.ptr(buf),
           N.stream_handle(p.device))
    return buf, p.offs


def generate_slotted(prog: GenProgram, n: int, device, seed: int = 1, row0: int = 0,
                     base_ms: Optional[int] = None, step_us: int = 0):
    """Render n events in ONE device pass → (buf, offs [n+1], ends [n]): event i lands in its own 16-B aligned slot
    of ``prog.max_len()`` bytes (rounded up), so there is no length pass, no scan and no host read of the total size
    before the render — the whole generation is one launch queued on the current stream.  Records have gaps between
    them, which the parser takes as it does Kafka values (``RawBatch.ends``).  Bytes are identical to ``generate``'s
    records.  On the CPU this is ``generate_cpu`` with ends = offs[1:]."""
    device = torch.device(device)
    base_ms = int(time.time() * 1000) if base_ms is None else base_ms
    if device.type != "cuda":
        buf, offs = generate_cpu(prog, n, seed, row0, base_ms, step_us)
        return buf, offs, offs[1:].clone()
    stride = max(16, (prog.max_len() + 15) // 16 * 16)
    ops, pool, tab = prog.device(device)
    buf = torch.empty(n * stride + 16, dtype=torch.uint8, device=device)
    buf[n * stride:].zero_()     # the parser's read window past the last slot
    offs = torch.empty(n + 1, dtype=torch.int64, device=device)
    ends = torch.empty(max(n, 1), dtype=torch.int64, device=device)[:n]
    if n == 0:
        offs.zero_()
        return buf, offs, ends
    N.call("dxa_datagen_slotted", N.ptr(ops), len(prog.ops), N.ptr(pool), pool.numel() // 8, N.ptr(tab), tab.numel(),
           seed & (2**64 - 1), row0, n, base_ms, step_us, stride, N.ptr(offs), N.ptr(ends), N.ptr(buf),
           N.stream_handle(device))
    return buf, offs, ends


M64 = (1 << 64) - 1


def _pick(r: int, span: int) -> int:
    """A value in [0, span) from 64 random bits (datagen.hip pick): multiply-shift of the top 32 bits below 2^32."""
    return ((r >> 32) * span) >> 32 if span <= 0xFFFFFFFF else r % span
GOLD = 0x9E3779B97F4A7C15


def _fmix(x):
    x ^= x >> 33
    x = (x * 0xff51afd7ed558ccd) & M64
    x ^= x >> 33
    x = (x * 0xc4ceb9fe1a85ec53) & M64
    x ^= x >> 33
    return x


def _rnd(seed, row, k):
    return _fmix(seed ^ _fmix((row * GOLD + k * 0x632BE59BD9B4E019) & M64))


def _civil(days):
    import datetime as dt
    d = dt.date(1970, 1, 1) + dt.timedelta(days=days)
    return d.year, d.month, d.day


def render_cpu(prog: GenProgram, row: int, seed: int, base_ms: int, step_us: int) -> bytes:
    out = bytearray()
    skip = 0
    pool = bytes(prog.pool)
    for k, (code, a, b, x, y) in enumerate(prog.ops):
        if skip:
            skip -= 1
            continue
        if code == OP_LIT:
            out += pool[a:a + b]
        elif code == OP_INT:
            span = (y - x) & M64
            out += str(x + (_pick(_rnd(seed, row, k), span) if span else 0)).encode()
        elif code == OP_DBL:
            lo, hi = struct.unpack("<d", struct.pack("<q", x))[0], struct.unpack("<d", struct.pack("<q", y))[0]
            u = (_rnd(seed, row, k) >> 11) * (1.0 / 9007199254740992.0)
            v = lo + u * (hi - lo)
            scale = 10 ** a
            fixed = _llround(v * scale)
            neg = fixed < 0
            af = -fixed if neg else fixed
            s = ("-" if neg else "") + str(af // scale)
            if a > 0:
                s += "." + str(af % scale).rjust(a, "0")
            out += s.encode()
        elif code == OP_CHOICE:
            idx = _pick(_rnd(seed, row, k), b)
            off, ln = prog.table[a + idx]
            out += pool[off:off + ln]
        elif code == OP_TS_MS:
            out += str(base_ms + (row * step_us) // 1000 + x).encode()
        elif code == OP_TS_STR:
            secs = (base_ms + (row * step_us) // 1000) // 1000 + x
            days, sod = divmod(secs, 86400)
            Y, M, D = _civil(days)
            hh, mi, ss = sod // 3600, sod // 60 % 60, sod % 60
            if a == 0:
                s = f"{M:02d}/{D:02d}/{Y} {hh:02d}:{mi:02d}:{ss:02d}"
            else:
                s = f"{Y}-{M:02d}-{D:02d}{'T' if a == 1 else ' '}{hh:02d}:{mi:02d}:{ss:02d}" + ("Z" if a == 1 else "")
            out += ('"' + s + '"').encode()
        elif code == OP_BOOL:
            out += b"true" if _rnd(seed, row, k) & 1 else b"false"
        elif code == OP_ALNUM:
            r = _rnd(seed, row, k)
            s = []
            for q in range(a):
                if (q & 7) == 7:
                    r = _fmix((r + q) & M64)
                c = r % 62
                r //= 62
                s.append(chr(48 + c) if c < 10 else chr(65 + c - 10) if c < 36 else chr(97 + c - 36))
            out += ('"' + "".join(s) + '"').encode()
        elif code == OP_NULLP:
            if _rnd(seed, row, k) % 1000 < a:
                out += b"null"
                skip = b
    return bytes(out)


def _llround(v: float) -> int:
    import math
    return int(math.floor(v + 0.5)) if v >= 0 else -int(math.floor(-v + 0.5))


def generate_cpu(prog: GenProgram, n: int, seed: int = 1, row0: int = 0, base_ms: int = 0, step_us: int = 0):
    from ..ops.jsonparse import frame_records
    recs = [render_cpu(prog, row0 + i, seed & M64, base_ms, step_us) for i in range(n)]
    return frame_records(recs)
