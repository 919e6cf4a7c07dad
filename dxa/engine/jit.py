"""Fused expression kernels: scalar SQL expression trees → one generated HIP kernel per expression shape.

The tensor evaluator (``expr.evaluate``) runs every operator as its own PyTorch kernel, plus extra kernels for
three-valued null logic — a rule condition such as ``temperature > 80 AND humidity < 30 OR status IS NULL`` is a
dozen launches and as many full passes over HBM.  Here the whole tree becomes straight-line code in one grid-stride
loop: each row's inputs are read once, intermediates stay in registers, and one value + one validity byte are
written.  It is the MI355X counterpart of the JVM whole-stage codegen the reference relies on inside ``spark.sql``
(DataProcessing/datax-host/src/main/scala/datax/processor/CommonProcessorFactory.scala:253-289) for WHERE clauses,
projections and the rules engine's ``IF(cond, …)`` conditions (Services/DataX.Flow/DataX.Flow.CodegenRules/
Engine.cs:232-266).

Fused: numeric/boolean/timestamp columns and literals; ``+ - * / % div & | ^``, comparisons (incl. ``<=>``),
``AND/OR/NOT`` with SQL null semantics, unary ``-``/``~``, ``IS [NOT] NULL``, ``BETWEEN``, ``IN (…)``.  Any other
subtree (string predicates, function calls, …) is evaluated by the tensor evaluator and enters the kernel as an
input column, so e.g. ``deviceType = 'Heating' AND temp > 70`` still fuses the comparison and the AND.  Semantics
mirror ``expr.py`` exactly (integer ops wrap, ``x/0`` and ``x%0`` are NULL, NaN compares like torch).

Compiled with hipRTC (``dxa.ops.rtc``) on first use and cached by source; ``backend="host"`` compiles the same
row body with g++ for CPU tests.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from ..sql import ast as A
from .column import Column, ConstColumn, PrimColumn
from .decimal import is_decimal
from .types import common_type

NUMERIC = {"byte", "short", "int", "long", "double", "float", "decimal"}
FRACTIONAL = {"double", "float", "decimal"}
INTEGRAL_STORAGE = {"byte", "short", "int", "long", "timestamp", "date"}
# int64 storage of a narrower logical integer: the C cast that wraps a result to the width (JVM overflow)
_NARROW_C = {"int": "int", "short": "short", "byte": "signed char"}


def _wrap(v: str, dtype: str) -> str:
    c = _NARROW_C.get(dtype)
    return f"(long long)({c})({v})" if c else v
CTYPE = {torch.float64: "double", torch.int64: "long long", torch.bool: "unsigned char"}
MIN_ROWS = int(os.environ.get("DXA_JIT_MIN_ROWS", "65536"))
MIN_OPS = 2
ENABLED = os.environ.get("DXA_JIT", "1") != "0"
STATS = {"fused": 0, "fallback": 0}
_NOT_FUSIBLE: Dict[str, bool] = {}


class NotFusible(Exception):
    pass


@dataclass
class R:
    """Codegen result of one node: C expressions for value and validity."""
    val: str
    ok: str
    dtype: str
    nullable: bool
    const: Optional[ConstColumn] = None
    col: Optional[Column] = None


def _lit(v, dtype: str) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if dtype in FRACTIONAL:
        f = float(v)
        if math.isnan(f):
            return "__builtin_nan(\"\")"
        if math.isinf(f):
            return "__builtin_inf()" if f > 0 else "(-__builtin_inf())"
        return f"({f.hex()})"
    i = int(v)
    if i == -(1 << 63):
        return "(-9223372036854775807LL - 1)"
    return f"{i}LL"


def _c_of(dtype: str) -> str:
    if dtype == "boolean":
        return "bool"
    if dtype in FRACTIONAL:
        return "double"
    return "long long"


class _Gen:
    def __init__(self, scope, ctx, subst, evaluate):
        self.scope, self.ctx, self.subst, self.evaluate = scope, ctx, subst, evaluate
        self.inputs: List[Tuple[torch.Tensor, Optional[torch.Tensor], str]] = []
        self.lines: List[str] = []
        self.nops = 0
        self.k = 0

    def tmp(self, ctype: str, expr: str) -> str:
        name = f"t{self.k}"
        self.k += 1
        self.lines.append(f"const {ctype} {name} = {expr};")
        return name

    # ---- leaves -----------------------------------------------------------------------------------------------
    def leaf(self, col: Column) -> R:
        if isinstance(col, ConstColumn):
            dt = col.dtype
            if col.value is None:
                return R("0", "false", dt if dt in NUMERIC | INTEGRAL_STORAGE | {"boolean"} else "null", True,
                         const=col, col=col)
            if dt == "boolean" or isinstance(col.value, bool):
                return R("true" if col.value else "false", "true", "boolean", False, const=col, col=col)
            if dt in NUMERIC | INTEGRAL_STORAGE:
                return R(_lit(col.value, dt), "true", dt, False, const=col, col=col)
            if is_decimal(dt):
                # a decimal literal fuses only next to a double (Spark compares / computes that pair in double):
                # see _decimal_pair
                return R(_lit(float(col.value), "double"), "true", dt, False, const=col, col=col)
            if dt == "string":
                return R("0", "true", "string", False, const=col, col=col)      # only usable after coercion
            raise NotFusible(dt)
        if not isinstance(col, PrimColumn) or col.data.dim() != 1:
            raise NotFusible(type(col).__name__)
        dt = col.dtype
        if dt not in NUMERIC | INTEGRAL_STORAGE | {"boolean"} or col.data.dtype not in CTYPE:
            raise NotFusible(dt)
        if (col.data.dtype == torch.bool) != (dt == "boolean"):
            raise NotFusible("storage/type mismatch")
        j = len(self.inputs)
        self.inputs.append((col.data, col.valid, dt))
        raw = f"in{j}[i]"
        val = self.tmp("bool" if col.data.dtype == torch.bool else CTYPE[col.data.dtype],
                       f"{raw} != 0" if col.data.dtype == torch.bool else raw)
        if col.valid is not None:
            ok = self.tmp("bool", f"ok{j}[i] != 0")
            return R(val, ok, dt, True, col=col)
        return R(val, "true", dt, False, col=col)

    def opaque(self, e) -> R:
        """A subtree the generator does not fuse: evaluate it with the tensor evaluator, feed the result in."""
        return self.leaf(self.evaluate(e, self.scope, self.ctx, self.subst, _jit=False))

    # ---- nodes ------------------------------------------------------------------------------------------------
    def node(self, e) -> R:
        if self.subst:
            k = e.key()
            if k in self.subst:
                return self.leaf(self.subst[k])
        if isinstance(e, A.Literal):
            return self.leaf(ConstColumn(e.value, e.type, self.scope.length, self.scope.device))
        if isinstance(e, A.Ident):
            return self.leaf(self.scope.resolve(e.parts))
        try:
            return self._op(e)
        except NotFusible:
            return self.opaque(e)

    def _op(self, e) -> R:
        if isinstance(e, A.BinOp):
            if e.op in ("and", "or"):
                return self.logic(e.op, self.node(e.left), self.node(e.right))
            if e.op in ("=", "!=", "<", "<=", ">", ">=", "<=>"):
                return self.compare(e.op, self.node(e.left), self.node(e.right))
            if e.op in ("+", "-", "*", "/", "%", "div", "&", "|", "^"):
                return self.arith(e.op, self.node(e.left), self.node(e.right))
            raise NotFusible(e.op)
        if isinstance(e, A.UnaryOp):
            v = self.node(e.operand)
            if e.op == "not":
                self._need(v, {"boolean"})
                self.nops += 1
                return R(self.tmp("bool", f"!{v.val}"), v.ok, "boolean", v.nullable)
            if e.op == "-":
                self._need(v, NUMERIC)
                self.nops += 1
                if v.dtype in FRACTIONAL:
                    return R(self.tmp("double", f"-{v.val}"), v.ok, v.dtype, v.nullable)
                return R(self.tmp("long long", _wrap(f"(long long)(0ULL - (unsigned long long){v.val})", v.dtype)),
                         v.ok, v.dtype, v.nullable)
            if e.op == "~":
                self._need(v, {"byte", "short", "int", "long"})
                self.nops += 1
                return R(self.tmp("long long", f"~{v.val}"), v.ok, v.dtype, v.nullable)
            if e.op == "+":
                return v
            raise NotFusible(e.op)
        if isinstance(e, A.IsNull):
            v = self.node(e.operand)
            self.nops += 1
            return R(self.tmp("bool", f"{v.ok}" if e.negated else f"!({v.ok})"), "true", "boolean", False)
        if isinstance(e, A.Between):
            v = self.node(e.operand)
            lo = self.compare(">=", v, self.node(e.low))
            hi = self.compare("<=", v, self.node(e.high))
            r = self.logic("and", lo, hi)
            return self.not_(r) if e.negated else r
        if isinstance(e, A.InList):
            v = self.node(e.operand)
            acc = None
            for it in e.items:
                c = self.compare("=", v, self.node(it))
                acc = c if acc is None else self.logic("or", acc, c)
            return self.not_(acc) if e.negated else acc
        raise NotFusible(type(e).__name__)

    @staticmethod
    def _need(v: R, kinds):
        if v.dtype not in kinds:
            raise NotFusible(v.dtype)

    def not_(self, v: R) -> R:
        self.nops += 1
        return R(self.tmp("bool", f"!{v.val}"), v.ok, "boolean", v.nullable)

    def logic(self, op: str, a: R, b: R) -> R:
        for v in (a, b):
            if v.dtype not in ("boolean", "null"):
                raise NotFusible(v.dtype)
        self.nops += 1
        at = self.tmp("bool", f"{a.ok} && {a.val}")
        bt = self.tmp("bool", f"{b.ok} && {b.val}")
        if not (a.nullable or b.nullable):
            return R(self.tmp("bool", f"{at} {'&&' if op == 'and' else '||'} {bt}"), "true", "boolean", False)
        af = self.tmp("bool", f"{a.ok} && !{a.val}")
        bf = self.tmp("bool", f"{b.ok} && !{b.val}")
        if op == "and":
            t = self.tmp("bool", f"{at} && {bt}")
            f = self.tmp("bool", f"{af} || {bf}")
        else:
            t = self.tmp("bool", f"{at} || {bt}")
            f = self.tmp("bool", f"{af} && {bf}")
        return R(t, self.tmp("bool", f"{t} || {f}"), "boolean", True)

    def _coerce(self, a: R, b: R) -> Tuple[R, R]:
        from .expr import _coerce_const_for
        if b.const is not None and a.const is None and a.col is not None:
            b = self.leaf(_coerce_const_for(a.col, b.const))
        elif b.const is not None and a.const is None:
            if isinstance(b.const.value, str):
                raise NotFusible("string literal vs computed value")
        if a.const is not None and b.const is None and b.col is not None:
            a = self.leaf(_coerce_const_for(b.col, a.const))
        elif a.const is not None and b.const is None:
            if isinstance(a.const.value, str):
                raise NotFusible("string literal vs computed value")
        return a, b

    @staticmethod
    def _decimal_pair(a: R, b: R) -> Tuple[R, R]:
        """decimal literal ⊕ double operand → both double (Spark DecimalPrecision: a double side wins); any other
        decimal operand stays on the tensor evaluator (exact 64/128-bit lanes)."""
        if not (is_decimal(a.dtype) or is_decimal(b.dtype)):
            return a, b
        out = []
        for x, y in ((a, b), (b, a)):
            if is_decimal(x.dtype) and x.const is not None and y.dtype in FRACTIONAL:
                x = R(x.val, x.ok, "double", x.nullable, const=ConstColumn(float(x.const.value), "double",
                                                                           x.const.length, x.const.device))
            out.append(x)
        a, b = out
        if is_decimal(a.dtype) or is_decimal(b.dtype):
            raise NotFusible("decimal")
        return a, b

    def compare(self, op: str, a: R, b: R) -> R:
        if op == "<=>":
            eq = self.compare("=", a, b)
            self.nops += 1
            return R(self.tmp("bool", f"(({a.ok}) && ({b.ok}) && ({eq.ok}) && {eq.val}) || (!({a.ok}) && !({b.ok}))"),
                     "true", "boolean", False)
        a, b = self._decimal_pair(*self._coerce(a, b))
        okinds = NUMERIC | INTEGRAL_STORAGE | {"boolean", "null"}
        if a.dtype not in okinds or b.dtype not in okinds:
            raise NotFusible("compare types")
        if (a.const is not None and a.const.value is None) or (b.const is not None and b.const.value is None):
            self.nops += 1
            return R("false", "false", "boolean", True)
        self.nops += 1
        if a.dtype == "boolean" or b.dtype == "boolean":
            x, y = f"(long long)({a.val})", f"(long long)({b.val})"
        elif a.dtype in FRACTIONAL or b.dtype in FRACTIONAL:
            x, y = f"(double)({a.val})", f"(double)({b.val})"
        else:
            x, y = f"(long long)({a.val})", f"(long long)({b.val})"
        cop = {"=": "==", "!=": "!=", "<": "<", "<=": "<=", ">": ">", ">=": ">="}[op]
        nullable = a.nullable or b.nullable
        return R(self.tmp("bool", f"{x} {cop} {y}"), self._and_ok(a, b), "boolean", nullable)

    def _and_ok(self, a: R, b: R) -> str:
        if not a.nullable and not b.nullable:
            return "true"
        if not a.nullable:
            return b.ok
        if not b.nullable:
            return a.ok
        return self.tmp("bool", f"{a.ok} && {b.ok}")

    def arith(self, op: str, a: R, b: R) -> R:
        a, b = self._decimal_pair(a, b)
        kinds = NUMERIC | {"null"}
        if a.dtype not in kinds or b.dtype not in kinds:
            raise NotFusible("arith types")           # timestamps, booleans, strings: tensor evaluator
        rt = common_type(a.dtype, b.dtype)
        if op == "/":
            rt = "double"
        if rt == "null":
            rt = "int"
        st = "double" if rt in FRACTIONAL else "long"
        if op in ("&", "|", "^") and st != "long":
            raise NotFusible("bitwise on fractional")
        if (a.const is not None and a.const.value is None) or (b.const is not None and b.const.value is None):
            self.nops += 1
            return R("0", "false", rt, True)
        self.nops += 1
        ct = "double" if st == "double" else "long long"
        x, y = f"(({ct})({a.val}))", f"(({ct})({b.val}))"
        ok = self._and_ok(a, b)
        nullable = a.nullable or b.nullable
        if op in ("+", "-", "*"):
            if st == "double":
                v = f"{x} {op} {y}"
            else:
                v = _wrap(f"(long long)((unsigned long long){x} {op} (unsigned long long){y})", rt)
            return R(self.tmp(ct, v), ok, rt, nullable)
        if op in ("&", "|", "^"):
            return R(self.tmp(ct, f"{x} {op} {y}"), ok, rt, nullable)
        xs, ys = self.tmp(ct, x), self.tmp(ct, y)
        nz = self.tmp("bool", f"{ys} != 0")
        ok2 = self.tmp("bool", f"({ok}) && {nz}")
        if op == "/":
            return R(self.tmp("double", f"{nz} ? (double){xs} / (double){ys} : 0.0"), ok2, "double", True)
        if op == "%":
            if st == "double":
                v = f"{nz} ? __builtin_fmod({xs}, {ys}) : 0.0"
            else:
                v = f"({nz} && {ys} != -1LL) ? {xs} % {ys} : 0LL"
            return R(self.tmp(ct, v), ok2, rt, True)
        # div: truncating integer division
        if st == "double":
            v = f"{nz} ? (long long)__builtin_trunc({xs} / {ys}) : 0LL"
        else:
            v = (f"{nz} ? ({ys} == -1LL ? (long long)(0ULL - (unsigned long long){xs}) : {xs} / {ys}) : 0LL")
        return R(self.tmp("long long", v), ok2, "long", True)


def _params(inputs) -> List[str]:
    ps = []
    for j, (data, valid, _dt) in enumerate(inputs):
        ps.append(f"const {CTYPE[data.dtype]}* __restrict__ in{j}")
        if valid is not None:
            ps.append(f"const unsigned char* __restrict__ ok{j}")
    return ps


def _out_ctype(dtype: str) -> str:
    return "unsigned char" if dtype == "boolean" else ("double" if dtype in FRACTIONAL else "long long")


def _render(g: _Gen, res: R, name: str, host: bool) -> str:
    ps = ["long long n"] + _params(g.inputs) + [f"{_out_ctype(res.dtype)}* __restrict__ out"]
    if res.nullable:
        ps.append("unsigned char* __restrict__ out_ok")
    body = "\n    ".join(g.lines)
    store = (f"const bool okr = {res.ok};\n    out[i] = okr ? ({_out_ctype(res.dtype)})({res.val}) : "
             f"({_out_ctype(res.dtype)})0;\n    out_ok[i] = okr;") if res.nullable else \
        f"out[i] = ({_out_ctype(res.dtype)})({res.val});"
    row = f"{body}\n    {store}"
    if host:
        return (f"#include <cmath>\nextern \"C\" void {name}({', '.join(ps)}) {{\n"
                f"  for (long long i = 0; i < n; ++i) {{\n    {row}\n  }}\n}}\n")
    return (f"extern \"C\" __global__ __launch_bounds__(256) void {name}({', '.join(ps)}) {{\n"
            f"  const long long stride = (long long)gridDim.x * 256;\n"
            f"  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {{\n"
            f"    {row}\n  }}\n}}\n")


def _out_torch(dtype: str):
    return torch.bool if dtype == "boolean" else (torch.float64 if dtype in FRACTIONAL else torch.int64)


def try_fused(e, scope, ctx, subst, evaluate, backend: str = "auto") -> Optional[Column]:
    """Evaluate ``e`` as one generated kernel, or return None (caller uses the tensor evaluator)."""
    key = e.key()
    if _NOT_FUSIBLE.get(key):
        return None
    g = _Gen(scope, ctx, subst, evaluate)
    try:
        res = g._op(e)
    except NotFusible:
        _NOT_FUSIBLE[key] = True
        STATS["fallback"] += 1
        return None
    if g.nops < MIN_OPS or not g.inputs or res.dtype not in NUMERIC | INTEGRAL_STORAGE | {"boolean"}:
        _NOT_FUSIBLE[key] = True
        STATS["fallback"] += 1
        return None
    n = scope.length
    dev = scope.device
    host = backend == "host" or (backend == "auto" and dev.type != "cuda")
    name = "dxa_fused"
    src = _render(g, res, name, host)
    out = torch.empty(n, dtype=_out_torch(res.dtype), device=dev)
    out_ok = torch.empty(n, dtype=torch.bool, device=dev) if res.nullable else None
    args = [ctypes.c_longlong(n)]
    keep = []
    for data, valid, _dt in g.inputs:
        data = data.contiguous()
        keep.append(data)
        args.append(ctypes.c_void_p(data.data_ptr()))
        if valid is not None:
            v = valid.contiguous()
            keep.append(v)
            args.append(ctypes.c_void_p(v.data_ptr()))
    args.append(ctypes.c_void_p(out.data_ptr()))
    if out_ok is not None:
        args.append(ctypes.c_void_p(out_ok.data_ptr()))
    from ..ops import rtc
    if host:
        fn = getattr(rtc.host_compile(src), name)
        fn.restype = None
        fn(*args)
    else:
        from ..ops import native as N
        f = rtc.function(src, name)
        grid = max(1, min((n + 255) // 256, 65535))
        rtc.launch(f, grid, 256, N.stream_handle(dev), args)
    STATS["fused"] += 1
    rt = res.dtype if res.dtype != "null" else "boolean"
    return PrimColumn(rt, out, out_ok)


def eligible(e, scope) -> bool:
    return (ENABLED and scope.length >= MIN_ROWS and scope.device.type == "cuda"
            and isinstance(e, (A.BinOp, A.UnaryOp, A.IsNull, A.Between, A.InList))
            and not (isinstance(e, A.BinOp) and e.op == "||"))
