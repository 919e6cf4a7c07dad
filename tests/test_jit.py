"""Fused expression kernels (dxa/engine/jit.py) against the tensor evaluator (dxa/engine/expr.py).

CPU: the generated row body is compiled with g++ (``backend="host"``) and must agree with the evaluator on random
tables with nulls, NaN, zero divisors and int64 edge values; the same source also has to compile with hipRTC for
gfx950 (no device needed).  GPU: the hipRTC kernel runs on the MI355X through the evaluator's own hook and must
agree with the evaluator run with the JIT off.
"""
import random

import pytest
import torch

from dxa.engine import jit
from dxa.engine.column import ConstColumn, PrimColumn, StrColumn, column_from_pylist
from dxa.engine.expr import EvalContext, Scope, evaluate
from dxa.sql.parser import parse_expression

EXPRS = [
    "a + b * 3 > c",
    "a - b < 0 AND c >= 1.5 OR d",
    "NOT d AND (a % 7 = 3 OR b div 4 > 2)",
    "a / b > 0.5",
    "(a * b) - (a * b) = 0",
    "c BETWEEN -1.0 AND 2.5 AND a IN (1, 2, 3, 40)",
    "a NOT IN (5, 6) OR c IS NULL",
    "b IS NOT NULL AND -a > -10",
    "a <=> b",
    "c * 2 + a - b",
    "a % b + a div b",
    "(a & 12) | (b ^ 3) > 4",
    "c / 0.0 IS NULL OR c % 2.0 > 0.5",
    "s = 'x' AND a > 2",
    "a > '3' AND c < '1.5'",
    "e > 5 AND e < 100 OR a = 1",
    "a + NULL > 1 OR d",
    "d AND NULL",
    "d OR NULL",
    "c > 1e300 OR c < -1e300 OR c = c",
    # Spark integer widths: INT / SMALLINT / TINYINT arithmetic wraps to its own width (two's complement)
    "i + i > e OR i * 3 < 0",
    "-i * 2 + h",
    "h * h + t * t - 1",
    "t + t + t",
    "i + 1 < i AND h - 1 > h OR t * 2 = t + t",
]


def _table(n, seed, device):
    rnd = random.Random(seed)

    def ints():
        vals = [rnd.choice([0, 1, -1, 2, 3, 7, 40, -(1 << 63), (1 << 63) - 1, rnd.randint(-50, 50)]) for _ in range(n)]
        return PrimColumn("long", torch.tensor(vals, dtype=torch.int64, device=device),
                          torch.tensor([rnd.random() > 0.2 for _ in range(n)], device=device))

    def narrow(t):
        bits = {"int": 32, "short": 16, "byte": 8}[t]
        lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
        vals = [rnd.choice([lo, hi, lo + 1, hi - 1, 0, -1, 1, rnd.randint(lo, hi)]) for _ in range(n)]
        return PrimColumn(t, torch.tensor(vals, dtype=torch.int64, device=device),
                          torch.tensor([rnd.random() > 0.1 for _ in range(n)], device=device))

    c_vals = [rnd.choice([0.0, -0.0, 1.5, -2.25, float("nan"), float("inf"), 1e308, rnd.uniform(-3, 3)])
              for _ in range(n)]
    cols = {
        "a": ints(),
        "b": PrimColumn("long", torch.tensor([rnd.randint(-5, 5) for _ in range(n)], dtype=torch.int64,
                                             device=device)),
        "c": PrimColumn("double", torch.tensor(c_vals, dtype=torch.float64, device=device),
                        torch.tensor([rnd.random() > 0.1 for _ in range(n)], device=device)),
        "d": PrimColumn("boolean", torch.tensor([rnd.random() > 0.5 for _ in range(n)], device=device),
                        torch.tensor([rnd.random() > 0.3 for _ in range(n)], device=device)),
        "e": PrimColumn("int", torch.tensor([rnd.randint(0, 200) for _ in range(n)], dtype=torch.int64,
                                            device=device)),
        "s": column_from_pylist([rnd.choice(["x", "y", None]) for _ in range(n)], "string", device),
        "i": narrow("int"), "h": narrow("short"), "t": narrow("byte"),
    }
    names = list(cols)
    return Scope(names, [cols[k] for k in names], [None] * len(names), n, torch.device(device))


def _norm(col, n):
    """(values, valid) as python lists with null slots blanked; NaN made comparable."""
    if isinstance(col, ConstColumn):
        return [col.value] * n if col.value is not None else [None] * n
    vals = col.data.cpu().tolist()
    ok = col.valid.cpu().tolist() if col.valid is not None else [True] * n
    out = []
    for v, k in zip(vals, ok):
        if not k:
            out.append(None)
        elif isinstance(v, float) and v != v:
            out.append("nan")
        else:
            out.append(bool(v) if col.dtype == "boolean" else v)
    return out


@pytest.mark.parametrize("sql", EXPRS)
def test_host_codegen_matches_evaluator(sql):
    n = 700
    scope = _table(n, hash(sql) & 0xffff, "cpu")
    ctx = EvalContext()
    e = parse_expression(sql)
    want = evaluate(e, scope, ctx, _jit=False)
    jit._NOT_FUSIBLE.clear()
    got = jit.try_fused(e, scope, ctx, None, evaluate, backend="host")
    if got is None:
        pytest.skip("not fused (too few operators)")
    assert got.dtype == want.dtype
    assert _norm(got, n) == _norm(want, n), sql
    from dxa.engine.types import INT_RANGE
    if got.dtype in INT_RANGE:                      # every value inside its type's range
        lo, hi = INT_RANGE[got.dtype]
        assert all(v is None or lo <= v <= hi for v in _norm(got, n)), sql


def test_string_subtree_is_an_input_column():
    scope = _table(300, 3, "cpu")
    g = jit._Gen(scope, EvalContext(), None, evaluate)
    g._op(parse_expression("s = 'x' AND a > 2 AND c < 1"))
    kinds = [dt for _, _, dt in g.inputs]
    assert "boolean" in kinds and "long" in kinds and g.nops >= 3


def test_hiprtc_compiles_generated_kernel():
    """The device form of a generated kernel compiles for gfx950 with hipRTC (no GPU needed to compile)."""
    from dxa.ops import native, rtc
    try:
        native.lib()
    except Exception as ex:      # pragma: no cover - library must build in this image
        pytest.fail(f"native library: {ex}")
    scope = _table(100, 1, "cpu")
    g = jit._Gen(scope, EvalContext(), None, evaluate)
    res = g._op(parse_expression("a + b * 3 > c AND NOT d OR a % b = 1"))
    src = jit._render(g, res, "dxa_fused", host=False)
    code = rtc.compile_code_object(src, "dxa_fused")
    assert code[:4] == b"\x7fELF"


@pytest.mark.gpu
def test_gpu_fused_kernels_match_evaluator():
    assert torch.cuda.is_available()
    dev = torch.device("cuda", 0)
    n = 1 << 17
    ctx = EvalContext()
    before = jit.STATS["fused"]
    for i, sql in enumerate(EXPRS):
        scope = _table(n if i % 2 else 70_000, i, dev)
        e = parse_expression(sql)
        jit.ENABLED = False
        try:
            want = evaluate(e, scope, ctx)                 # tensor evaluator only
        finally:
            jit.ENABLED = True
        got = evaluate(e, scope, ctx)                      # JIT hook (eligible: cuda, >= 64K rows)
        assert _norm(got, scope.length) == _norm(want, scope.length), sql
    assert jit.STATS["fused"] - before >= 12               # the hipRTC path actually ran
