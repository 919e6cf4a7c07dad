"""Fused expression kernel vs tensor evaluator on a 2M-row device batch (one expression, synchronized timing).

    python tools/jit_bench.py [--rows 2000000]
Prints one JSON line per expression: ms with the JIT off/on and the number of kernels each launched."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

EXPRS = [
    "temperature * 1.8 + 32 > 100 AND humidity BETWEEN 20 AND 80 AND (pressure - 1000) / 10 < 3 OR co2 IS NULL",
    "(temperature > 30 AND humidity > 70) OR (temperature < -10 AND co2 > 1500) OR noise / 2 > 60",
    "rpm % 7 = 3 AND status IN (1, 2, 5) AND NOT motion",
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from dxa.engine import jit
    from dxa.engine.column import PrimColumn
    from dxa.engine.expr import EvalContext, Scope, evaluate
    from dxa.ops import native
    from dxa.sql.parser import parse_expression
    native.lib()
    dev = torch.device("cuda", 0)
    n = a.rows
    g = torch.Generator(device=dev).manual_seed(1)

    def f(lo, hi, null=0.05):
        return PrimColumn("double", torch.rand(n, device=dev, generator=g, dtype=torch.float64) * (hi - lo) + lo,
                          torch.rand(n, device=dev, generator=g) > null)

    def i(lo, hi):
        return PrimColumn("long", torch.randint(lo, hi, (n,), device=dev, generator=g))
    cols = {"temperature": f(-30, 50), "humidity": f(0, 100), "pressure": f(950, 1050), "co2": f(300, 2000, 0.1),
            "noise": f(20, 140), "rpm": i(0, 1000), "status": i(0, 6),
            "motion": PrimColumn("boolean", torch.rand(n, device=dev, generator=g) > 0.5)}
    scope = Scope(list(cols), list(cols.values()), [None] * len(cols), n, dev)
    ctx = EvalContext()
    for sql in EXPRS:
        e = parse_expression(sql)
        res = {}
        for mode in ("off", "on"):
            jit.ENABLED = mode == "on"
            evaluate(e, scope, ctx)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                evaluate(e, scope, ctx)
            torch.cuda.synchronize()
            res[mode] = (time.perf_counter() - t0) / a.reps * 1e3
        print(json.dumps({"expr": sql, "rows": n, "tensor_ms": round(res["off"], 3), "fused_ms": round(res["on"], 3),
                          "speedup": round(res["off"] / res["on"], 2), "jit_stats": dict(jit.STATS)}))


if __name__ == "__main__":
    main()
