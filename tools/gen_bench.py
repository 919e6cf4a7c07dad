"""GPU event generator throughput on bench-shaped data (SimulatedData IoT events, 32-leaf schema).

    python tools/gen_bench.py [--events 1000000]
Prints one JSON line: best/median ms of ``datagen.generate`` (length pass + scan + write pass) and GB/s written."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from dxa.models import iot
    from dxa.ops import native
    from dxa.simulate.datagen import generate
    native.lib()
    dev = torch.device("cuda", 0)
    prog = iot.program()
    buf, offs = generate(prog, a.events, dev, seed=1, row0=0, base_ms=1_700_000_000_000, step_us=1)
    torch.cuda.synchronize()
    t = []
    for r in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        buf, offs = generate(prog, a.events, dev, seed=r + 2, row0=r * a.events, base_ms=1_700_000_000_000,
                             step_us=1)
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    total = int(offs[-1])
    best = min(t)
    print(json.dumps({"events": a.events, "bytes": total, "best_ms": round(best * 1e3, 3),
                      "median_ms": round(sorted(t)[len(t) // 2] * 1e3, 3),
                      "GB_per_s": round(total / best / 1e9, 1)}))


if __name__ == "__main__":
    main()
