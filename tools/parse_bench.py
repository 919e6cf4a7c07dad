"""JSON parse kernel throughput on bench-shaped data (2M SimulatedData IoT events, full 32-leaf schema).

    python tools/parse_bench.py [--events 2000000]
Prints one JSON line: best/median ms of ``jsonparse.parse`` (device buffer already framed) and GB/s."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--pruned", action="store_true",
                    help="keep only the groupby flow's fields (the rest parsed and dropped at assembly, as after pruning)")
    ap.add_argument("--skip-unread", action="store_true",
                    help="with --pruned: the unread fields as FT_SKIP nodes (matched by key, skipped unstored)")
    a = ap.parse_args()
    from dxa.models import iot
    from dxa.ops import native
    from dxa.ops.jsonparse import ParsePlan, parse
    from dxa.simulate.datagen import generate
    native.lib()
    dev = torch.device("cuda", 0)
    buf, offs = generate(iot.program(), a.events, dev, seed=1, row0=0, base_ms=1_700_000_000_000)
    keep = None
    if a.pruned:
        keep = {("deviceDetails", f) for f in ("deviceId", "deviceType", "homeId", "status", "eventTime")} | \
               {("telemetry", f) for f in ("temperature", "humidity", "power", "batteryLevel")}
    plan = ParsePlan(iot.iot_spark_schema(), keep, skip_unread=a.skip_unread)
    parse(buf, offs, plan)
    torch.cuda.synchronize()
    t = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        parse(buf, offs, plan)
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    total = int(offs[-1])
    print(json.dumps({"events": a.events, "pruned": a.pruned, "skip_unread": a.skip_unread, "bytes": total, "best_ms": round(min(t) * 1e3, 3),
                      "median_ms": round(sorted(t)[len(t) // 2] * 1e3, 3),
                      "gbps": round(total / min(t) / 1e9, 1)}))


if __name__ == "__main__":
    main()
