"""Stage-1 structural index prototype vs the engine's parser on the same bench batch (1 M SimulatedData IoT events).

    python tools/json_index_bench.py [--events 1000000] [--per-seg 64]
Prints one JSON line: median ms and GB/s of json_parse (jsonparse.parse: kernel + null counts + assembly) and of
the structural index pass, plus the structural characters per record."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def _time(fn, reps):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--per-seg", type=int, default=64)
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    from dxa.models import iot
    from dxa.ops import native
    from dxa.ops.json_index import structural_index
    from dxa.ops.jsonparse import ParsePlan, parse
    from dxa.simulate.datagen import generate
    native.lib()
    dev = torch.device("cuda", 0)
    buf, offs = generate(iot.program(), a.events, dev, seed=1, row0=0, base_ms=1_700_000_000_000)
    total = int(offs[-1])
    plan = ParsePlan(iot.iot_spark_schema())
    work = buf.clone()

    def do_parse():
        work.copy_(buf)                     # the parser un-escapes strings in place
        parse(work, offs, plan)
    copy_ms = _time(lambda: work.copy_(buf), a.reps)
    parse_ms = _time(do_parse, a.reps) - copy_ms
    counts, _ = structural_index(buf, offs, a.per_seg)
    torch.cuda.synchronize()
    index_ms = _time(lambda: structural_index(buf, offs, a.per_seg), a.reps)
    print(json.dumps({"events": a.events, "bytes": total, "per_seg": a.per_seg,
                      "parse_ms": round(parse_ms, 3), "parse_gb_s": round(total / parse_ms / 1e6, 1),
                      "index_ms": round(index_ms, 3), "index_gb_s": round(total / index_ms / 1e6, 1),
                      "structurals_per_record": round(int(counts.sum()) / a.events, 1)}))


if __name__ == "__main__":
    main()
