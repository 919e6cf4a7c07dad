"""Host-side (Python) profile of a bench flow's micro-batches: cProfile over K batches after warm-up.

    python tools/host_profile.py --flow full [--events 1000000] [--warmup 8] [--batches 8]
Prints the top functions by own time and by cumulative time (the GPU work is asynchronous, so time spent
waiting in host synchronisations shows up under .item()/.tolist()/synchronize)."""
import argparse
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flow", default="full")
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    from dxa.engine.processor import Processor, RawBatch
    from dxa.models import iot
    from dxa.ops import native
    from dxa.simulate.datagen import generate
    native.lib()
    dev = torch.device(a.device)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    proc = Processor(iot.flow_settings(workdir=f"/tmp/dxa_hprof_{a.flow}", variant=a.flow, ref_rows=1_000_000), dev)
    if a.flow in ("join", "full"):
        proc.reference["RefDevices"] = iot.reference_table(1_000_000, dev)
    prog = iot.program()
    t0 = 1_700_000_000_000_000
    bufs = []
    for i in range(a.warmup + a.batches):
        bufs.append(generate(prog, a.events, dev, seed=i + 1, row0=i * a.events,
                             base_ms=t0 // 1000 - 1000, step_us=max(1, 1_000_000 // a.events)))
    sync()
    for i in range(a.warmup):
        proc.process_batch(RawBatch(bufs[i][0], bufs[i][1], a.events), t0 + i * 1_000_000, 1_000_000)
    proc.drain()
    sync()
    pr = cProfile.Profile()
    pr.enable()
    for i in range(a.warmup, a.warmup + a.batches):
        proc.process_batch(RawBatch(bufs[i][0], bufs[i][1], a.events), t0 + i * 1_000_000, 1_000_000)
    proc.drain()
    sync()
    pr.disable()
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
        print(f"==== by {key} ({a.batches} batches)")
        print("\n".join(l for l in s.getvalue().splitlines() if l.strip())[:12000])


if __name__ == "__main__":
    main()
