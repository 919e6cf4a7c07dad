"""Count host<->device synchronisations per micro-batch of a bench flow, by source line.

    python tools/sync_audit.py [--flow groupby] [--events 200000] [--batches 4] [--warmup 4]

Runs the flow's Processor on generated batches with ``torch.cuda.set_sync_debug_mode("warn")`` after ``--warmup``
batches (a window's dense state starts once it holds two panes; a cached join reads its build multiplicity once) and
prints, per (file:line in dxa/), how many synchronising calls a steady-state batch makes on the batch thread.  The
output pool's render reads (ops/serialize.py) run on other threads and are listed as well."""
import argparse
import collections
import os
import sys
import traceback
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flow", default="groupby")
    ap.add_argument("--events", type=int, default=200_000)
    ap.add_argument("--batches", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=4)
    a = ap.parse_args()
    from dxa.engine.processor import Processor, RawBatch
    from dxa.models import iot
    from dxa.ops import native
    from dxa.simulate.datagen import generate
    native.lib()
    dev = torch.device("cuda", 0)
    proc = Processor(iot.flow_settings(workdir="/tmp/dxa_sync_audit", variant=a.flow, ref_rows=1_000_000), dev,
                     pipeline_outputs=True)
    if a.flow == "join":
        proc.reference["RefDevices"] = iot.reference_table(1_000_000, dev)
    prog = iot.program()
    t0 = 1_700_000_000_000_000
    sites = collections.Counter()

    other = collections.Counter()            # syncs on other threads (the output pool's render reads)

    def hook(message, category, filename, lineno, file=None, line=None):
        import threading
        if "prototype feature" in str(message):       # the mode's own notice when it is switched on
            return
        where = sites if threading.current_thread() is threading.main_thread() else other
        st = traceback.extract_stack()[:-1]
        frames = [f for f in st if "/dxa/" in f.filename]
        if frames:
            f = frames[-1]
            where[(f.filename.split("/dxa/")[-1], f.lineno, f.name)] += 1
        else:
            where[("<other>", 0, str(message)[:60])] += 1

    for i in range(a.batches + a.warmup):
        buf, offs = generate(prog, a.events, dev, seed=i + 1, row0=i * a.events, base_ms=t0 // 1000 - 1000,
                             step_us=max(1, 1_000_000 // a.events))
        torch.cuda.synchronize()
        if i == a.warmup:
            warnings.showwarning = hook
            warnings.simplefilter("always")
            torch.cuda.set_sync_debug_mode("warn")
        proc.process_batch(RawBatch(buf, offs, a.events), t0 + i * 1_000_000, 1_000_000)
    torch.cuda.set_sync_debug_mode("default")
    proc.drain()
    total = sum(sites.values())
    print(f"# {a.flow}: {total / a.batches:.1f} synchronising calls per batch on the batch thread")
    for (f, ln, fn), c in sites.most_common():
        print(f"{c / a.batches:6.1f}  {f}:{ln}  {fn}")
    print(f"# other threads (output rendering): {sum(other.values()) / a.batches:.1f} per batch")
    for (f, ln, fn), c in other.most_common():
        print(f"{c / a.batches:6.1f}  {f}:{ln}  {fn}")


if __name__ == "__main__":
    main()
