"""Attribute a flow's per-batch device work to source lines: every ATen op (≈ one kernel or copy launch) and every
native HIP entry point (dxa.ops.native.call) is counted under the innermost ``dxa/`` frame that issued it, and host
syncs (``_local_scalar_dense`` = .item()/.tolist(), D2H copies) are counted separately.

    python tools/launch_attrib.py --flow full --batches 8 [--events 1000000] > attrib.txt

Runs the bench's gpu-sim batches through the Processor like tests/test_flows_gpu.py; the first two batches are warmup
(not counted).  The Processor's ``torch.inference_mode`` is replaced by a no-op context here: under it the dispatch
mode sees composite ops before they decompose (``to.dtype`` no-ops, ``item``), which miscounts launches and syncs."""
from __future__ import annotations

import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CPU_MODE = "--device" in sys.argv and "cpu" in sys.argv
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


DEPTH = int(os.environ.get("ATTRIB_DEPTH", "1"))


def _site(skip_native=False):
    out = []
    for fr in reversed(traceback.extract_stack()[:-2]):
        f = fr.filename
        if "/dxa/" in f and not f.endswith("launch_attrib.py") and not (skip_native and f.endswith("native.py")):
            out.append(f"{os.path.relpath(f, ROOT).replace('dxa/', '')}:{fr.lineno} {fr.name}")
            if len(out) >= DEPTH:
                break
    return " < ".join(out) if out else "<other>"


# ATen ops that only make views / allocate: no kernel launch
NO_LAUNCH = ("view", "_unsafe_view", "slice", "select", "as_strided", "expand", "unsqueeze", "squeeze", "permute",
             "t.", "transpose", "alias", "detach", "_reshape_alias", "empty", "new_empty", "empty_strided", "set_",
             "resize_", "unbind", "split", "narrow", "lift_fresh", "_to_copy.default?", "reshape", "unfold",
             "is_pinned", "_pin_memory", "pin_memory", "split_with_sizes", "chunk", "_local_scalar_dense")


def _launches(name: str) -> bool:
    base = name.split(".")[0]
    return not any(base == x.rstrip(".") or name.startswith(x) for x in NO_LAUNCH)


class Counter(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = collections.Counter()
        self.names = collections.Counter()
        self.syncs = collections.Counter()
        self.by_name_site = collections.Counter()
        self.on = False

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        if self.on:
            name = func.__name__ if hasattr(func, "__name__") else str(func)
            dev_args = [a for a in list(args) + list((kwargs or {}).values()) if torch.is_tensor(a)]
            on_dev = True if CPU_MODE else (any(a.is_cuda for a in dev_args) or (torch.is_tensor(out) and out.is_cuda))
            if on_dev:
                site = None
                if _launches(name):
                    site = _site()
                    self.ops[site] += 1
                    self.names[name] += 1
                    self.by_name_site[(name, site)] += 1
                if "_local_scalar_dense" in name or ("copy" in name and torch.is_tensor(out) and not out.is_cuda):
                    self.syncs[site or _site()] += 1
        return out


def main():
    import contextlib
    torch.inference_mode = lambda *a, **k: contextlib.nullcontext()      # see the module docstring
    ap = argparse.ArgumentParser()
    ap.add_argument("--flow", default="full")
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    import tempfile
    from dxa.engine.processor import Processor, RawBatch
    from dxa.models import iot
    from dxa.ops import native as N
    from dxa.simulate.datagen import generate
    dev = torch.device(a.device)
    workdir = tempfile.mkdtemp(prefix="dxa_attrib_")
    extra = {"datax.job.process.pipelineoutputs": "false"}
    settings = iot.flow_settings(workdir=workdir, variant=a.flow, sink="null", extra=extra,
                                 ref_rows=100_000 if a.flow == "join" else iot.REF_ROWS)
    if a.flow == "join":
        path = settings.get("datax.job.input.default.referencedata.RefDevices.path")
        if not os.path.exists(path):
            iot.write_reference_csv(path, 100_000, "cpu")
    proc = Processor(settings, dev)
    prog = iot.program()
    cnt = Counter()
    native = collections.Counter()
    native_sites = collections.Counter()
    real_call = N.call

    def counting_call(name, *args):
        if cnt.on:
            native[name] += 1
            native_sites[_site(skip_native=True)] += 1
        return real_call(name, *args)
    N.call = counting_call
    interval = 1_000_000
    t0 = 1_700_000_000_000_000
    with cnt:
        for i in range(a.batches + 2):
            bt = t0 + i * interval
            buf, offs = generate(prog, a.events, dev, seed=7919 + i, row0=i * a.events, base_ms=t0 // 1000 - interval // 1000,
                                 step_us=max(1, interval // a.events))
            if dev.type == "cuda":
                torch.cuda.synchronize()
            cnt.on = i >= 2
            proc.process_batch(RawBatch(buf, offs, a.events), bt, interval)
            proc.drain()
            if dev.type == "cuda":
                torch.cuda.synchronize()
            cnt.on = False
    nb = a.batches
    tot_ops = sum(cnt.ops.values())
    tot_native = sum(native.values())
    print(f"flow={a.flow} events/batch={a.events} batches={nb}")
    print(f"per batch: {tot_ops / nb:.1f} ATen device ops, {tot_native / nb:.1f} native launches, "
          f"{sum(cnt.syncs.values()) / nb:.1f} host syncs (item/tolist/D2H)")
    print("\n== ATen ops by site (per batch)")
    for s, c in cnt.ops.most_common(a.top):
        print(f"{c / nb:7.1f}  {s}")
    print("\n== ATen ops by name (per batch)")
    for s, c in cnt.names.most_common(40):
        print(f"{c / nb:7.1f}  {s}")
    print("\n== (op, site) pairs (per batch)")
    for (nm, st), c in cnt.by_name_site.most_common(50):
        print(f"{c / nb:7.1f}  {nm:28s} {st}")
    print("\n== host syncs by site (per batch)")
    for s, c in cnt.syncs.most_common(40):
        print(f"{c / nb:7.1f}  {s}")
    print("\n== native launches by entry point (per batch)")
    for s, c in native.most_common(40):
        print(f"{c / nb:7.1f}  {s}")
    print("\n== native launches by site (per batch)")
    for s, c in native_sites.most_common(40):
        print(f"{c / nb:7.1f}  {s}")


if __name__ == "__main__":
    main()
