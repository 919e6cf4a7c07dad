"""Where do a flow's framework ("glue") kernels come from?  Runs bench.py's flow for a few batches under a
TorchDispatchMode that records every ATen op launched on a large CUDA tensor (copies, casts, fills, cats,
arithmetic, scans) with the engine frame that called it, and prints the origins by count.

    python tools/op_origins.py --flow window [--batches 4] [--min-numel 100000]
"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

# ops that only make views (no kernel)
VIEWS = {"select", "slice", "view", "_unsafe_view", "as_strided", "t", "transpose", "unsqueeze", "squeeze", "expand",
         "alias", "detach", "permute", "narrow", "unbind", "split", "split_with_sizes", "lift_fresh", "empty",
         "empty_strided", "_local_scalar_dense", "is_nonzero", "unfold", "view_as_real", "view_as_complex",
         "empty_like", "new_empty", "new_empty_strided", "record_stream", "set_", "resize_", "_reshape_alias"}


class Origins(TorchDispatchMode):
    def __init__(self, min_numel):
        super().__init__()
        self.min = min_numel
        self.hits = collections.Counter()
        self.on = False

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        if self.on:
            name = func.overloadpacket.__name__
            big = any(isinstance(t, torch.Tensor) and t.is_cuda and t.numel() >= self.min
                      for t in list(args) + [out] if isinstance(t, torch.Tensor))
            if big and name not in VIEWS:
                frames = [f for f in traceback.extract_stack()[:-2] if "/dxa/" in f.filename]
                where = " <- ".join(f"{f.filename.split('/dxa/')[-1]}:{f.lineno}({f.name})" for f in frames[-4:][::-1])
                t0 = next((t for t in args if isinstance(t, torch.Tensor)), None)
                sig = "" if t0 is None else f"{str(t0.dtype)[6:]}{list(t0.shape)}{'' if t0.is_contiguous() else '!c'}"
                if isinstance(out, torch.Tensor):
                    sig += f"->{str(out.dtype)[6:]}{'=' if t0 is not None and out.data_ptr() == t0.data_ptr() else ''}"
                self.hits[(f"{name} {sig}", where)] += 1
        return out


def _no_inference_mode():
    """The Processor runs batches under torch.inference_mode, where the dispatch mode sees composite ops before
    they decompose (``to`` that copies nothing); attribute the decomposed ops instead."""
    import contextlib
    torch.inference_mode = lambda *a, **k: contextlib.nullcontext()


def main():
    _no_inference_mode()
    ap = argparse.ArgumentParser()
    ap.add_argument("--flow", default="window")
    ap.add_argument("--batches", type=int, default=4)
    ap.add_argument("--min-numel", type=int, default=100_000)
    a = ap.parse_args()
    from dxa.engine.processor import Processor, RawBatch
    from dxa.models import iot
    from dxa.simulate.datagen import generate
    dev = torch.device("cuda", 0)
    extra = {"datax.job.process.pipelineoutputs": "false"}
    proc = Processor(iot.flow_settings(variant=a.flow, sink="null", extra=extra, ref_rows=100_000), dev)
    prog = iot.program()
    n = 1_000_000
    mode = Origins(a.min_numel)
    t0 = 1_700_000_000_000_000
    with mode:
        for i in range(a.batches + 2):
            bt = t0 + i * 1_000_000
            # bench.py sim_gen_args: a constant base, so batch i's events fall in the interval before its batch time
            buf, offs = generate(prog, n, dev, seed=11 + i, row0=i * n, base_ms=(t0 - 1_000_000) // 1000, step_us=1)
            mode.on = i >= 2                                     # after the first batches (layouts, caches)
            proc.process_batch(RawBatch(buf, offs, n), bt, 1_000_000)
            proc.drain()
            torch.cuda.synchronize()
    for (name, where), k in mode.hits.most_common(40):
        print(f"{k / a.batches:5.1f}/batch  {name:40s} {where}")


if __name__ == "__main__":
    main()
