"""Device radix argsort (dxa.ops.sort, radix_sort.hip) vs torch.argsort(stable=True) on int64 keys.

    python tools/sort_bench.py [--n 2000000]
Prints one JSON line per key shape: best ms of each and the number of radix passes the byte skipping left."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def best(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    return min(t) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from dxa.ops import native, sort as SO
    native.lib()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    shapes = {
        "random64": torch.randint(-(2**62), 2**62, (a.n,), device=dev, generator=g),
        "ids_0_10k": torch.randint(0, 10_000, (a.n,), device=dev, generator=g),
        "ts_ms_1day": 1_700_000_000_000 + torch.randint(0, 86_400_000, (a.n,), device=dev, generator=g),
    }
    for name, k in shapes.items():
        key = SO.order_key(k, "int")
        hist_passes = int((torch.stack([torch.bincount(((key >> (8 * b)) & 255), minlength=256).amax()
                                        for b in range(8)]) < a.n).sum())
        ours = best(lambda: SO.argsort_words([key]), a.reps)
        ref = best(lambda: torch.argsort(k, stable=True), a.reps)
        assert torch.equal(SO.argsort_words([key]), torch.argsort(k, stable=True))
        print(json.dumps({"keys": name, "n": a.n, "radix_passes": hist_passes, "dxa_radix_ms": round(ours, 3),
                          "torch_argsort_stable_ms": round(ref, 3)}))


if __name__ == "__main__":
    main()
