"""Find reference cycles that keep device tensors alive until the cyclic collector runs.

Runs bench.py in-process with the automatic collector disabled and ``DEBUG_SAVEALL``, then lists what one collection
would have freed: object types, and every tensor above 1 MiB with the chain of container types that refer to it.
Usage: python tools/gc_cycles.py [bench.py args]"""
import collections
import gc
import runpy
import sys

import torch

gc.disable()
gc.set_debug(gc.DEBUG_SAVEALL)
sys.argv = ["bench.py"] + sys.argv[1:]
try:
    runpy.run_path("bench.py", run_name="__main__")
except SystemExit:
    pass
gc.collect()
g = gc.garbage
ids = {id(o) for o in g}
cnt = collections.Counter(type(o).__module__ + "." + type(o).__qualname__ for o in g)
print("garbage objects", len(g))
for k, v in cnt.most_common(30):
    print(f"{v:6d} {k}")
tens = [o for o in g if isinstance(o, torch.Tensor)]
big = [t for t in tens if t.numel() * t.element_size() > (int(__import__("os").environ.get("GC_MIN_BYTES", 1 << 20)))]
print("tensors in cycles", len(tens), "bytes", sum(t.numel() * t.element_size() for t in tens), "big", len(big))


def describe(o):
    t = type(o).__qualname__
    if isinstance(o, dict):
        return t + "{" + ",".join(str(k) for k in list(o)[:6]) + "}"
    if type(o).__name__ == "function":
        return "function " + o.__qualname__
    if type(o).__name__ == "cell":
        return "cell"
    if type(o).__name__ == "frame":
        return f"frame {o.f_code.co_name}@{o.f_code.co_filename.split('/')[-1]}:{o.f_lineno}"
    return t


seen = set()
for t in big[:12]:
    chain, cur = [], t
    for _ in range(8):
        refs = [r for r in gc.get_referrers(cur) if id(r) in ids and r is not g]
        if not refs:
            break
        cur = refs[0]
        chain.append(describe(cur))
    key = tuple(chain)
    if key in seen:
        continue
    seen.add(key)
    print(tuple(t.shape), t.dtype, t.device, "<-", " <- ".join(chain))
frames = [o for o in g if type(o).__name__ == "frame"]
for f in frames[:10]:
    print("frame", describe(f))
