"""Device gzip throughput / ratio on serialized IoT JSON (the passthrough flow's output) vs host zlib level 6."""
import gzip
import time
import zlib

import torch

from dxa.ops.deflate import gzip_device
from tests.test_deflate import _json_lines

base = _json_lines(40000, seed=5)
reps = (800 << 20) // len(base) + 1
data = (base + b"\n") * reps
data = data[:800 << 20]
t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
for chunk, dyn in ((4096, False), (8192, False), (16384, False), (32768, False), (8192, True), (32768, True)):
    out = gzip_device(t, len(data), chunk, dyn)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        out = gzip_device(t, len(data), chunk, dyn)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    host = bytes(out[:4 << 20].cpu().numpy())
    print(f"chunk {chunk:6} {'dynamic' if dyn else 'fixed  '}: {len(data) / dt / 1e9:6.1f} GB/s in, ratio {len(data) / out.numel():5.2f}, "
          f"{dt * 1e3:6.2f} ms per 800 MB")
full = bytes(out.cpu().numpy())
assert gzip.decompress(full) == data
t0 = time.perf_counter()
z = zlib.compress(data[:64 << 20], 6)
print(f"host zlib level 6: {64 / (time.perf_counter() - t0):.0f} MB/s per thread, ratio {(64 << 20) / len(z):.2f}")
