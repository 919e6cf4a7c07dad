"""One device gzip of ~800 MB of serialized JSON (for rocprofv3 counter passes over gzip_chunks_kernel)."""
import sys

import torch

from dxa.ops.deflate import gzip_device
from tests.test_deflate import _json_lines

base = _json_lines(40000, seed=5) + b"\n"
data = (base * ((800 << 20) // len(base) + 1))[:800 << 20]
t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
for _ in range(2):
    out = gzip_device(t, len(data), chunk)
torch.cuda.synchronize()
print("ratio", len(data) / out.numel())
