"""Device LZ4 decode throughput on bench-shaped data (SimulatedData IoT JSON lines, 16 KiB frame blocks).

    python tools/lz4_bench.py [--events 2000000] [--reps 10]
Prints one JSON line: decompressed GB/s of ``lz4.decompress_device`` (frame already in HBM)."""
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
    ap.add_argument("--block", type=int, default=16384)
    ap.add_argument("--level", type=int, default=9, help="producer compression level (0 = fast greedy)")
    a = ap.parse_args()
    from dxa.ops import native, lz4
    from dxa.models import iot
    from dxa.simulate.datagen import generate
    dev = torch.device("cuda", 0)
    native.lib()
    buf, offs = generate(iot.program(newline=True), a.events, dev, seed=1, row0=0, base_ms=1_700_000_000_000)
    total = int(offs[-1])
    host = buf[:total].cpu()
    frame = lz4.compress_frame(host, a.block, threads=16, level=a.level)
    fr = lz4.DeviceFrame.from_frame(frame, a.block).to(dev)
    out = lz4.decompress_device(fr, check=True)
    torch.cuda.synchronize()
    assert torch.equal(out[:total].cpu(), host), "device decode mismatch"
    t = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lz4.decompress_device(fr)
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    best = min(t)
    print(json.dumps({"bytes_out": total, "bytes_in": int(frame.size), "ratio": round(total / frame.size, 3),
                      "blocks": fr.comp_off.shape[0], "best_ms": round(best * 1e3, 3),
                      "median_ms": round(sorted(t)[len(t) // 2] * 1e3, 3),
                      "gbps_out": round(total / best / 1e9, 1)}))


if __name__ == "__main__":
    main()
