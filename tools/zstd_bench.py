"""zstd frame decoder (zstd.hip) on bench-shaped frames: SimulatedData IoT events, 26 records per frame (the Kafka
record batch the bench's producer writes), compressed by libzstd at --level.

    python tools/zstd_bench.py [--events 1000000] [--per 26] [--level 3] [--reps 5]

Prints one JSON line: kernel time (best / median of --reps, events on the stream), decoded GB/s, and the mean
per-frame phase cycles from the instrumented launch (dxa_zstd_decode_prof): Huffman table build, literal streams,
sequence-table builds, sequence loop, with blocks / sequences / literals per frame."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

PHASES = ("total", "huf_table", "literals", "seq_tables", "seq_loop", "blocks", "sequences", "literal_bytes")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--per", type=int, default=26)
    ap.add_argument("--level", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from dxa.io.kafka import zstd_compress
    from dxa.models import iot
    from dxa.ops import native as N
    from dxa.simulate.datagen import generate_cpu
    N.lib()
    buf, offs = generate_cpu(iot.program(), a.events, 1, 0, 1_700_000_000_000, 1000)
    raw = bytes(buf.numpy())
    o = offs.tolist()
    frames, sizes = [], []
    for i in range(0, a.events, a.per):
        chunk = raw[o[i]:o[min(i + a.per, a.events)]]
        frames.append(zstd_compress(chunk, a.level))
        sizes.append(len(chunk))
    nb = len(frames)
    comp_len = np.array([len(f) for f in frames], dtype=np.int32)
    comp_off = np.zeros(nb, dtype=np.int64)
    comp_off[1:] = np.cumsum(comp_len[:-1].astype(np.int64))
    cap = np.array(sizes, dtype=np.int64)
    out_off = np.zeros(nb, dtype=np.int64)
    out_off[1:] = np.cumsum(cap[:-1])
    dev = torch.device("cuda", 0)
    src = torch.zeros(int(comp_len.sum()) + 64, dtype=torch.uint8)
    src[:int(comp_len.sum())] = torch.frombuffer(bytearray(b"".join(frames)), dtype=torch.uint8)
    src = src.to(dev)
    t = {k: torch.from_numpy(v).to(dev) for k, v in (("co", comp_off), ("cl", comp_len), ("oo", out_off),
                                                       ("cap", cap))}
    kind = torch.full((nb,), 4, dtype=torch.uint8, device=dev)
    total = int(cap.sum())
    dst = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    produced = torch.empty(nb, dtype=torch.int64, device=dev)
    status = torch.empty(nb, dtype=torch.int32, device=dev)
    st = N.stream_handle(dev)
    args = [N.ptr(src), N.ptr(t["co"]), N.ptr(t["cl"]), N.ptr(kind), N.ptr(t["oo"]), N.ptr(t["cap"]), nb,
            N.ptr(dst), N.ptr(produced), N.ptr(status)]
    times = []
    for _ in range(a.reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        N.call("dxa_zstd_decode_into", *args, st)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    times = times[1:]
    bad = int((status != 0).sum())
    ok = bad == 0 and bytes(dst[:total].cpu().numpy()) == raw[:total]
    prof = torch.zeros(nb * 8, dtype=torch.int64, device=dev)
    N.call("dxa_zstd_decode_prof", *args, N.ptr(prof), st)
    torch.cuda.synchronize()
    pm = prof.view(nb, 8).double().mean(0).tolist()
    print(json.dumps({"frames": nb, "events": a.events, "per": a.per, "level": a.level, "ratio":
                      round(total / int(comp_len.sum()), 3), "ok": ok, "bad_frames": bad,
                      "best_ms": round(min(times), 3), "median_ms": round(sorted(times)[len(times) // 2], 3),
                      "gbps": round(total / min(times) / 1e6, 1),
                      "per_frame": {k: round(v, 1) for k, v in zip(PHASES, pm)}}))


if __name__ == "__main__":
    main()
