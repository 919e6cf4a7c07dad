"""Can one host feed 8 ranks?  Kafka batch planning with host CRC-32C (``check.crcs=host``) in K concurrent rank
processes, each bound as ``bind_to_device`` binds a rank and planning its own pinned Fetch of LZ4 record batches
(the groupby bench's 2 M-event batch: ~441 MB) in a loop, as the bench's planner thread does one batch ahead.

    python tools/host8_bench.py --ranks 8 --threads 2 --seconds 8       # 8 ranks x 2 planner threads
    python tools/host8_bench.py --ranks 1 --threads 1,2,4,8,16           # one rank's thread scaling

Each rank prints its planned GB/s; the parent prints one JSON line per configuration with the aggregate, the
per-thread rate and the ratio to what K PCIe-bound ranks ingest (K x ``--need-gbs``, default 57 GB/s, the measured
MI355X pinned H2D rate).  The records are generated on the GPU (one process per rank, within the box's process
limit) and copied to pinned host memory before any timing."""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main(rank: int, ranks: int, threads: int, seconds: float, events: int, out: str):
    import numpy as np
    import torch
    from dxa.parallel.affinity import bind_to_device
    cpus = bind_to_device(0)
    from dxa.io import kafka as K
    from dxa.io import kafka_device as KD
    from dxa.models import iot
    from dxa.simulate.datagen import generate
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    buf, offs = generate(iot.program(), events, dev, seed=1000 * rank + 1, row0=0, base_ms=1_700_000_000_000)
    hb, ho = buf.cpu().numpy(), offs.cpu().numpy()
    del buf, offs
    parts = 16
    cuts = np.linspace(0, events, parts + 1).astype(np.int64)
    sets = [K.encode_stream(hb, ho[cuts[q]:cuts[q + 1] + 1], 26, base_offset=0, compression="lz4", level=9,
                            block_size=16384, threads=threads) for q in range(parts)]
    total = sum(x.size for x in sets)
    staging = torch.empty(total + 64, dtype=torch.uint8, pin_memory=dev.type == "cuda").numpy()
    bounds, pos = [], 0
    for x in sets:
        staging[pos:pos + x.size] = x
        bounds.append((pos, pos + x.size))
        pos += x.size
    pool = KD.PlanBufferPool()
    # start together: every rank waits for the parent's go file
    go = out + ".go"
    open(out + ".ready", "w").close()
    while not os.path.exists(go):
        time.sleep(0.01)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        plan = KD.plan_many(staging, bounds, [0] * len(bounds), threads=threads, buffer=pool.get(), verify_crc=True)
        plan.buffer.release()
        n += 1
    dt = time.perf_counter() - t0
    with open(out, "w") as f:
        json.dump({"rank": rank, "plans": n, "seconds": dt, "bytes": total, "gb_s": n * total / dt / 1e9,
                   "cpus_bound": None if cpus is None else len(cpus)}, f)


def run(ranks: int, threads: int, seconds: float, events: int, need: float) -> dict:
    import tempfile
    d = tempfile.mkdtemp(prefix="host8_")
    procs = []
    for r in range(ranks):
        out = os.path.join(d, f"r{r}.json")
        procs.append((out, subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", str(r),
                                             "--ranks", str(ranks), "--threads", str(threads), "--seconds",
                                             str(seconds), "--events", str(events), "--out", out])))
    deadline = time.time() + 600
    while not all(os.path.exists(o + ".ready") for o, _ in procs):
        if time.time() > deadline or any(p.poll() not in (None, 0) for _, p in procs):
            for _, p in procs:
                p.kill()
            raise SystemExit("host8_bench: a rank failed before planning")
        time.sleep(0.05)
    for o, _ in procs:
        open(o + ".go", "w").close()
    rc = [p.wait() for _, p in procs]
    if any(rc):
        raise SystemExit(f"host8_bench: rank exit codes {rc}")
    res = [json.load(open(o)) for o, _ in procs]
    agg = sum(x["gb_s"] for x in res)
    return {"ranks": ranks, "threads_per_rank": threads, "seconds": seconds, "batch_mb": round(res[0]["bytes"] / 1e6, 1),
            "per_rank_gb_s": [round(x["gb_s"], 2) for x in res], "aggregate_gb_s": round(agg, 2),
            "per_thread_gb_s": round(agg / (ranks * threads), 2),
            "need_gb_s": round(need * ranks, 1), "fraction_of_need": round(agg / (need * ranks), 3),
            "cpus_bound": res[0]["cpus_bound"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--threads", default="2")
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--events", type=int, default=2_000_000)
    ap.add_argument("--need-gbs", type=float, default=57.0)
    ap.add_argument("--child", type=int, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.child is not None:
        rank_main(a.child, a.ranks, int(a.threads), a.seconds, a.events, a.out)
        return
    for t in [int(x) for x in a.threads.split(",")]:
        print(json.dumps(run(a.ranks, t, a.seconds, a.events, a.need_gbs)), flush=True)


if __name__ == "__main__":
    main()
