#!/usr/bin/env python3
"""Flagship benchmark: SimulatedData IoT stream → JSON parse → projection → SQL group-by aggregate + alert view →
outputs, one micro-batch per step, one process per MI355X (BASELINE.json config 2; metric "events/sec (node) +
p99 latency").

Each step is a complete micro-batch exactly as the streaming host runs it: the batch's raw JSON bytes are copied from
pinned host memory into HBM (the ingest boundary — events arrive from the network into host memory), parsed
(32 leaf columns), projected (``stringToTimestamp`` + ``Raw.*``), aggregated by (deviceId, deviceType, homeId) with 9
aggregates, filtered into an alert view, both outputs serialised to JSON lines, and the batch metrics emitted.
With N>1 ranks the group-by is two-phase: rank-local partial aggregates are exchanged by key hash over RCCL
all-to-all and merged by the owning rank (weak scaling: events per GPU per step are fixed).

    python bench.py                       # 1 GPU, defaults
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--events-per-batch", type=int, default=2_000_000, help="events per GPU per micro-batch")
    ap.add_argument("--pool", type=int, default=3, help="distinct pre-generated batches cycled through")
    ap.add_argument("--source", choices=["pinned", "device"], default="pinned",
                    help="pinned: H2D copy of raw bytes every step (default); device: NIC-direct style, bytes already"
                         " in HBM")
    ap.add_argument("--profile-stages", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")

    from dxa.ops import native
    if device.type == "cuda":
        native.lib()
    from dxa.engine.processor import Processor, RawBatch
    from dxa.models import iot
    from dxa.simulate.datagen import generate
    from dxa import parallel

    if world > 1:
        parallel.init(dist.group.WORLD, device)

    E = args.events_per_batch
    proc = Processor(iot.flow_settings(workdir=f"/tmp/dxa_bench_{rank}"), device)
    prog = iot.program()
    pool = []
    t_gen = time.perf_counter()
    base_ms = int(time.time() * 1000)
    for p in range(args.pool):
        buf, offs = generate(prog, E, device, seed=1000 * rank + p + 1, row0=p * E, base_ms=base_ms)
        if args.source == "pinned" and device.type == "cuda":
            pool.append((buf.cpu().pin_memory(), offs.cpu().pin_memory()))
            del buf, offs
        else:
            pool.append((buf, offs))
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    gen_s = time.perf_counter() - t_gen
    avg_bytes = float(pool[0][1][-1].item()) / E

    copy_stream = torch.cuda.Stream(device) if (device.type == "cuda" and args.source == "pinned") else None
    staged = {}

    def stage(i):
        hb, ho = pool[i % len(pool)]
        if copy_stream is None:
            staged[i] = (hb, ho, None)
            return
        with torch.cuda.stream(copy_stream):
            db = hb.to(device, non_blocking=True)
            do = ho.to(device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(copy_stream)
        staged[i] = (db, do, ev)

    lat = []
    interval_us = 1_000_000

    def step(i):
        db, do, ev = staged.pop(i)
        if ev is not None:
            torch.cuda.current_stream(device).wait_event(ev)
            db.record_stream(torch.cuda.current_stream(device))
            do.record_stream(torch.cuda.current_stream(device))
        stage(i + 1)   # prefetch the next batch's bytes while this one is processed
        bt = int(time.time() * 1e6)
        m = proc.process_batch(RawBatch(db, do, E), bt, interval_us)
        lat.append(m["Latency-Process"])
        return m

    stage(0)
    for i in range(args.warmup):
        step(i)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    lat.clear()
    t0 = time.perf_counter()
    last = None
    for i in range(args.warmup, args.warmup + args.steps):
        last = step(i)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        lt = torch.tensor(sorted(lat), dtype=torch.float64, device=device)
        gathered = [torch.empty_like(lt) for _ in range(world)]
        dist.all_gather(gathered, lt)
        lat = sorted(float(x) for g in gathered for x in g.tolist())
    lat_sorted = sorted(lat)

    def pct(p):
        if not lat_sorted:
            return None
        k = min(len(lat_sorted) - 1, max(0, int(round(p / 100.0 * (len(lat_sorted) - 1)))))
        return lat_sorted[k] * 1000.0

    total_events = E * world * args.steps
    value = total_events / elapsed
    out = {
        "metric": "events/sec (node) + p99 latency, SimulatedData IoT Flow",
        "value": value,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1000.0,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp64/int64 columns (no reduced precision)",
        "data": "synthetic (SimulatedData-schema JSON generated on device, random seeds per rank/batch)",
        "config": {"model": "SimulatedData IoT flow: 32-col JSON parse + projection + GROUP BY (deviceId, deviceType,"
                            " homeId) 9 aggregates + alert view + JSON outputs",
                   "global_batch": E * world, "seq_len": None, "parallelism": f"dp{world}",
                   "events_per_gpu_per_batch": E, "avg_event_bytes": round(avg_bytes, 1), "source": args.source},
        "p50_latency_process_ms": pct(50),
        "p99_latency_process_ms": pct(99),
        "events_per_sec_per_gpu": value / world,
        "vs_target_1M_events_per_sec_per_gpu": value / world / 1e6,
        "output_groups": last.get("Output_DeviceSummary_Sink_InputEvents") if last else None,
        "generation_s": round(gen_s, 3),
    }
    if args.profile_stages:
        out["stage_s"] = {k: round(v, 5) for k, v in proc.stage_times.items()}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
