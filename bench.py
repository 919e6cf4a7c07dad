#!/usr/bin/env python3
"""Flagship benchmark: SimulatedData IoT stream → JSON parse → projection → SQL → outputs, one micro-batch per step,
one process per MI355X (BASELINE.json metric "events/sec (node) + p99 latency").

``--flow`` picks the BASELINE configuration (default ``groupby`` = config 2, the headline):

* ``groupby`` — 32-col JSON parse, projection, GROUP BY (deviceId, deviceType, homeId) with 9 aggregates, alert view,
  JSON outputs (config 2);
* ``window``  — the same aggregate over a 5-minute sliding window with a 1-s slide (config 3; answered from cached
  per-pane partial aggregates, merged across ranks with one RCCL all-to-all of partials);
* ``join``    — stream–static hash join against a 100M-row reference table resident in HBM (config 4);
* ``full``    — codegen'd rules + windowed SQL with a device UDF + reference join + accumulator state (config 5);
* ``passthrough`` — tag rules on every event and every event written as JSON (config 1's shape at full rate).

Each step is a complete micro-batch exactly as the streaming host runs it.  Sources: ``kafka`` (default for
groupby/join/passthrough) — each batch arrives in pinned host memory as a multi-partition Fetch of Kafka v2 record
batches with the LZ4 codec (producer batches of ~16 KiB, compression.lz4.level 9; produced outside the step), and
every step plans the batch headers on the host, copies the compressed bytes into HBM, decompresses and frames the
records on the GPU and parses the values in place — the Kafka / Event Hubs source's own path
(``dxa.io.kafka_device``); ``pinned-lz4`` — one LZ4 frame of newline-delimited JSON, newline-framed on the GPU;
``pinned`` — the raw JSON bytes are copied into HBM every step (≈2.4x more PCIe bytes); ``gpu-sim`` — the SimulatedData generator renders the next batch on the GPU with event
times inside that batch's second (needed by the windowed flows, whose windows must see advancing event time; its
cost is inside the timed step).  Batch times advance one interval per step on a simulated clock.
With N>1 ranks, per-GPU work is fixed (weak scaling); GROUP BYs are two-phase over RCCL.

    python bench.py                                   # 1 GPU, config 2
    python bench.py --flow window                     # config 3 (warms up 305 steps to fill the 5-min window)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

DEFAULT_EVENTS = {"groupby": 2_000_000, "window": 1_000_000, "join": 2_000_000, "full": 1_000_000,
                  "passthrough": 1_000_000}
DEFAULT_WARMUP = {"groupby": 5, "window": 305, "join": 3, "full": 305, "passthrough": 3}
DEFAULT_SOURCE = {"groupby": "kafka", "window": "gpu-sim", "join": "kafka", "full": "gpu-sim",
                  "passthrough": "kafka"}
MODEL = {
    "groupby": "SimulatedData IoT flow: 32-col JSON parse + projection + GROUP BY (deviceId, deviceType, homeId) "
               "9 aggregates + alert view + JSON outputs",
    "window": "SimulatedData IoT flow: 32-col JSON parse + projection + 5-min sliding-window GROUP BY (1-s slide) "
              "9 aggregates + alert view",
    "join": "SimulatedData IoT flow: 32-col JSON parse + stream-static hash join vs {ref}-row HBM-resident "
            "reference table + GROUP BY",
    "full": "SimulatedData IoT flow: rules (ProcessRules codegen) + 5-min windowed SQL with device UDF + "
            "reference join + accumulator state table",
    "passthrough": "SimulatedData IoT flow: tag rules on every event + every tagged event serialised to JSON "
                   "(config 1 shape at full rate)",
}


def _cpu_lines(raw, length):
    """CPU rehearsal of the newline framing (record offsets of '\\n'-terminated events)."""
    import torch
    nl = torch.nonzero(raw[:length] == 10).flatten()
    return torch.cat([torch.zeros(1, dtype=torch.int64), nl + 1])


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """``--gpus N`` without a launcher: start N rank processes of this script (one per GPU, the environment
    ``torch.distributed.run`` would give them) and wait for all of them.  Runs before anything touches the GPU — no
    ``import torch`` in this process — and never execs: the children are subprocesses, rank 0's JSON line reaches
    stdout through the inherited descriptor, and the parent exits non-zero when any rank fails (the survivors are
    stopped then, so a dead rank cannot leave the others blocked in a collective).  The reference scales the same
    way, one partition per executor task (EventHubStreamingFactory.scala:86, StreamingHost.scala:68-69)."""
    import signal
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))

    def forward(sig, _frame):                 # a signal to the launcher (a time limit) reaches every rank
        for q in procs:
            if q.poll() is None:
                q.send_signal(sig)
    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.send_signal(signal.SIGTERM)
        if live:
            time.sleep(0.1)
    return rc


def sim_gen_args(j: int, rank: int, E: int, clock0_us: int, interval_us: int) -> dict:
    """Generator arguments of batch ``j`` for the ``gpu-sim`` source.  The event time of row r is
    base_ms + r * step_us / 1000 and batch j renders rows j*E .. j*E + E-1, so a constant base puts batch j's events
    in the interval before its batch time, [clock0 + j*interval - interval, clock0 + j*interval).  (A base that
    advanced with j as well ran event time at twice the batch clock: a 5-min window then held ~120 of its 300
    panes, profiles/round5/evtime/.)"""
    return dict(seed=7919 * rank + j + 1, row0=j * E, base_ms=(clock0_us - interval_us) // 1000,
                step_us=max(1, interval_us // E))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--flow", choices=list(DEFAULT_EVENTS), default="groupby")
    ap.add_argument("--events-per-batch", type=int, default=None, help="events per GPU per micro-batch")
    ap.add_argument("--ref-rows", type=int, default=100_000_000, help="reference table rows (join flow)")
    ap.add_argument("--pool", type=int, default=3, help="distinct pre-generated batches cycled (pinned source)")
    ap.add_argument("--prefetch", type=int, default=2,
                    help="batches whose ingest (H2D copy + decode, or generation) is in flight ahead of the one "
                         "being processed")
    ap.add_argument("--lz4-chunks", type=int, default=4, help="pinned-lz4: copy/decode pipeline depth per batch")
    ap.add_argument("--lz4-block", type=int, default=None,
                    help="pinned-lz4: LZ4 frame block size (default: dxa.ops.lz4.DEFAULT_BLOCK)")
    ap.add_argument("--lz4-level", type=int, default=9,
                    help="pinned-lz4: producer compression level (Kafka compression.lz4.level; 9 is Kafka's default, "
                         "0 = fast greedy compressor)")
    ap.add_argument("--source", choices=["pinned", "pinned-lz4", "kafka", "device", "gpu-sim"], default=None,
                    help="pinned: H2D copy of raw bytes every step; pinned-lz4: H2D copy of an LZ4 frame of JSON "
                         "lines, decoded + newline-framed on the GPU; kafka: Kafka v2 record batches (LZ4 codec) as "
                         "a multi-partition Fetch returns them, planned on the host, decompressed and record-framed "
                         "on the GPU (the Kafka source's path); device: bytes already in HBM; gpu-sim: GPU "
                         "generator renders each batch")
    ap.add_argument("--kafka-partitions", type=int, default=16, help="kafka: partitions per fetch (planned in "
                    "parallel on the host, as per-partition fetch threads would)")
    ap.add_argument("--kafka-batch-records", type=int, default=26,
                    help="kafka: records per producer batch (26 SimulatedData events = ~16 KiB, one LZ4 block)")
    ap.add_argument("--kafka-batch-size", type=int, default=None, metavar="BYTES",
                    help="kafka: size record batches as a Java producer with batch.size=BYTES does (the estimated "
                         "compressed size fills batch.size; dxa.io.kafka.records_per_batch) instead of a fixed "
                         "--kafka-batch-records")
    ap.add_argument("--kafka-codec", choices=["lz4", "gzip", "snappy", "zstd"], default="lz4",
                    help="kafka: record batch compression codec, decoded on the GPU (lz4.hip; gzip = the Event Hubs "
                         "Kafka endpoint's codec, inflate.hip; snappy = snappy-java's xerial stream, snappy.hip; "
                         "zstd = zstd-jni's frames, zstd.hip)")
    ap.add_argument("--zstd-level", type=int, default=3, help="kafka zstd: producer compression.zstd.level")
    ap.add_argument("--crc", choices=["auto", "host", "device", "off"], default="auto",
                    help="kafka: where record batches' CRC-32C is checked (consumer check.crcs): auto (default: host "
                         "planner threads while the node's host memory budget covers this rank, else the GPU — "
                         "dxa.parallel.affinity.crc_placement), host, the GPU (kafka_crc_kernel), or not at all")
    ap.add_argument("--workdir", default=None,
                    help="keep the run's files (state table, sink output) here, rank r in <dir>_<r>, cleared of state "
                         "at start; default: a fresh temporary directory per rank, removed at the end")
    ap.add_argument("--column-pruning", choices=["on", "off"], default="on",
                    help="datax.job.process.columnpruning: parse and retain only the raw fields statements read")
    ap.add_argument("--sink", choices=["null", "blob"], default="null",
                    help="output sink: null (rendered JSON lands in host memory) or blob (gzip files under /tmp)")
    ap.add_argument("--compute-priority", choices=["high", "normal"], default="normal",
                    help="HIP priority of the stream the batch's statements run on: high lets the critical path's "
                         "short kernels (and the syncs waiting on them) go ahead of the ingest / generator / "
                         "parse-ahead streams, which stay at normal priority and fill the rest of the chip")
    ap.add_argument("--switch-interval-ms", type=float, default=None,
                    help="the interpreter's GIL switch interval (default: Python's 5 ms); the batch thread shares the "
                         "GIL with the output, state-writer and planner threads")
    ap.add_argument("--profile-stages", action="store_true")
    ap.add_argument("--sync-outputs", action="store_true",
                    help="finish each batch's sink writes before the next batch starts (default: pipelined)")
    ap.add_argument("--torch-profile", default=None, metavar="PATH",
                    help="run the timed steps under torch.profiler and write op/stage tables to PATH")
    args = ap.parse_args()
    flow = args.flow
    warmup = DEFAULT_WARMUP[flow] if args.warmup is None else args.warmup
    E = args.events_per_batch or DEFAULT_EVENTS[flow]
    source = args.source or DEFAULT_SOURCE[flow]
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            sys.exit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} from the launcher but --gpus {args.gpus}")
    elif args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # NUMA placement first, from sysfs alone: threads the HIP runtime and RCCL start later inherit the mask, and the
    # pinned staging buffers are first-touched on the GPU's socket
    from dxa.parallel.affinity import bind_to_device
    ndev = torch.cuda.device_count()
    # DXA_DIST_BACKEND=gloo: rehearsal of the multi-rank path with several ranks sharing a GPU (collectives staged
    # through host memory); the default on GPUs is RCCL with one rank per GPU
    backend = os.environ.get("DXA_DIST_BACKEND") or ("nccl" if ndev else "gloo")
    dev_index = local % ndev if (ndev and backend == "gloo") else local
    numa_cpus = bind_to_device(dev_index) if ndev > dev_index else None
    # host worker threads (producer-side compression before the timed region, Kafka batch planning inside it): this
    # rank's share of the CPUs its socket's ranks are bound to — 16 on a 1-GPU run
    from dxa.parallel.affinity import crc_placement, host_threads
    host_thr = host_threads(dev_index, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    if args.crc == "auto":
        args.crc = crc_placement(local, int(os.environ.get("LOCAL_WORLD_SIZE", "1")), host_thr)
    device = torch.device("cuda", dev_index) if torch.cuda.is_available() else torch.device("cpu")
    if world > 1:
        if device.type == "cuda":
            torch.cuda.set_device(dev_index)
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=device)      # RCCL over xGMI
            else:
                dist.init_process_group("gloo")
        else:
            dist.init_process_group("gloo")                              # CPU rehearsal of the same code path
    on_gpu = device.type == "cuda"
    if on_gpu and args.compute_priority == "high":
        # the batch's own kernels (parse result assembly, projection, statements, the syncs that wait on them) on a
        # high-priority stream; every helper stream created later (ingest copies, generator, parse-ahead, output
        # rendering) is a normal one
        torch.cuda.set_stream(torch.cuda.Stream(device, priority=-1))
    if os.environ.get("DXA_BENCH_FAIL_RANK") == str(rank):        # fault injection (tests): this rank dies
        raise SystemExit(f"bench.py: rank {rank} failing on request (DXA_BENCH_FAIL_RANK)")

    from dxa.ops import native
    if on_gpu:
        native.lib()
    from dxa.engine.processor import Processor, RawBatch
    from dxa.models import iot
    from dxa.simulate.datagen import generate, generate_begin, generate_finish
    from dxa import parallel

    if world > 1:
        parallel.init(dist.group.WORLD, device)

    # passthrough is bound by the D2H of its rendered JSON: two batches' outputs in flight overlap one batch's copy
    # with the next one's rendering (profiles/round4/output_depth/: 64.5 -> 71.8 M ev/s); the other flows keep one
    # (no gain measured, lower latency).  DXA_OUTPUT_DEPTH overrides.
    depth_extra = {"datax.job.process.outputdepth": "2"} if flow == "passthrough" else {}
    depth_extra["datax.job.process.columnpruning"] = "true" if args.column_pruning == "on" else "false"
    # a fresh work directory per run and rank: every run starts from an empty accumulator (a state table left by an
    # earlier run would be reloaded and change the first batches' work, making back-to-back A/B runs
    # order-dependent), and concurrent runs never share state or output files
    import shutil
    import tempfile
    if args.workdir:
        workdir = f"{args.workdir}_{rank}"
        shutil.rmtree(os.path.join(workdir, "state"), ignore_errors=True)
    else:
        workdir = tempfile.mkdtemp(prefix=f"dxa_bench_{flow}_r{rank}_", dir="/tmp")
    settings = iot.flow_settings(workdir=workdir, variant=flow, sink=args.sink,
                                 ref_rows=args.ref_rows, extra=depth_extra)
    ref_write_s = None
    if flow == "join":
        # config 4's reference table is a real CSV read through datax.job.input.default.referencedata.* (rank 0
        # reads it, one RCCL broadcast of the bytes, device tokenizer); the file is written once, untimed
        ref_csv = settings.get("datax.job.input.default.referencedata.RefDevices.path")
        if rank == 0 and not os.path.exists(ref_csv):
            t_w = time.perf_counter()
            tmp = ref_csv + f".tmp{os.getpid()}"
            iot.write_reference_csv(tmp, args.ref_rows, device)
            os.replace(tmp, ref_csv)
            ref_write_s = round(time.perf_counter() - t_w, 3)
        if world > 1:
            dist.barrier()
    t_ref = time.perf_counter()
    proc = Processor(settings, device, pipeline_outputs=not args.sync_outputs)
    if on_gpu:
        torch.cuda.synchronize(device)
    ref_s = time.perf_counter() - t_ref
    prog = iot.program()
    interval_us = 1_000_000
    clock0_us = (int(time.time()) - 3600) * 1_000_000      # simulated clock, aligned to the interval

    def batch_time(i):
        return clock0_us + i * interval_us

    t_gen = time.perf_counter()
    pool = []
    comp_bytes = []
    import numpy as np
    from dxa.ops import lz4
    lz4_block_k = args.lz4_block or lz4.DEFAULT_BLOCK
    if source == "pinned-lz4":
        from dxa.ops import lz4
        from dxa.ops.jsonparse import frame_lines_gpu
        prog_nl = iot.program(newline=True)
        lz4_block = args.lz4_block or lz4.DEFAULT_BLOCK
        base_ms = clock0_us // 1000
        for p in range(args.pool):
            buf, offs = generate(prog_nl, E, device, seed=1000 * rank + p + 1, row0=p * E, base_ms=base_ms)
            total = int(offs[-1])
            frame = lz4.compress_frame(buf[:total].cpu(), lz4_block, threads=host_thr, level=args.lz4_level)
            del buf, offs
            comp_bytes.append(frame.size)
            pool.append(lz4.DeviceFrame.from_frame(frame, lz4_block, pin=on_gpu))
    kafka_parts, kafka_json = [], []
    if source == "kafka":
        from dxa.io import kafka as K
        parts = max(1, args.kafka_partitions)
        for p in range(args.pool):
            buf, offs = generate(prog, E, device, seed=1000 * rank + p + 1, row0=p * E, base_ms=clock0_us // 1000)
            hb, ho = buf.cpu().numpy(), offs.cpu().numpy()
            del buf, offs
            cuts = np.linspace(0, E, parts + 1).astype(np.int64)
            if args.kafka_batch_size and p == 0:
                # batch.size semantics of the Java producer: records per batch from the learned compression ratio
                args.kafka_batch_records, _r = K.records_per_batch(
                    hb, ho, args.kafka_batch_size, compression=args.kafka_codec,
                    level=args.zstd_level if args.kafka_codec == "zstd" else args.lz4_level, block_size=lz4_block_k)
            clevel = args.zstd_level if args.kafka_codec == "zstd" else args.lz4_level
            sets = [K.encode_stream(hb, ho[cuts[q]:cuts[q + 1] + 1], args.kafka_batch_records, base_offset=0,
                                    compression=args.kafka_codec, level=clevel, block_size=lz4_block_k,
                                    threads=host_thr) for q in range(parts)]
            total = sum(x.size for x in sets)
            staging = torch.empty(total + 64, dtype=torch.uint8, pin_memory=on_gpu)
            sn = staging.numpy()
            bounds, pos = [], 0
            for x in sets:
                sn[pos:pos + x.size] = x
                bounds.append((pos, pos + x.size))
                pos += x.size
            comp_bytes.append(total)
            pool.append(staging)
            kafka_parts.append(bounds)
            kafka_json.append(int(ho[-1]))
    if source in ("pinned", "device"):
        base_ms = clock0_us // 1000
        for p in range(args.pool):
            buf, offs = generate(prog, E, device, seed=1000 * rank + p + 1, row0=p * E, base_ms=base_ms)
            if source == "pinned" and on_gpu:
                pool.append((buf.cpu().pin_memory(), offs.cpu().pin_memory()))
                del buf, offs
            else:
                pool.append((buf, offs))
    if on_gpu:
        torch.cuda.synchronize(device)
    gen_s = time.perf_counter() - t_gen

    # this box's own pinned H2D bandwidth, measured once before the timed region on a copy of the size one step
    # ingests (best of 3): the record then says whether a step was bound by the link or by the code
    # (pcie_fraction = ingest bytes per step / (h2d_gb_s * step time))
    h2d_gb_s = None
    if on_gpu and comp_bytes:
        kmax = max(range(len(comp_bytes)), key=comp_bytes.__getitem__)
        nb = comp_bytes[kmax]
        hsrc = pool[kmax] if isinstance(pool[kmax], torch.Tensor) else torch.empty(nb, dtype=torch.uint8,
                                                                                   pin_memory=True)
        hsrc = hsrc[:nb]
        ddst = torch.empty(nb, dtype=torch.uint8, device=device)
        best = None
        for _ in range(3):
            torch.cuda.synchronize(device)
            t_c = time.perf_counter()
            ddst.copy_(hsrc, non_blocking=True)
            torch.cuda.synchronize(device)
            dt = time.perf_counter() - t_c
            best = dt if best is None else min(best, dt)
        h2d_gb_s = nb / best / 1e9
        del ddst

    side = torch.cuda.Stream(device) if (on_gpu and source in ("pinned", "pinned-lz4", "kafka", "gpu-sim")) else None
    ingest = lz4.ChunkedIngest(device, chunks=args.lz4_chunks, copy_stream=side) \
        if (on_gpu and source == "pinned-lz4") else None
    kdec = None
    plan_threads = None
    if source == "kafka":
        from dxa.io import kafka_device as KD
        from concurrent.futures import ThreadPoolExecutor
        plan_bufs = KD.PlanBufferPool()
        plan_threads = host_thr
        planner = ThreadPoolExecutor(max_workers=1)
        plan_futs = {}

        def make_plan(i):
            b = kafka_parts[i % len(pool)]
            return KD.plan_many(pool[i % len(pool)].numpy(), b, [0] * len(b), threads=plan_threads,
                                buffer=plan_bufs.get(),
                                verify_crc=args.crc == "host")
        if on_gpu:
            kdec = KD.DeviceRecordDecoder(device, chunks=args.lz4_chunks, copy_stream=side,
                                          verify_crc=args.crc == "device")
    staged = {}
    gen_pending = {}           # gpu-sim: batches whose length pass is queued (datagen.generate_begin)
    sizes = []
    framing_checks = []        # device flags: a frame's newline count differed from its producer's record count

    def stage(i):
        """Make batch i's raw bytes available in HBM — on a side stream, overlapping batch i-1's processing."""
        arrival[i] = time.perf_counter()
        if source == "kafka":
            staging, bounds = pool[i % len(pool)], kafka_parts[i % len(pool)]
            sn = staging.numpy()
            # per-partition plans (headers only), walked in parallel native threads as per-partition fetch threads
            # would, one batch ahead on a planner thread (the native walk releases the GIL); the merged tables
            # land in a pinned buffer for one H2D copy
            fut = plan_futs.pop(i, None) or planner.submit(make_plan, i)
            plan_futs[i + 1] = planner.submit(make_plan, i + 1)
            plan = fut.result()
            if kdec is not None:
                raw, ev = kdec.decode(staging, plan)
            else:
                out, st, en = KD.decode_on_host_like(sn, plan)
                plan.buffer.release()
                raw, ev = RawBatch(torch.from_numpy(out), torch.from_numpy(np.append(st, plan.out_bytes)),
                                   plan.nrec, ends=torch.from_numpy(en)), None
            staged[i] = (raw, None, ev)
            return
        if source == "gpu-sim":
            def gen_args(j):
                return sim_gen_args(j, rank, E, clock0_us, interval_us)
            if side is None:
                staged[i] = generate(prog, E, device, **gen_args(i)) + (None,)
                return
            with torch.cuda.stream(side):
                # batch i's length pass was queued one stage earlier, so its size is already known here; queue
                # batch i+1's now (the host never waits on a length pass stuck behind the compute stream's kernels)
                pend = gen_pending.pop(i, None) or generate_begin(prog, E, device, **gen_args(i))
                gen_pending[i + 1] = generate_begin(prog, E, device, **gen_args(i + 1))
                db, do = generate_finish(pend)
                ev = torch.cuda.Event()
                ev.record(side)
            staged[i] = (db, do, ev)
            return
        if source == "pinned-lz4":
            fr = pool[i % len(pool)]
            if side is None:
                raw = lz4.decompress_device(fr)
                offs = (frame_lines_gpu(raw, fr.content_size, expected=E, mismatches=framing_checks) if on_gpu
                        else _cpu_lines(raw, fr.content_size))
                staged[i] = (raw, offs, None)
                return
            # chunked: chunk k's H2D copy overlaps chunk k-1's decode (copy and decode streams)
            raw, _ = ingest.stage(fr)
            ds = ingest.decode_stream
            with torch.cuda.stream(ds):
                offs = frame_lines_gpu(raw, fr.content_size, expected=E, mismatches=framing_checks)
                ev = torch.cuda.Event()
                ev.record(ds)
            staged[i] = (raw, offs, ev)
            return
        hb, ho = pool[i % len(pool)]
        if side is None:
            staged[i] = (hb, ho, None)
            return
        with torch.cuda.stream(side):
            db = hb.to(device, non_blocking=True)
            do = ho.to(device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(side)
        staged[i] = (db, do, ev)

    lat = []
    # Latency-Batch (CommonProcessorFactory.scala:373: completion wall time − batch time).  The bench runs the stream
    # saturated, so a batch's time is the wall-clock moment it closes and starts arriving — when stage(i) begins its
    # ingest (``prefetch`` steps before it is processed) — and it completes when its last sink write finishes.  (The
    # simulated clock passed to process_batch only drives event times / windows.)
    arrival = {}
    lat_batch = []

    def on_complete(bt, m):
        lat.append(m["Latency-Process"])
        i = (bt - clock0_us) // interval_us
        t_arr = arrival.pop(i, None)
        if t_arr is not None:
            lat_batch.append(proc.last_done_perf - t_arr)
    host_trace = [] if os.environ.get("DXA_BENCH_HOST_TRACE") else None
    host_sections_trace = []     # DXA_BENCH_HOST_TRACE: per step, the host sections' ms (DXA_HOST_TIMERS=1 for more)
    proc.on_batch_complete = on_complete

    ready = {}
    parse_ahead = on_gpu
    # parse-ahead on its own stream, queued BEFORE the previous batch's process_batch so the parse overlaps that
    # batch's query kernels — for the device-resident source, where the parse is on the critical path.  With a
    # PCIe-bound ingest (kafka / pinned sources) it measured no throughput gain and higher latency
    # (profiles/round4/parse_stream/: passthrough 64 -> 61 M ev/s, join p50 8.9 -> 13.7 ms), so there the parse is
    # queued behind the batch's kernels after process_batch.
    parse_stream = torch.cuda.Stream(device) if parse_ahead and source == "gpu-sim" else None

    def take(i):
        db, do, ev = staged.pop(i)
        rb = db if isinstance(db, RawBatch) else RawBatch(db, do, E)
        if ev is not None:
            cur = torch.cuda.current_stream(device)
            cur.wait_event(ev)
            for t in (rb.buf, rb.offs, rb.ends):
                if t is not None:
                    t.record_stream(cur)
        return rb

    def take_to(i, stream):
        """Batch i for a parse on ``stream``: ordered after its ingest there; its bytes are also read later on the
        compute stream (string columns view them), so both streams hold them."""
        db, do, ev = staged.pop(i)
        rb = db if isinstance(db, RawBatch) else RawBatch(db, do, E)
        if ev is not None:
            stream.wait_event(ev)
        cur = torch.cuda.current_stream(device)
        for t in (rb.buf, rb.offs, rb.ends):
            if t is not None:
                t.record_stream(stream)
                t.record_stream(cur)
        return rb

    def step(i):
        rb = ready.pop(i, None) or take(i)
        t_s = time.perf_counter()
        stage(i + depth)
        t_p = time.perf_counter()
        # parse-ahead (Processor.prepare).  Never across the warm-up → timed boundary or past the last timed batch,
        # so every timed batch parses inside the timed region
        ahead = parse_ahead and i + 1 in staged and i + 1 != warmup and i + 1 < warmup + args.steps
        if ahead and parse_stream is not None:
            ready[i + 1] = proc.prepare(take_to(i + 1, parse_stream), stream=parse_stream)
        m = proc.process_batch(rb, batch_time(i), interval_us)
        if ahead and parse_stream is None:          # behind batch i's kernels on the compute stream
            ready[i + 1] = proc.prepare(take(i + 1))
        if host_trace is not None:
            host_trace.append((i, round((t_p - t_s) * 1e3, 2), round((time.perf_counter() - t_p) * 1e3, 2)))
            acc = dict(getattr(proc, "host_acc", {}))
            from dxa.telemetry import tracing as _trs
            acc.update(_trs.HOST_ACC)
            prev = host_sections_trace[-1][1] if host_sections_trace else {}
            host_sections_trace.append((i, {k: v for k, v in acc.items()}))
            host_sections_trace[-1] = (i, acc, {k: round((v - prev.get(k, 0.0)) * 1e3, 3) for k, v in acc.items()
                                                if v - prev.get(k, 0.0) > 5e-5})
        sizes.append(kafka_json[i % len(pool)] + 16 if source == "kafka" else rb.buf.shape[0])
        return m

    from dxa.utils import settle_gc
    settle_gc()
    if args.switch_interval_ms is not None:
        sys.setswitchinterval(args.switch_interval_ms / 1e3)
    depth = max(1, args.prefetch)
    for i in range(depth):
        stage(i)
    for i in range(warmup):
        step(i)
    proc.drain()
    if on_gpu:
        torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    lat.clear()
    lat_batch.clear()
    sizes.clear()
    prof = None
    if args.torch_profile:
        from dxa.telemetry import tracing
        tracing.enable_profiler_ranges()
        acts = [torch.profiler.ProfilerActivity.CPU] + ([torch.profiler.ProfilerActivity.CUDA] if on_gpu else [])
        prof = torch.profiler.profile(activities=acts)
        prof.__enter__()
    cprof = None
    if os.environ.get("DXA_BENCH_CPROFILE"):            # host profile of the timed steps (diagnostics only)
        import cProfile
        cprof = cProfile.Profile()
        cprof.enable()
    from dxa.ops import serialize as _ser0
    ser_stats0 = dict(_ser0.STATS)
    host0 = dict(getattr(proc, "host_acc", {}))
    from dxa.engine import processor as _pm
    out_cpu0 = _pm.OUTPUT_CPU[0]
    from dxa.telemetry import tracing as _tr
    _tr.time_host_syncs()
    sec0 = dict(_tr.HOST_ACC)
    t0 = time.perf_counter()
    last = None
    for i in range(warmup, warmup + args.steps):
        step(i)
    last = proc.drain() or proc.last_metrics           # the last batch's outputs complete inside the timed region
    if on_gpu:
        torch.cuda.synchronize(device)
    if cprof is not None:
        cprof.disable()
        cprof.dump_stats(os.environ["DXA_BENCH_CPROFILE"])
    if prof is not None:
        prof.__exit__(None, None, None)
        ka = prof.key_averages()
        with open(args.torch_profile, "w") as f:
            f.write(f"# {flow}: {args.steps} steps (profiled run; timings include profiler overhead)\n")
            f.write(ka.table(sort_by="cuda_time_total" if on_gpu else "cpu_time_total", row_limit=60,
                             max_name_column_width=60))
            f.write("\n# by self CPU time\n")
            f.write(ka.table(sort_by="self_cpu_time_total", row_limit=40, max_name_column_width=60))
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        cdev = device if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        def gather_all(xs):
            lt = torch.tensor(sorted(xs), dtype=torch.float64, device=cdev)
            gathered = [torch.empty_like(lt) for _ in range(world)]
            dist.all_gather(gathered, lt)
            return sorted(float(x) for g in gathered for x in g.tolist())
        lat = gather_all(lat)
        lat_batch = gather_all(lat_batch) if len(lat_batch) == args.steps else lat_batch
    lat_sorted = sorted(lat)
    latb_sorted = sorted(lat_batch)
    if framing_checks:
        from dxa.ops.jsonparse import check_framing
        check_framing(framing_checks)                      # after the timed region: one host sync
    if kdec is not None:
        kdec.check()                                       # every record batch decoded (one host sync)

    def pct(p, xs=None):
        xs = lat_sorted if xs is None else xs
        if not xs:
            return None
        k = min(len(xs) - 1, max(0, int(round(p / 100.0 * (len(xs) - 1)))))
        return xs[k] * 1000.0

    total_events = E * world * args.steps
    value = total_events / elapsed
    avg_bytes = (sum(sizes) / len(sizes) - 16) / E if sizes else None
    out = {
        "metric": "events/sec (node) + p99 latency, SimulatedData IoT Flow",
        "value": value,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": warmup,
        "ms_per_step": elapsed / args.steps * 1000.0,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp64/int64 columns (no reduced precision)",
        "data": "synthetic (SimulatedData-schema JSON generated on device, random seeds per rank/batch"
                + ("; delivered as LZ4-framed batches in pinned host memory, decompressed on the GPU in every step)"
                   if source == "pinned-lz4" else
                   f"; delivered as Kafka v2 record batches with the {args.kafka_codec.upper()} codec in pinned host memory (a "
                   "multi-partition Fetch), planned on the host, "
                   + ({"host": "CRC-32C-verified on the host (check.crcs), ",
                       "device": "CRC-32C-verified on the GPU (check.crcs), "}.get(args.crc, "")) +
                   "decompressed and record-framed on the GPU in every step)" if source == "kafka" else ")"),
        "config": {"model": MODEL[flow].format(ref=args.ref_rows), "flow": flow,
                   "global_batch": E * world, "seq_len": None, "parallelism": f"dp{world}",
                   "events_per_gpu_per_batch": E, "avg_event_bytes": round(avg_bytes, 1) if avg_bytes else None,
                   "source": source, "ingest_prefetch_batches": depth, "batch_interval_s": interval_us / 1e6,
                   "outputs": "sync" if args.sync_outputs else (
                       "pipelined (batch t sinks overlap batch t+1)" if proc.output_depth == 1 else
                       f"pipelined, {proc.output_depth} batches' outputs in flight"),
                   "sink": args.sink, "compute_stream_priority": args.compute_priority,
                   "gil_switch_interval_ms": round(sys.getswitchinterval() * 1e3, 3)},
        "p50_latency_process_ms": pct(50),
        "p99_latency_process_ms": pct(99),
        "p50_latency_batch_ms": pct(50, latb_sorted),
        "p99_latency_batch_ms": pct(99, latb_sorted),
        "events_per_sec_per_gpu": value / world,
        "vs_target_1M_events_per_sec_per_gpu": value / world / 1e6,
        "generation_s": round(gen_s, 3),
        "host_cpus_bound": None if numa_cpus is None else len(numa_cpus),
        "host_plan_threads": plan_threads,
    }
    if comp_bytes:
        out["config"]["ingest_bytes_per_event"] = round(sum(comp_bytes) / len(comp_bytes) / E, 1)
        out["config"]["compression_ratio"] = round((sum(sizes) / len(sizes) - 16) / (sum(comp_bytes) / len(comp_bytes)),
                                                   2)
        out["config"]["lz4_level"] = args.lz4_level
        out["config"]["lz4_block_bytes"] = lz4_block_k
        if h2d_gb_s:
            step_bytes = sum(comp_bytes) / len(comp_bytes)
            out["h2d_gb_s"] = round(h2d_gb_s, 2)
            out["ingest_mb_per_step"] = round(step_bytes / 1e6, 1)
            out["pcie_fraction"] = round(step_bytes / (h2d_gb_s * 1e9 * elapsed / args.steps), 3)
    if source == "kafka":
        out["config"]["kafka_partitions"] = args.kafka_partitions
        out["config"]["kafka_batch_records"] = args.kafka_batch_records
        if args.kafka_batch_size:
            out["config"]["kafka_batch_size"] = args.kafka_batch_size
        out["config"]["check_crcs"] = args.crc
        out["config"]["kafka_codec"] = args.kafka_codec
        if args.kafka_codec == "zstd":
            out["config"]["zstd_level"] = args.zstd_level
    if host_trace is not None:
        out["host_trace_ms"] = host_trace[-8:]           # (batch, stage() host ms, process_batch() host ms)
        out["host_sections_trace_ms"] = [(i, d) for i, _, d in host_sections_trace[-4:]]
        out["latency_trace_ms"] = [round(x * 1e3, 2) for x in lat]
    if last:
        out["last_batch_outputs"] = {k: v for k, v in last.items() if k.startswith("Output_")}
    if flow == "join":
        st = proc.reference_stats.get("RefDevices", {})
        out["reference_build_s"] = round(ref_s, 3)           # processor start incl. the CSV load
        out["reference_load"] = {"rows": st.get("rows"), "bytes": st.get("bytes"),
                                 "read_s": round(st.get("read_s", 0.0), 3), "load_s": round(st.get("total_s", 0.0), 3),
                                 "gb_per_s": round(st["bytes"] / st["total_s"] / 1e9, 2) if st.get("total_s") else None,
                                 "csv_written_s": ref_write_s,
                                 "host_staged_on_this_rank": st.get("host_staged"),
                                 "path": "referencedata CSV: rank-0 read + broadcast, device line framing + tokenizer "
                                         "(csv.hip), schema cast on device"}
    if flow in ("window", "full") and proc.window_store is not None:
        out["window_panes"] = len(proc.window_store.past)
        out["window_retained_rows"] = proc.window_store.retained_rows()
    if on_gpu:
        from dxa.ops import serialize as _ser
        rs = {k: v - ser_stats0.get(k, 0) for k, v in _ser.STATS.items()}
        if rs["d2h_bytes"]:
            # rendered output text crossing PCIe (sinks' D2H), per timed step; d2h_s is the copies' wall time
            out["output_d2h"] = {"mb_per_step": round(rs["d2h_bytes"] / args.steps / 1e6, 1),
                                 "ms_per_step": round(rs["d2h_s"] / args.steps * 1e3, 2),
                                 "gb_per_s": round(rs["d2h_bytes"] / rs["d2h_s"] / 1e9, 2) if rs["d2h_s"] else None,
                                 "render_launch_pairs_per_step": round(rs["launch_pairs"] / args.steps, 2)}
        out["max_hbm_allocated_gb"] = round(torch.cuda.max_memory_allocated(device) / 2**30, 2)
    if args.profile_stages:
        out["stage_s"] = {k: round(v, 5) for k, v in proc.stage_times.items()}
        out["host_ms_per_step"] = {k: round((v - host0.get(k, 0.0)) / args.steps * 1e3, 3)
                                   for k, v in getattr(proc, "host_acc", {}).items()}
        from dxa.engine import processor as _pm
        out["host_ms_per_step"]["outputs:thread_cpu"] = round((_pm.OUTPUT_CPU[0] - out_cpu0) / args.steps * 1e3, 3)
        if _tr.HOST_ACC:
            out["host_sections_ms_per_step"] = {k: round((v - sec0.get(k, 0.0)) / args.steps * 1e3, 3)
                                                for k, v in sorted(_tr.HOST_ACC.items())}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if not args.workdir:
        shutil.rmtree(workdir, ignore_errors=True)


if __name__ == "__main__":
    main()
