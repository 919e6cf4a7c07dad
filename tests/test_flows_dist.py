"""Multi-rank correctness gate for the five benchmark flows (bench.py --flow …, BASELINE configs 1-5).

The same SimulatedData batches run through the Processor once on one rank and once split over two gloo ranks (each
rank holds every other event, as two source partitions would).  Batch by batch, the union of the two ranks' sink
rows must equal the one-rank run's rows (exact for strings / integers / timestamps, 1e-9 relative for floating
aggregates whose summation order differs), the union of the ranks' accumulator parts must equal the one-rank state,
and the job-wide batch metrics rank 0 emits (all-reduced) must equal the one-rank metrics.  The reference has no
distributed tests: Spark's exchanges are trusted; here the RCCL exchanges are ours, so this is the gate.

Also: the batch-metric reduction across ranks whose sources attach different metrics (a blob-pointer rank with an
empty batch next to one with file times) — keys zero-filled, ``Latency-Blobs`` maxed, not summed
(CommonProcessorFactory.scala:573-576) — and the loud failure when ranks' metric keys still differ."""
import json
import math
import os
import socket
import traceback

import pytest
import torch
import torch.multiprocessing as mp

from dxa.models import iot

N_EVENTS = 1500
N_BATCHES = 6
INTERVAL_US = 1_000_000
REF_ROWS = 5000


def _settings(variant, workdir, shared):
    extra = {"datax.job.process.pipelineoutputs": "false"}
    if variant == "join":
        extra["datax.job.input.default.referencedata.RefDevices.path"] = os.path.join(shared, "ref.csv")
    if variant == "full":          # one accumulator location for all ranks (per-rank part files)
        extra["datax.job.process.statetable.DeviceState.location"] = os.path.join(shared, "state", "DeviceState")
    if variant in ("window", "full"):
        # the flows' 5-minute window shortened to 3 s so a few batches fill it (view name unchanged)
        extra["datax.job.process.timewindow.DataXProcessedInput_5minutes.windowduration"] = "3 seconds"
    return iot.flow_settings(workdir=workdir, variant=variant, sink="memory", extra=extra, ref_rows=REF_ROWS)


def _batches(clock0_us):
    from dxa.simulate.datagen import generate
    prog = iot.program()
    out = []
    for i in range(N_BATCHES):
        bt = clock0_us + i * INTERVAL_US
        buf, offs = generate(prog, N_EVENTS, "cpu", seed=7919 + i, row0=i * N_EVENTS, base_ms=bt // 1000 - 1000,
                             step_us=max(1, INTERVAL_US // N_EVENTS))
        data = buf.numpy().tobytes()
        o = offs.tolist()
        out.append((bt, [data[o[k]:o[k + 1]] for k in range(N_EVENTS)]))
    return out


def _raw(records, device):
    from dxa.engine.processor import RawBatch
    from dxa.ops.jsonparse import frame_records
    buf, offs = frame_records(records)
    return RawBatch(buf.to(device), offs.to(device), len(records))


EMPTY_BATCH = 2          # the batch in which the last rank's share is empty


def _share(records, rank, world, b):
    """Rank ``rank``'s records of batch ``b``: every world-th event (as world source partitions would hold them),
    except that in batch EMPTY_BATCH the last rank receives nothing (an idle partition) and the others split it."""
    if world > 1 and b == EMPTY_BATCH:
        return [] if rank == world - 1 else records[rank::world - 1]
    return records[rank::world]


def _run(variant, rank, world, workdir, shared, batches, device="cpu"):
    """This rank's share of every batch through a Processor: per batch (sink lines by output, state rows, metrics)."""
    from dxa.engine.processor import Processor
    from dxa.io import sinks
    sinks.MEMORY_SINKS.clear()
    proc = Processor(_settings(variant, workdir, shared), device)
    out = []
    for b, (bt, records) in enumerate(batches):
        proc.clock = lambda bt=bt: bt / 1e6 + 0.25         # current_timestamp() (alert EventTime) pinned per batch
        m = proc.process_batch(_raw(_share(records, rank, world, b), device), bt, INTERVAL_US)
        m = proc.drain() or m
        lines = {k: list(v) for k, v in sinks.MEMORY_SINKS.items()}
        sinks.MEMORY_SINKS.clear()
        state = {n: st.active.to_pylist() for n, st in proc.state_tables.items()}
        metrics = {k: v for k, v in m.items() if k.startswith(("Input_", "Output_"))}
        out.append((lines, json.loads(json.dumps(state, default=str)), metrics))
    return out


def _worker(rank, world, port, q, variant, workdir, shared, batches, device):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import torch.distributed as dist
        if device != "cpu":
            torch.cuda.set_device(0)           # every rank on the one GPU; collectives staged through gloo
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dxa import parallel as P
        P.init(dist.group.WORLD, device)
        res = _run(variant, rank, world, workdir, shared, batches, device)
        q.put((rank, res, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(world, target, args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            rank, r, err = q.get(timeout=300)
            assert err is None, err
            res[rank] = r
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


def _key(row):
    def strip(v):
        if isinstance(v, dict):
            return tuple((k, strip(x)) for k, x in sorted(v.items()))
        if isinstance(v, list):
            return tuple(strip(x) for x in v)
        if isinstance(v, float):
            return "<f>"
        return v
    return repr(strip(row))


def _close(a, b, path=""):
    if isinstance(a, float) or isinstance(b, float):
        assert isinstance(a, (int, float)) and isinstance(b, (int, float)), (path, a, b)
        if math.isnan(a) and math.isnan(b):
            return
        assert math.isclose(a, b, rel_tol=1e-9, abs_tol=1e-9), (path, a, b)
        return
    if isinstance(a, dict):
        assert isinstance(b, dict) and a.keys() == b.keys(), (path, a, b)
        for k in a:
            _close(a[k], b[k], f"{path}.{k}")
        return
    if isinstance(a, list):
        assert isinstance(b, list) and len(a) == len(b), (path, len(a), len(b))
        for i, (x, y) in enumerate(zip(a, b)):
            _close(x, y, f"{path}[{i}]")
        return
    assert a == b, (path, a, b)


def _rows_equal(got, want, path):
    got = sorted(got, key=_key)
    want = sorted(want, key=_key)
    assert len(got) == len(want), (path, len(got), len(want))
    _close(got, want, path)


@pytest.mark.parametrize("world,device", [(2, "cpu"), (3, "cpu"), (4, "cpu"),
                                          pytest.param(2, "cuda", marks=pytest.mark.gpu),
                                          pytest.param(3, "cuda", marks=pytest.mark.gpu),
                                          pytest.param(4, "cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("variant", ["groupby", "window", "join", "full", "passthrough"])
def test_flow_ranks_match_one(variant, world, device, tmp_path):
    """W ranks (2, 3 — a world that is not a power of two, so ``owner_of``'s modulo is uneven — and 4), the last
    one idle in one batch, against the one-rank run.  ``cuda``: every rank on the test box's one GPU (every kernel,
    incl. the exchange pack / unpack kernels, on the device; the collectives staged through gloo)."""
    import time
    from dxa import parallel as P
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    shared1, shared2 = str(tmp_path / "one_shared"), str(tmp_path / "two_shared")     # state dirs differ per run
    for s in (shared1, shared2):
        os.makedirs(s, exist_ok=True)
        if variant == "join":
            iot.write_reference_csv(os.path.join(s, "ref.csv"), REF_ROWS, "cpu")
    clock0 = (int(time.time()) - 3600) * 1_000_000
    batches = _batches(clock0)
    P.shutdown()
    one = _run(variant, 0, 1, str(tmp_path / "one" / "w"), shared1, batches, device)
    two = _spawn_flow(variant, tmp_path, shared2, batches, device, world)
    ranks = range(world)
    rows_seen = 0
    for b in range(N_BATCHES):
        lines1, state1, m1 = one[b]
        names = set(lines1).union(*(set(two[r][b][0]) for r in ranks))
        for name in sorted(names):
            want = [json.loads(l) for l in lines1.get(name, [])]
            got = [json.loads(l) for r in ranks for l in two[r][b][0].get(name, [])]
            _rows_equal(got, want, f"batch{b}.{name}")
            rows_seen += len(want)
        for name in state1:
            _rows_equal([x for r in ranks for x in two[r][b][1][name]], state1[name], f"batch{b}.state.{name}")
        # the job-wide metrics (all-reduced) equal the one-rank metrics on every rank
        for r in ranks:
            assert two[r][b][2].keys() == m1.keys(), (b, r, sorted(set(two[r][b][2]) ^ set(m1)))
            for k in m1:
                assert two[r][b][2][k] == pytest.approx(m1[k]), (b, r, k)
    assert rows_seen, "no output rows at all"
    if variant == "full":
        assert one[-1][1]["DeviceState"], "accumulator never updated"
        # accumulator rows live on exactly one rank each
        ks = [{(x["deviceId"], x["homeId"], x["deviceType"]) for x in two[r][-1][1]["DeviceState"]} for r in ranks]
        assert all(ks)
        assert sum(len(k) for k in ks) == len(set().union(*ks))


def _spawn_flow(variant, tmp_path, shared, batches, device="cpu", world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, variant, str(tmp_path / f"two{r}" / "w"), shared,
                                               batches, device)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            rank, r, err = q.get(timeout=300)
            assert err is None, err
            res[rank] = r
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


# ---------------------------------------------------------------------------------------------------------------
# batch-metric reduction: rank-independent keys, MAX latencies, loud mismatch
# ---------------------------------------------------------------------------------------------------------------

def _write_blob(root, account, rel, lines):
    p = os.path.join(root, "wasbs", "data", f"{account}.blob.core.windows.net", rel)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        f.write("\n".join(json.dumps(l) for l in lines) + "\n")
    return f"wasbs://data@{account}.blob.core.windows.net/{rel}"


def _blob_worker(rank, world, port, q, root, work):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          DXA_FS_ROOT=root)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dxa import parallel as P
        from dxa.config.settings import SettingDictionary
        from dxa.engine.host import StreamingHost
        from dxa.engine.processor import Processor
        from dxa.io.sources import build_source
        P.init(dist.group.WORLD, "cpu")
        os.makedirs(work, exist_ok=True)
        for n, text in (("s.json", '{"type":"struct","fields":[{"name":"v","type":"long","nullable":true,'
                                   '"metadata":{}}]}'),
                        ("p.txt", "Raw.*\n"), ("t.txt", "--DataXQuery--\nT = SELECT v FROM DataXProcessedInput\n")):
            with open(os.path.join(work, n), "w") as f:
                f.write(text)
        d = SettingDictionary({
            "datax.job.name": "bp", "datax.job.input.default.blobschemafile": os.path.join(work, "s.json"),
            "datax.job.process.projection": os.path.join(work, "p.txt"),
            "datax.job.process.transform": os.path.join(work, "t.txt"),
            "datax.job.input.default.source.acct1.target": "TGT",
            "datax.job.input.default.filetimeregex": r"/(\d{4}-\d{2}-\d{2}T\d{2}_\d{2}_\d{2})/",
            "datax.job.output.T.null.enabled": "true"})
        proc = Processor(d, "cpu")
        src = build_source(d, "cpu", "blobpointer")
        # batch 0: rank 0 reads two files with file times, rank 1's batch is empty
        # batch 1: rank 1 reads one file with a file time, rank 0 one without
        if rank == 0:
            src.inner.push_many([json.dumps({"BlobPath": p}) for p in (
                _write_blob(root, "acct1", "2024-05-06T07_08_09/a.json", [{"v": 1}, {"v": 2}]),
                _write_blob(root, "acct1", "2024-05-06T07_00_00/b.json", [{"v": 3}]))])
        hist = []
        host = StreamingHost(proc, src, 1.0, max_batches=1, realtime=False, pipeline=False,
                             on_batch=lambda bt, m: hist.append(dict(m)))
        host.run()
        if rank == 1:
            src.inner.push_many([json.dumps({"BlobPath": _write_blob(root, "acct1", "2024-05-06T08_00_00/c.json",
                                                                     [{"v": 4}])})])
        else:
            src.inner.push_many([json.dumps({"BlobPath": _write_blob(root, "acct1", "notime/d.json", [{"v": 5}])})])
        host = StreamingHost(proc, src, 1.0, max_batches=1, realtime=False, pipeline=False,
                             on_batch=lambda bt, m: hist.append(dict(m)))
        host.run()
        # a rank whose metrics carry an extra key must fail loudly on every rank, not hang the collective
        err = None
        try:
            P.reduce_metrics({"a": 1.0, **({"extra": 1.0} if rank == 1 else {})}, "cpu")
        except P.MetricKeysMismatch as e:
            err = str(e)
        q.put((rank, (hist, err), None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def test_blob_pointer_metrics_with_an_empty_rank(tmp_path):
    import datetime as _dt
    res = _spawn(2, _blob_worker, (str(tmp_path / "fs"), str(tmp_path / "work")))
    now = _dt.datetime.utcnow()
    for r in (0, 1):
        hist, err = res[r]
        assert len(hist) == 2
        b0, b1 = hist
        assert b0["InputBlobs"] == 2 and b0["Input_DataXProcessedInput_Events_Count"] == 3
        # the earliest file time of the whole batch (07:00:00), not the sum over ranks
        exp0 = (now - _dt.datetime(2024, 5, 6, 7, 0, 0)).total_seconds()
        assert abs(b0["Latency-Blobs"] - exp0) < 120
        assert b1["InputBlobs"] == 2 and b1["Input_DataXProcessedInput_Events_Count"] == 2
        exp1 = (now - _dt.datetime(2024, 5, 6, 8, 0, 0)).total_seconds()
        assert abs(b1["Latency-Blobs"] - exp1) < 120
        assert err is not None and "differ across ranks" in err


def test_latency_dropped_when_no_rank_measures_it():
    from dxa import parallel as P
    P.shutdown()
    m = P.reduce_metrics({"InputBlobs": 0.0, "Latency-Blobs": float("-inf")}, "cpu")
    assert m == {"InputBlobs": 0.0}


def test_corrupt_device_batch_never_reaches_sinks_or_state(tmp_path):
    """A batch whose source-side decode failed raises before its rows reach a sink or an accumulator (the device
    decoder reports through ``RawBatch.status``, checked by ``process_batch`` ahead of the transform)."""
    from dxa.engine.processor import Processor
    from dxa.io import sinks
    from dxa.io.kafka_device import DecodeError
    from dxa import parallel as P
    P.shutdown()
    shared = str(tmp_path / "shared")
    proc = Processor(_settings("full", str(tmp_path / "w"), shared), "cpu")
    batches = _batches((1_700_000_000 // 1) * 1_000_000)[:2]
    sinks.MEMORY_SINKS.clear()
    bt, recs = batches[0]
    proc.clock = lambda: bt / 1e6
    proc.process_batch(_raw(recs, "cpu"), bt, INTERVAL_US)
    proc.drain()
    state_before = proc.state_tables["DeviceState"].active.to_pylist()
    sinks.MEMORY_SINKS.clear()

    class Bad:
        def raise_if_failed(self, what):
            raise DecodeError(f"{what}: corrupt")
    bt, recs = batches[1]
    raw = _raw(recs, "cpu")
    raw.status = Bad()
    with pytest.raises(DecodeError):
        proc.process_batch(raw, bt, INTERVAL_US)
    proc.drain()
    assert not any(sinks.MEMORY_SINKS.values())
    assert proc.state_tables["DeviceState"].active.to_pylist() == state_before
