"""Rank-partitioned ingest: every source and the blob batch host must split the stream across
ranks, never duplicate it — 2 gloo ranks produce the same totals and the same aggregate as 1 rank.
(Reference: BlobBatchingHost.scala:68-105 ``sc.makeRDD(filesToProcess)``; KafkaStreamingFactory.scala:70-74.)"""
import datetime as dt
import gzip
import json
import os
import socket
import traceback

import pytest
import torch.multiprocessing as mp

SCHEMA = ('{"type":"struct","fields":[{"name":"k","type":"long","nullable":true,"metadata":{}},'
          '{"name":"v","type":"long","nullable":true,"metadata":{}}]}')
TRANSFORM = """--DataXQuery--
Agg = SELECT k, COUNT(*) AS c, SUM(v) AS sv FROM DataXProcessedInput GROUP BY k
"""


def _settings(work, extra):
    from dxa.config.settings import SettingDictionary
    os.makedirs(work, exist_ok=True)
    p = {n: os.path.join(work, n) for n in ("schema.json", "projection.txt", "transform.txt")}
    open(p["schema.json"], "w").write(SCHEMA)
    open(p["projection.txt"], "w").write("Raw.*\n")
    open(p["transform.txt"], "w").write(TRANSFORM)
    d = {"datax.job.name": "srctest", "datax.job.input.default.blobschemafile": p["schema.json"],
         "datax.job.process.projection": p["projection.txt"], "datax.job.process.transform": p["transform.txt"],
         "datax.job.output.Agg.null.enabled": "true"}
    d.update(extra)
    return SettingDictionary(d)


def _make_inputs(root):
    """Files for the file source (12 files, one gzip) and the batch host (3 hourly partitions)."""
    files = os.path.join(root, "files")
    os.makedirs(files, exist_ok=True)
    for i in range(12):
        lines = "\n".join(json.dumps({"k": (i * 5 + j) % 7, "v": i * 100 + j}) for j in range(9)) + "\n"
        path = os.path.join(files, f"part-{i:02d}.json" + (".gz" if i == 3 else ""))
        with open(path, "wb") as f:
            f.write(gzip.compress(lines.encode()) if i == 3 else lines.encode())
    for h in range(3):
        d = os.path.join(root, "blobs", f"2020-01-02", f"{h:02d}")
        os.makedirs(d, exist_ok=True)
        for j in range(4):
            with open(os.path.join(d, f"f{j}.json"), "w") as f:
                f.write("\n".join(json.dumps({"k": (h + j + r) % 5, "v": h * 1000 + j * 10 + r})
                                  for r in range(6)) + "\n")


def _collect(proc, P):
    m = proc.last_metrics
    agg = proc.last_views["Agg"]
    if P.active() and P.dist_of(agg) != P.REPLICATED:
        agg = P.allgather_table(agg)
    return m["Input_DataXProcessedInput_Events_Count"], sorted((tuple(r.values()) for r in agg.to_pylist()), key=repr)


def _run_all(rank, world, root):
    from dxa import parallel as P
    from dxa.engine.host import BlobBatchingHost
    from dxa.engine.processor import Processor
    from dxa.io.sources import PartitionedReplaySource, build_source
    out = {}
    # local generator: the job's rate split across ranks
    proc = Processor(_settings(os.path.join(root, f"w-local-{rank}"),
                               {"datax.job.input.default.local.eventsperbatch": "101"}), "cpu")
    proc.keep_views = True
    src = build_source(proc.settings, "cpu")
    for b in range(2):
        proc.process_batch(src.next_batch(1_000_000 * (b + 1)), 1_000_000 * (b + 1), 1_000_000)
    proc.drain()
    out["local"] = _collect(proc, P)
    # file source
    proc = Processor(_settings(os.path.join(root, f"w-file-{rank}"),
                               {"datax.job.input.default.file.pattern": os.path.join(root, "files", "*.json*")}),
                     "cpu")
    proc.keep_views = True
    src = build_source(proc.settings, "cpu")
    proc.process_batch(src.next_batch(1_000_000), 1_000_000, 1_000_000)
    proc.drain()
    out["file"] = _collect(proc, P)
    # replay (partitioned log) source: 5 partitions
    logs = {f"p{i}": [json.dumps({"k": (i + j) % 4, "v": j}).encode() for j in range(7 + i)] for i in range(5)}
    proc = Processor(_settings(os.path.join(root, f"w-replay-{rank}"), {}), "cpu")
    proc.keep_views = True
    src = PartitionedReplaySource(logs, "cpu", checkpoint_dir=os.path.join(root, f"ckpt-w{world}"))
    proc.process_batch(src.next_batch(1_000_000), 1_000_000, 1_000_000)
    proc.drain()
    src.commit(1_000_000)
    out["replay"] = _collect(proc, P)
    # blob batch host: one batch over every partition's files
    proc = Processor(_settings(os.path.join(root, f"w-batch-{rank}"), {}), "cpu")
    proc.keep_views = True
    host = BlobBatchingHost(proc, "cpu", [os.path.join(root, "blobs", "{yyyy-MM-dd}", "{HH}")],
                            dt.datetime(2020, 1, 2, 0), dt.datetime(2020, 1, 2, 2), dt.timedelta(hours=1))
    res = host.run()
    out["batch"] = _collect(proc, P) + (res[0]["InputBlobs"], len(res))
    return out


def _worker(rank, world, port, root, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dxa import parallel as P
        P.init(dist.group.WORLD, "cpu")
        q.put((rank, _run_all(rank, world, root), None))
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


def test_sources_split_across_ranks(tmp_path):
    root = str(tmp_path)
    _make_inputs(root)
    from dxa import parallel as P
    P.shutdown()
    one = _run_all(0, 1, root)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, root, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, r, err = q.get(timeout=240)
        assert err is None, err
        res[rank] = r
    for p in procs:
        p.join(timeout=60)
    assert one["local"][0] == 101 and one["file"][0] == 12 * 9 and one["replay"][0] == sum(7 + i for i in range(5))
    assert one["batch"][0] == 3 * 4 * 6 and one["batch"][2] == 12 and one["batch"][3] == 1
    for kind in ("local", "file", "replay", "batch"):
        for r in (0, 1):
            assert res[r][kind] == one[kind], (kind, r, res[r][kind], one[kind])
    # each rank checkpointed only its own partitions, and restore merges every rank's file
    from dxa.io.sources import Checkpointer
    merged = Checkpointer(os.path.join(root, "ckpt-w2"), 0, 1).restore()
    assert merged == {("replay", f"p{i}"): 7 + i for i in range(5)}


def test_socket_source_listens_per_rank():
    from dxa.io.sources import SocketSource
    port = _free_port()
    a = SocketSource("cpu", port=port, rank=0)
    try:
        b = SocketSource("cpu", port=port, rank=1)      # no address-in-use: rank 1 listens on port + 1
    except OSError:
        pytest.skip("port + 1 taken by another process")
    try:
        assert (a.port, b.port) == (port, port + 1)
    finally:
        a.close()
        b.close()


def test_list_matching_globs(tmp_path):
    from dxa.io import fs
    for rel in ("a/x.json", "a/y.txt", "a/b/z.json", "c.json"):
        p = tmp_path / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text("{}\n")
    base = str(tmp_path)
    assert [os.path.relpath(f, base) for f in fs.list_matching(base + "/a/*.json")] == ["a/x.json"]
    assert [os.path.relpath(f, base) for f in fs.list_matching(base + "/a/**/*.json")] == ["a/b/z.json", "a/x.json"]
    assert len(fs.list_matching(base + "/a")) == 3                      # a folder is listed recursively
    assert fs.owned_by_rank(["x", "y", "z"], 0, 1) == ["x", "y", "z"]
    shares = [fs.owned_by_rank([f"f{i}" for i in range(40)], r, 3) for r in range(3)]
    assert sorted(sum(shares, [])) == sorted(f"f{i}" for i in range(40)) and all(shares)
