"""Concurrent views at N ranks (Processor._run_concurrent + parallel.branch_groups): five independent views that
each shuffle rows or partials between ranks run on worker threads, branch i on communicator i, and a join reads
two of them.  On 2 gloo ranks the union of every view must equal the 1-rank statement-order run, batch by batch;
the schedule really runs a level of more than four branches (two rounds of slots)."""
import os
import socket
import traceback

import torch.multiprocessing as mp

TRANSFORM = """--DataXQuery--
ByKey = SELECT k, COUNT(*) AS c FROM DataXProcessedInput GROUP BY k

--DataXQuery--
ByMod = SELECT k % 3 AS m, MAX(v) AS mv, MIN(v) AS nv FROM DataXProcessedInput GROUP BY k % 3

--DataXQuery--
ByRem = SELECT v % 5 AS r, SUM(k) AS s FROM DataXProcessedInput GROUP BY v % 5

--DataXQuery--
Keys = SELECT DISTINCT k FROM DataXProcessedInput

--DataXQuery--
Totals = SELECT COUNT(*) AS n, SUM(v) AS sv FROM DataXProcessedInput

--DataXQuery--
Joined = SELECT a.k, a.c, d.k AS dk FROM ByKey a JOIN Keys d ON a.k = d.k
"""

SCHEMA = ('{"type":"struct","fields":[{"name":"k","type":"long","nullable":true,"metadata":{}},'
          '{"name":"v","type":"long","nullable":true,"metadata":{}}]}')
VIEWS = ["ByKey", "ByMod", "ByRem", "Keys", "Joined", "Totals"]


def _settings(work):
    from dxa.config.settings import SettingDictionary
    os.makedirs(work, exist_ok=True)
    paths = {n: os.path.join(work, n) for n in ("schema.json", "projection.txt", "transform.txt")}
    open(paths["schema.json"], "w").write(SCHEMA)
    open(paths["projection.txt"], "w").write("Raw.*\n")
    open(paths["transform.txt"], "w").write(TRANSFORM)
    d = {"datax.job.name": "cvtest",
         "datax.job.input.default.blobschemafile": paths["schema.json"],
         "datax.job.process.projection": paths["projection.txt"],
         "datax.job.process.transform": paths["transform.txt"]}
    d.update({f"datax.job.output.{v}.null.enabled": "true" for v in VIEWS})
    return SettingDictionary(d)


def _run(rank, world, work, batches):
    from dxa import parallel as P
    from dxa.engine.processor import Processor, RawBatch
    from dxa.ops.jsonparse import frame_records
    proc = Processor(_settings(os.path.join(work, f"r{rank}")), "cpu")
    proc.keep_views = True
    steps = proc._view_schedule(None)
    out = []
    for b in batches:
        rows = [((i * 7 + b) % 11, b * 1000 + i) for i in range(40 + 3 * b)]
        mine = [f'{{"k":{k},"v":{v}}}'.encode() for k, v in rows][rank::world]
        buf, offs = frame_records(mine)
        proc.process_batch(RawBatch(buf, offs, len(mine)), 1_000_000 * (b + 1), 1_000_000)
        proc.drain()
        views = {}
        for name in VIEWS:
            t = proc.last_views[name]
            if P.active() and P.dist_of(t) != P.REPLICATED:
                t = P.allgather_table(t)
            views[name] = sorted(tuple(r.values()) for r in t.to_pylist())
        out.append(views)
    return [len(s) for s in steps], out


def _worker(rank, world, port, work, batches, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          DXA_VIEW_STREAMS="threads")
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dxa import parallel as P
        P.init(dist.group.WORLD, "cpu")
        res = _run(rank, world, work, batches)
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


def test_concurrent_views_two_ranks_equal_sequential_one(tmp_path, monkeypatch):
    from dxa import parallel as P
    P.shutdown()
    monkeypatch.setenv("DXA_VIEW_STREAMS", "0")
    seq_steps, one = _run(0, 1, str(tmp_path / "w1"), [0, 1, 2])
    assert all(n == 1 for n in seq_steps)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path / "w2"), [0, 1, 2], q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, r, err = q.get(timeout=240)
        assert err is None, err
        res[rank] = r
    for p in procs:
        p.join(timeout=60)
    steps, two = res[0]
    assert max(steps) == 5, steps                # ByKey, ByMod, ByRem, Keys, Totals together: two rounds of four slots
    for i in range(3):
        for name in VIEWS:
            assert two[i][name] == one[i][name], (i, name, two[i][name], one[i][name])
        assert res[1][1][i] == two[i]
