"""Accumulator (state) tables across ranks: the ``UNION ALL <state> … GROUP BY`` upsert pattern of BASELINE config 5
run on 2 gloo ranks must equal the 1-rank run, batch by batch, and survive a kill-and-restart — including a restart
at a different world size (reference: StateTableHandler.scala:70-128, CommonProcessorFactory.scala:244-264,318-320).
"""
import os
import socket
import traceback

import pytest
import torch.multiprocessing as mp

TRANSFORM = """--DataXQuery--
Agg = SELECT k, COUNT(*) AS c, MAX(v) AS mv FROM DataXProcessedInput GROUP BY k

--DataXQuery--
S = SELECT k, SUM(c) AS c, MAX(mv) AS mv
    FROM (SELECT k, c, mv FROM Agg UNION ALL SELECT k, c, mv FROM S) u
    GROUP BY k

--DataXQuery--
G = SELECT COUNT(*) AS n, SUM(c) AS total FROM S
"""

SCHEMA = ('{"type":"struct","fields":[{"name":"k","type":"long","nullable":true,"metadata":{}},'
          '{"name":"v","type":"long","nullable":true,"metadata":{}}]}')

N_KEYS = 13


def _settings(work, state_dir):
    from dxa.config.settings import SettingDictionary
    os.makedirs(work, exist_ok=True)
    paths = {n: os.path.join(work, n) for n in ("schema.json", "projection.txt", "transform.txt")}
    open(paths["schema.json"], "w").write(SCHEMA)
    open(paths["projection.txt"], "w").write("Raw.*\n")
    open(paths["transform.txt"], "w").write(TRANSFORM)
    return SettingDictionary({
        "datax.job.name": "statetest",
        "datax.job.input.default.blobschemafile": paths["schema.json"],
        "datax.job.process.projection": paths["projection.txt"],
        "datax.job.process.transform": paths["transform.txt"],
        "datax.job.process.statetable.S.schema": "k long, c long, mv long",
        "datax.job.process.statetable.S.location": state_dir,
        "datax.job.output.S.null.enabled": "true",
        "datax.job.output.G.null.enabled": "true",
    })


def _batch_rows(b):
    # batch b: 3*N_KEYS + b events, keys skewed so each rank sees every key in some batches and not in others
    return [(i * 7 + b) % N_KEYS for i in range(3 * N_KEYS + b)]


def _run(rank, world, work, state_dir, batches):
    """Run ``batches`` on this rank; returns per batch this rank's state rows and the global view G."""
    from dxa import parallel as P
    from dxa.engine.processor import Processor, RawBatch
    from dxa.ops.jsonparse import frame_records
    proc = Processor(_settings(os.path.join(work, f"r{rank}"), state_dir), "cpu")
    proc.keep_views = True
    out = []
    for b in batches:
        rows = _batch_rows(b)
        mine = [f'{{"k":{k},"v":{b * 100 + i}}}'.encode() for i, k in enumerate(rows)][rank::world]
        buf, offs = frame_records(mine)
        proc.process_batch(RawBatch(buf, offs, len(mine)), 1_000_000 * (b + 1), 1_000_000)
        proc.drain()
        st = proc.state_tables["S"].active
        g = proc.last_views["G"]
        if P.active() and P.dist_of(g) != P.REPLICATED:
            g = P.allgather_table(g)
        out.append((sorted(tuple(r.values()) for r in st.to_pylist()), g.to_pylist()))
    return out


def _worker(rank, world, port, work, state_dir, batches, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dxa import parallel as P
        P.init(dist.group.WORLD, "cpu")
        res = _run(rank, world, work, state_dir, batches)
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


def _run_world(world, work, state_dir, batches):
    if world == 1:
        from dxa import parallel as P
        P.shutdown()
        return {0: _run(0, 1, work, state_dir, batches)}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, work, state_dir, batches, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, r, err = q.get(timeout=240)
        assert err is None, err
        res[rank] = r
    for p in procs:
        p.join(timeout=60)
    return res


def _expected(batches):
    acc = {}
    for b in batches:
        for i, k in enumerate(_batch_rows(b)):
            c, mv = acc.get(k, (0, None))
            acc[k] = (c + 1, max(mv or 0, b * 100 + i))
    return sorted((k, c, mv) for k, (c, mv) in acc.items())


def _union(res, i):
    return sorted(r for rank in res for r in res[rank][i][0])


def test_state_union_upsert_two_ranks_equals_one(tmp_path):
    one = _run_world(1, str(tmp_path / "w1"), str(tmp_path / "s1"), [0, 1, 2])
    two = _run_world(2, str(tmp_path / "w2"), str(tmp_path / "s2"), [0, 1, 2])
    for i in range(3):
        exp = _expected(range(i + 1))
        assert one[0][i][0] == exp
        assert _union(two, i) == exp, (i, two[0][i][0], two[1][i][0])
        # every key lives on exactly one rank (the owner of its hash), no duplicates
        keys0 = {r[0] for r in two[0][i][0]}
        keys1 = {r[0] for r in two[1][i][0]}
        assert not (keys0 & keys1)
        assert two[0][i][1] == two[1][i][1] == [{"n": N_KEYS, "total": sum(r[1] for r in exp)}]
    # per-rank parts on disk, one metadata file naming the world that wrote them
    meta = open(tmp_path / "s2" / "metadata.info").read()
    assert "parts=2" in meta and "dist=hashed" in meta
    active = dict(l.split("=", 1) for l in meta.splitlines())["active"]
    assert sorted(os.listdir(tmp_path / "s2" / active)) == ["part-0.parquet", "part-1.parquet"]


@pytest.mark.parametrize("w_before,w_after", [(2, 2), (2, 1), (1, 2)])
def test_state_restart_resumes(tmp_path, w_before, w_after):
    """Kill after two batches, restart (possibly at another world size) and run the third: same state as 3
    uninterrupted batches."""
    state = str(tmp_path / "state")
    _run_world(w_before, str(tmp_path / "a"), state, [0, 1])
    after = _run_world(w_after, str(tmp_path / "b"), state, [2])
    assert _union(after, 0) == _expected([0, 1, 2])


def test_pipelined_overwrite_defers_standby_write_until_previous_flip(tmp_path):
    """Batch t+1 overwrites the state before batch t is persisted (outputs pipelined): its standby write must wait
    for t's flip + release (it targets the copy t's on-disk metadata still names active), while the device-side
    state moves on at once."""
    import os
    from dxa.engine.column import column_from_pylist, Table
    from dxa.engine.state import StateTable
    from dxa.engine.types import parse_ddl_schema
    loc = str(tmp_path / "st")
    st = StateTable("S", parse_ddl_schema("k long, v long"), loc, "cpu")

    def tab(v):
        return Table(["k", "v"], [column_from_pylist([1], "long"), column_from_pylist([v], "long")], 1)

    def meta():
        return dict(line.split("=", 1) for line in open(os.path.join(loc, "metadata.info")).read().split())

    st.overwrite(tab(10), tag=1)              # batch 1 → copy B
    st.overwrite(tab(20), tag=2)              # batch 2 → copy A, deferred (batch 1 not flipped yet)
    assert st.active.columns[1].to_pylist() == [20]
    assert st._writes[1].job is not None and st._writes[1].fut is None
    st.flush(1)
    assert st.persist(1)
    assert meta()["active"] == "B"
    assert not os.path.exists(os.path.join(loc, "A", "part-0.parquet"))   # batch 2 has not touched A yet
    st.release()
    st.flush(2)
    assert os.path.exists(os.path.join(loc, "A", "part-0.parquet"))
    assert st.persist(2)
    st.release()
    assert meta()["active"] == "A" and not st.modified
    again = StateTable("S", parse_ddl_schema("k long, v long"), loc, "cpu")
    assert again.active.columns[1].to_pylist() == [20]
