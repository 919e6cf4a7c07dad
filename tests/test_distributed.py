"""Multi-process (gloo, world_size 2) tests of the RCCL-style exchange paths: two-phase distributed GROUP BY,
non-decomposable shuffle aggregation, DISTINCT, partitioned ⨝ partitioned joins, window functions (OVER) and the
table shuffle itself.
Each rank holds half of the rows; results must equal a single-process run over all rows."""
import json
import os
import random
import socket
import traceback

import pytest
import torch
import torch.multiprocessing as mp

QUERIES = [
    "SELECT k, s, COUNT(*) AS c, SUM(v) AS sv, MIN(v) AS mn, MAX(v) AS mx, AVG(v) AS av, STDDEV(v) AS sd "
    "FROM T GROUP BY k, s",
    "SELECT COUNT(*) AS c, SUM(v) AS sv, MAX(s) AS ms FROM T",
    "SELECT k, COUNT(DISTINCT s) AS ds FROM T GROUP BY k",
    "SELECT DISTINCT s FROM T",
    "SELECT a.k, COUNT(*) AS c FROM T a JOIN T2 b ON a.k = b.k GROUP BY a.k",
    "SELECT k, SUM(v) AS sv FROM T WHERE v > 0 GROUP BY k HAVING COUNT(*) > 3",
    # window functions: shuffled by PARTITION BY keys, or gathered without one / over grouped rows
    "SELECT k, s, v, RANK() OVER (PARTITION BY k ORDER BY v DESC) AS r, SUM(v) OVER (PARTITION BY k) AS tot, "
    "MAX(v) OVER (PARTITION BY k ORDER BY v ROWS BETWEEN 2 PRECEDING AND CURRENT ROW) AS m3 FROM T",
    "SELECT k, v, DENSE_RANK() OVER (ORDER BY k) AS dr, COUNT(*) OVER () AS n FROM T",
    "SELECT k, SUM(v) AS sv, RANK() OVER (ORDER BY k DESC) AS r FROM T GROUP BY k",
    # the extended SQL surface over partitioned inputs
    "SELECT k, percentile(v, 0.5) AS p, percentile_approx(v, 0.25) AS pa FROM T GROUP BY k",
    "WITH w AS (SELECT k, v FROM T WHERE v > 0) SELECT k, COUNT(*) AS c FROM w GROUP BY k",
    "SELECT k, v FROM T WHERE k IN (SELECT k FROM T2)",
    "SELECT k, v FROM T t WHERE NOT EXISTS (SELECT 1 FROM T2 b WHERE b.k = t.k)",
    "SELECT a.k, a.v, b.v AS bv FROM T a LEFT JOIN T2 b ON a.k = b.k AND a.v > 5",
    "SELECT k, explode(split(s, 'b')) AS part FROM T WHERE s IS NOT NULL",
    "SELECT (SELECT MAX(v) FROM T) AS m, COUNT(*) AS c FROM T",
    # the variance family's (n, mean, M2) partials merged with Chan's formula: with a 1e6 offset the one-pass
    # Σx² − n·mean² form loses the 6th decimal
    "SELECT k, STDDEV(v + 1e6) AS sd, VAR_POP(v - 1e6) AS vp FROM T GROUP BY k",
]


def _rows(seed, n):
    rnd = random.Random(seed)
    return [{"k": rnd.randrange(20), "s": rnd.choice(["a", "bb", "ccc", None]),
             "v": None if rnd.random() < 0.05 else round(rnd.uniform(-10, 10), 3)} for _ in range(n)]


def _canon(rows):
    out = []
    for r in rows:
        out.append(tuple((k, ("nan" if v != v else round(v, 6)) if isinstance(v, float) else v)
                         for k, v in sorted(r.items())))
    return sorted(out, key=repr)


def _worker(rank, world, port, q, device="cpu"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import torch.distributed as dist
        if device != "cpu":
            torch.cuda.set_device(0)       # every rank on the one GPU; collectives staged through gloo
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dxa import parallel as P
        from dxa.engine.column import Table
        from dxa.engine.expr import EvalContext
        from dxa.engine.query import Catalog, run_sql
        from dxa.engine.types import StructField, StructType
        P.init(dist.group.WORLD, device)
        schema = StructType((StructField("k", "long"), StructField("s", "string"), StructField("v", "double")))
        rows = _rows(1, 400)
        rows2 = [{"k": k, "s": "x", "v": 1.0} for k in range(0, 20, 2) for _ in range(2)]
        mine = rows[rank::world]
        mine2 = rows2[rank::world]
        t = Table.from_pylist(mine, schema, device)
        t.dist = P.PARTITIONED
        t2 = Table.from_pylist(mine2, schema, device)
        t2.dist = P.PARTITIONED
        cat = Catalog()
        cat.register("T", t)
        cat.register("T2", t2)
        results = []
        for qsql in QUERIES:
            out = run_sql(qsql, cat, EvalContext())
            if P.dist_of(out) != P.REPLICATED:
                out = P.allgather_table(out)
            results.append(out.to_pylist())
        # paned window aggregation over partitioned panes (partials exchanged, not rows)
        results.append(_window_results(t, P))
        # raw shuffle round trip
        dest = torch.tensor([i % world for i in range(t.length)], dtype=torch.int64, device=device)
        got = P.shuffle_table(t, dest)
        back = P.allgather_table(got)
        results.append(back.to_pylist())
        # round-robin rebalance of a skewed batch (input repartition): 300 + 100 rows → 200 + 200
        skew = Table.from_pylist(rows[:300] if rank == 0 else rows[300:], schema, device)
        reb = P.rebalance_table(skew)
        results.append((reb.length, P.allgather_table(reb).to_pylist()))
        q.put((rank, results, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, None, traceback.format_exc()))


WINDOW_QUERIES = ["SELECT k, COUNT(*) AS c, SUM(v) AS sv, AVG(v) AS av FROM WV GROUP BY k",
                  "SELECT COUNT(*) AS c, MIN(v) AS mn FROM WV"]


def _window_results(t, P):
    from dxa.engine.column import PrimColumn
    from dxa.engine.expr import EvalContext
    from dxa.engine.query import Catalog, run_sql
    from dxa.engine.windows import TimeWindowConf, WindowStore
    S = 1_000_000
    store = WindowStore(TimeWindowConf({"WV": 10 * S}, True, "ts", 0, 10 * S, False))
    views = None
    for b in range(4):
        T = (100 + b) * S
        ts = PrimColumn("timestamp", torch.full((t.length,), T + 1, dtype=torch.int64, device=t.device))
        tb = t.with_column("ts", ts)
        tb.dist = t.dist
        views, _ = store.process(tb, T, S)
    cat = Catalog()
    cat.register("WV", views["WV"])
    out = []
    for qsql in WINDOW_QUERIES:
        r = run_sql(qsql, cat, EvalContext())
        if P.active() and P.dist_of(r) != P.REPLICATED:
            r = P.allgather_table(r)
        out.append(r.to_pylist())
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_two_rank_queries_match_single_process(device):
    """``cuda``: both ranks on the one GPU of a test box, every kernel on the device and the collectives staged
    through gloo — the distributed operators' device code on real hardware, short of RCCL itself."""
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dxa.engine.column import Table
    from dxa.engine.expr import EvalContext
    from dxa.engine.query import Catalog, run_sql
    from dxa.engine.types import StructField, StructType
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, device)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, results, err = q.get(timeout=240)
        assert err is None, err
        res[rank] = results
    for p in procs:
        p.join(timeout=60)
    schema = StructType((StructField("k", "long"), StructField("s", "string"), StructField("v", "double")))
    rows = _rows(1, 400)
    rows2 = [{"k": k, "s": "x", "v": 1.0} for k in range(0, 20, 2) for _ in range(2)]
    cat = Catalog()
    cat.register("T", Table.from_pylist(rows, schema))
    cat.register("T2", Table.from_pylist(rows2, schema))
    for i, qsql in enumerate(QUERIES):
        expect = _canon(run_sql(qsql, cat, EvalContext()).to_pylist())
        for r in (0, 1):
            assert _canon(res[r][i]) == expect, (qsql, r)
    # windowed: 3 earlier batches (the current one is after E) of all rows
    expect_w = _window_results(Table.from_pylist(rows, schema), type("NoP", (), {"active": staticmethod(lambda: False)}))
    for r in (0, 1):
        for i in range(len(WINDOW_QUERIES)):
            assert _canon(res[r][len(QUERIES)][i]) == _canon(expect_w[i]), (WINDOW_QUERIES[i], r)
    # shuffle round trip preserves the multiset of rows
    for r in (0, 1):
        assert _canon(res[r][-2]) == _canon(rows)
    # rebalance: equal shares, same multiset
    for r in (0, 1):
        n_r, everything = res[r][-1]
        assert n_r == 200 and _canon(everything) == _canon(rows)


@pytest.mark.parametrize("flow,device", [("groupby", "cpu"), ("window", "cpu"), ("full", "cpu"), ("join", "cpu"),
                                         ("passthrough", "cpu"),
                                         pytest.param("groupby", "cuda", marks=pytest.mark.gpu),
                                         pytest.param("full", "cuda", marks=pytest.mark.gpu),
                                         pytest.param("join", "cuda", marks=pytest.mark.gpu)])
def test_bench_two_ranks_gloo(flow, device, tmp_path):
    """bench.py's multi-rank path (the driver's N-GPU scaling run) rehearsed on CPU: two ranks, gloo, one JSON line
    whose value aggregates both ranks — catches collective mismatches before they reach RCCL.  (Output correctness
    at two ranks — every flow's rows and state equal to the one-rank run — is gated by tests/test_flows_dist.py;
    here the bench's own ranks hold different random batches, so only the job-wide counts are checked.)"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    if device == "cuda":
        if not torch.cuda.is_available():
            pytest.skip("no GPU")
        env["DXA_DIST_BACKEND"] = "gloo"          # both ranks share the test box's one GPU
    else:
        env["HIP_VISIBLE_DEVICES"] = ""
    bench_args = [os.path.join(root, "bench.py"), "--gpus", "2", "--flow", flow, "--events-per-batch", "500",
                  "--steps", "2", "--warmup", "3", "--ref-rows", "5000"]
    for _attempt in range(3):         # the free port can be taken by a parallel test between probe and bind
        if device == "cuda":
            # bench.py starts its own ranks for --gpus N (no launcher): the driver's plain `bench.py --gpus N`
            r = subprocess.run([sys.executable] + bench_args, capture_output=True, text=True,
                               env=dict(env, MASTER_PORT=str(_free_port())), timeout=600, cwd=str(tmp_path))
        else:
            r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                                "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + bench_args,
                               capture_output=True, text=True, env=env, timeout=600, cwd=str(tmp_path))
        err = r.stderr.lower()
        if r.returncode == 0 or not any(m in err for m in ("address already in use", "eaddrinuse",
                                                           "failed to listen", "connection refused")):
            break
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 1000 and out["value"] > 0
    outs = out["last_batch_outputs"]
    # job-wide (all-reduced) sink counts: every output saw rows, and for the passthrough flow that is every event
    # of both ranks
    assert outs and all(v >= 0 for v in outs.values())
    if flow == "passthrough":
        assert outs["Output_Tagged_Sink_InputEvents"] == 1000
    # the value is the job's events over the MAX-over-ranks elapsed time
    assert out["value"] == pytest.approx(1000 * 2 / (out["ms_per_step"] * 2 / 1e3), rel=1e-9)


@pytest.mark.parametrize("n", [3, 4])
def test_bench_launches_its_own_ranks(n, tmp_path):
    """``python bench.py --gpus N`` with no launcher starts N rank processes itself (subprocesses, before any GPU
    call) and prints ONE job-wide line with ``n_gpus`` N: the driver's scaling run must not silently measure one
    rank.  Passthrough tags and writes every event, so its job-wide sink count is exactly N x events."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, HIP_VISIBLE_DEVICES="", MASTER_PORT=str(_free_port()))
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n), "--flow", "passthrough",
                        "--events-per-batch", "300", "--steps", "2", "--warmup", "2"], capture_output=True, text=True,
                       env=env, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["config"]["parallelism"] == f"dp{n}"
    assert out["config"]["global_batch"] == 300 * n
    assert out["last_batch_outputs"]["Output_Tagged_Sink_InputEvents"] == 300 * n


def test_bench_rejects_world_size_mismatch(tmp_path):
    """A launcher's WORLD_SIZE that disagrees with --gpus fails loudly instead of reporting the wrong n_gpus."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, HIP_VISIBLE_DEVICES="", WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, env=env, timeout=120, cwd=str(tmp_path))
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_bench_failing_rank_fails_the_job(tmp_path):
    """One rank dying makes the self-launched job exit non-zero (the survivors are stopped, not left hanging)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, HIP_VISIBLE_DEVICES="", MASTER_PORT=str(_free_port()),
               DXA_BENCH_FAIL_RANK="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--flow", "passthrough",
                        "--events-per-batch", "100", "--steps", "1", "--warmup", "1"], capture_output=True,
                       text=True, env=env, timeout=300, cwd=str(tmp_path))
    assert r.returncode != 0
    assert "exited with" in r.stderr and "failing on request" in r.stderr


def test_cpulist_parsing_and_cpu_noop():
    from dxa.parallel.affinity import bind_to_device, parse_cpulist
    assert parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert parse_cpulist("") == set()
    if not __import__("torch").cuda.is_available():
        assert bind_to_device(0) is None          # no GPU: nothing to bind to, affinity untouched


def test_kfd_topology_maps_hip_index_to_pci_folder(tmp_path, monkeypatch):
    """The GPU → PCI mapping comes from the KFD topology alone (usable before the HIP runtime starts)."""
    from dxa.parallel.affinity import kfd_pci_path
    topo, pci = tmp_path / "nodes", tmp_path / "pci"
    # node 0: CPU (no SIMDs); nodes 1, 2: GPUs on buses 0x05 and 0x75 (location_id = bus << 8)
    for n, simd, loc in ((0, 0, 0), (1, 256, 0x0500), (2, 256, 0x7500)):
        d = topo / str(n)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simd}\nlocation_id {loc}\ndomain 0\n")
    for bdf in ("0000:05:00.0", "0000:75:00.0"):
        (pci / bdf).mkdir(parents=True)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert kfd_pci_path(0, str(topo), str(pci)).endswith("0000:05:00.0")
    assert kfd_pci_path(1, str(topo), str(pci)).endswith("0000:75:00.0")
    assert kfd_pci_path(2, str(topo), str(pci)) is None
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert kfd_pci_path(0, str(topo), str(pci)).endswith("0000:75:00.0")


def _bcast_worker(rank, world, port, q, path, device="cpu"):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import torch.distributed as dist
        if device != "cpu":
            torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dxa import parallel as P
        from dxa.engine.column import Table
        from dxa.engine.types import StructField, StructType
        from dxa.io.refdata import load_csv
        P.init(dist.group.WORLD, device)
        schema = StructType((StructField("k", "long"), StructField("s", "string"), StructField("v", "double")))
        rows = _rows(3, 50) if rank == 0 else []
        t = P.broadcast_table(Table.from_pylist(rows, schema, device))
        st = {}
        ref = load_csv(path, ",", True, device, stats=st)
        # on a GPU only rank 0 stages the file in host memory; the others receive it straight into HBM
        assert device == "cpu" or st["host_staged"] == (rank == 0), st
        ag = P.allgather_table(Table.from_pylist(rows if rank == 0 else _rows(4, 7), schema, device))
        q.put((rank, (t.to_pylist(), ref.to_pylist(), ag.to_pylist()), None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_broadcast_table_and_reference_data(tmp_path, device):
    """Rank 0's table / reference file reaches every rank through broadcasts (no per-rank file reads); an
    all-gather of uneven shares (50 and 7 rows) gives every rank both, in rank order."""
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    path = tmp_path / "ref.csv"
    path.write_text('id,name\n1,"a,b"\n2,\n')
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bcast_worker, args=(r, 2, port, q, str(path), device)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, r, err = q.get(timeout=240)
        assert err is None, err
        res[rank] = r
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert _canon(res[r][0]) == _canon(_rows(3, 50))
        assert res[r][1] == [{"id": "1", "name": "a,b"}, {"id": "2", "name": None}]
        assert res[r][2] == res[0][2] and _canon(res[r][2]) == _canon(_rows(3, 50) + _rows(4, 7))
        assert [x["k"] for x in res[r][2]] == [x["k"] for x in _rows(3, 50) + _rows(4, 7)]     # rank order


def test_host_threads_share_the_socket(monkeypatch):
    """Co-located ranks bound to one socket split its CPUs for host-side batch work."""
    from dxa.parallel import affinity as AF
    monkeypatch.setattr(AF.os, "sched_getaffinity", lambda pid: set(range(64)))
    monkeypatch.setattr(AF, "local_cpus", lambda j: set(range(64)) if j < 4 else set(range(64, 128)))
    assert AF.host_threads(0, 1) == 16
    assert AF.host_threads(0, 8) == 16            # 4 ranks on 64 CPUs
    assert AF.host_threads(5, 8, cap=32) == 16
    monkeypatch.setattr(AF.os, "sched_getaffinity", lambda pid: set(range(16)))
    assert AF.host_threads(0, 8) == 4
    monkeypatch.setattr(AF, "local_cpus", lambda j: None)
    assert AF.host_threads(0, 8) == 2
