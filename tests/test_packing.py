"""Wire format of the RCCL table exchanges (dxa/parallel/packing.py, dxa/ops/csrc/exchange.hip): the device pack
(histogram + scan + scatter) must produce exactly the torch reference's send sizes, matrix and string arenas, and
unpacking a destination's block must give back that destination's rows in their original order.  The exchange
runs under every distributed GROUP BY / JOIN / DISTINCT — the multi-rank tests (test_distributed,
test_flows_dist) cover the collectives themselves."""
import random

import pytest
import torch

from dxa.engine.column import Table
from dxa.engine.types import StructField, StructType
from dxa.parallel import packing as PK

W = 5

SCHEMA = StructType((
    StructField("id", "long"), StructField("x", "double"), StructField("flag", "boolean"),
    StructField("name", "string"), StructField("note", "string"),
    StructField("st", StructType((StructField("a", "long"), StructField("b", "string")))),
))


def _rows(n, seed=3):
    rnd = random.Random(seed)

    def s(maxlen):
        if rnd.random() < 0.1:
            return None
        return "".join(rnd.choice("abcdefghij€é") for _ in range(rnd.randrange(0, maxlen)))
    out = []
    for i in range(n):
        out.append({"id": None if rnd.random() < 0.05 else rnd.randrange(-10**12, 10**12),
                    "x": rnd.choice([None, rnd.uniform(-1e6, 1e6), float("inf")]),
                    "flag": rnd.choice([None, True, False]), "name": s(24), "note": s(300),
                    "st": None if rnd.random() < 0.1 else {"a": rnd.randrange(100), "b": s(8)}})
    return out


def _canon(v):
    if isinstance(v, float) and v != v:
        return "nan"
    if isinstance(v, dict):
        return {k: _canon(x) for k, x in v.items()}
    return v


def _roundtrip(t, dest, force_torch):
    """Pack → per-destination unpack; returns (sizes, mat, arenas, [table per destination])."""
    lay = PK.Layout(t)
    sizes, state = PK.plan(lay, dest, W, force_torch)
    sz = sizes.tolist()
    send_rows = [r[0] for r in sz]
    send_bytes = [[r[1 + s] for r in sz] for s in range(lay.S)]
    mat, arenas = PK.scatter(lay, state, send_rows, send_bytes)
    outs = []
    r0 = 0
    b0 = [0] * lay.S
    for d in range(W):
        rows = send_rows[d]
        block = mat[r0:r0 + rows]
        ars = []
        for s in range(lay.S):
            nb = send_bytes[s][d]
            buf = torch.zeros(nb + 16, dtype=torch.uint8, device=t.device)
            buf[:nb] = arenas[s][b0[s]:b0[s] + nb]
            ars.append(buf)
            b0[s] += nb
        outs.append(PK.unpack(lay.names, lay.spec, lay.meta(), block, ars, [0, rows], [0],
                              [[0] for _ in range(lay.S)], rows, t.device, force_torch))
        r0 += rows
    return sz, mat, [a[:sum(send_bytes[s])] for s, a in enumerate(arenas)], outs


def _check_roundtrip(rows, dest, outs):
    for d in range(W):
        want = [_canon(r) for r, dd in zip(rows, dest) if dd == d]
        assert [_canon(r) for r in outs[d].to_pylist()] == want, d


def test_torch_pack_roundtrip_cpu():
    rows = _rows(3000)
    t = Table.from_pylist(rows, SCHEMA)
    dest = [random.Random(7).randrange(W) for _ in rows]
    _sz, _mat, _ar, outs = _roundtrip(t, torch.tensor(dest), True)
    _check_roundtrip(rows, dest, outs)


def _coalesced(t, dest, force_torch):
    """Coalesced pack (every string leaf in one destination-major buffer) → per-destination unpack, with the
    receive-side byte bases computed by ``coalesced_bytes`` exactly as ``shuffle_table`` does."""
    lay = PK.Layout(t)
    sizes, state = PK.plan(lay, dest, W, force_torch)
    sz = sizes.tolist()
    send_rows = [r[0] for r in sz]
    send_bytes = [[r[1 + s] for r in sz] for s in range(lay.S)]
    mat, (buf,) = PK.scatter(lay, state, send_rows, send_bytes, coalesce=True)
    per_rank, base = PK.coalesced_bytes(send_bytes)
    assert sum(per_rank) <= buf.shape[0]
    outs, r0 = [], 0
    for d in range(W):
        rows = send_rows[d]
        lo = sum(per_rank[:d])
        piece = torch.zeros(per_rank[d] + 16, dtype=torch.uint8, device=t.device)
        piece[:per_rank[d]] = buf[lo:lo + per_rank[d]]
        outs.append(PK.unpack(lay.names, lay.spec, lay.meta(), mat[r0:r0 + rows], [piece] * lay.S, [0, rows], [0],
                              [[base[s][d] - lo] for s in range(lay.S)], rows, t.device, force_torch))
        r0 += rows
    return buf[:sum(per_rank)], outs


def test_coalesced_bytes_layout():
    per_rank, base = PK.coalesced_bytes([[3, 0, 5], [1, 2, 0]])       # 2 leaves x 3 ranks
    assert per_rank == [4, 2, 5]
    assert base == [[0, 4, 6], [3, 4, 11]]


def test_torch_coalesced_roundtrip_cpu():
    rows = _rows(2000)
    t = Table.from_pylist(rows, SCHEMA)
    dest = [random.Random(5).randrange(W) for _ in rows]
    dest[:50] = [1] * 50
    dest = [d if d != 3 else 4 for d in dest]            # destination 3 receives nothing
    _buf, outs = _coalesced(t, torch.tensor(dest), True)
    _check_roundtrip(rows, dest, outs)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 777, 20000])
def test_device_coalesced_pack_matches_torch(gpu, n):
    rows = _rows(n, seed=9)
    rnd = random.Random(13)
    dest = [rnd.randrange(W) for _ in rows]
    t = Table.from_pylist(rows, SCHEMA, gpu)
    dt = torch.tensor(dest, dtype=torch.int64, device=gpu)
    buf_d, outs_d = _coalesced(t, dt, False)
    buf_t, outs_t = _coalesced(t, dt, True)
    assert torch.equal(buf_d.cpu(), buf_t.cpu())
    _check_roundtrip(rows, dest, outs_d)
    _check_roundtrip(rows, dest, outs_t)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 777, 20000])
def test_device_pack_matches_torch(gpu, n):
    rows = _rows(n)
    rnd = random.Random(11)
    dest = [rnd.randrange(W) for _ in rows]
    if n > 100:
        dest[: n // 3] = [2] * (n // 3)                  # skew: one destination takes a third of the rows
    t = Table.from_pylist(rows, SCHEMA, gpu)
    dt = torch.tensor(dest, dtype=torch.int64, device=gpu)
    assert PK.device_ok(PK.Layout(t), W)
    sz_d, mat_d, ar_d, outs_d = _roundtrip(t, dt, False)
    sz_t, mat_t, ar_t, outs_t = _roundtrip(t, dt, True)
    assert sz_d == sz_t
    assert torch.equal(mat_d.cpu(), mat_t.cpu())
    for a, b in zip(ar_d, ar_t):
        assert torch.equal(a.cpu(), b.cpu())
    _check_roundtrip(rows, dest, outs_d)
    _check_roundtrip(rows, dest, outs_t)


@pytest.mark.gpu
def test_device_pack_plain_and_narrow_types(gpu):
    """No destination (the all-gather / broadcast pack), int32 / int16 / uint8 data and a table of constants."""
    from dxa.engine.column import ConstColumn, PrimColumn
    n = 5000
    i32 = torch.arange(n, dtype=torch.int32, device=gpu) * 7 - 100
    i16 = (torch.arange(n, device=gpu) % 300 - 150).to(torch.int16)
    u8 = (torch.arange(n, device=gpu) % 251).to(torch.uint8)
    valid = torch.arange(n, device=gpu) % 3 != 0
    t = Table(["a", "b", "c", "k"], [PrimColumn("int", i32, valid), PrimColumn("short", i16),
                                     PrimColumn("byte", u8), ConstColumn("x", "string", n, gpu)], n, gpu)
    for force in (False, True):
        lay = PK.Layout(t)
        sizes, state = PK.plan(lay, None, 1, force)
        assert sizes.tolist() == [[n]]
        mat, arenas = PK.scatter(lay, state, [n], [])
        out = PK.unpack(lay.names, lay.spec, lay.meta(), mat, arenas, [0, n], [0], [], n, gpu, force)
        assert out.to_pylist() == t.to_pylist()


@pytest.mark.gpu
def test_exchange_launch_count(gpu):
    """The device send side is three launches (plan: histogram + scan; scatter) whatever the column count."""
    rows = _rows(4000)
    t = Table.from_pylist(rows, SCHEMA, gpu)
    dt = torch.tensor([i % W for i in range(len(rows))], dtype=torch.int64, device=gpu)
    lay = PK.Layout(t)
    for c in t.columns:                 # materialise lazily built inputs outside the counted region
        pass
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        sizes, state = PK.plan(lay, dt, W)
        sz = sizes.tolist()
        PK.scatter(lay, state, [r[0] for r in sz], [[r[1 + s] for r in sz] for s in range(lay.S)])
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    kernels = [n for n in names if "xchg" in n]
    assert len(kernels) == 3, names


@pytest.mark.gpu
def test_send_side_is_three_launches():
    """The shuffle's send side — partition histogram, scan (with the validity flags written into the size rows) and
    the scatter into the packed matrix + string arenas — is three kernel launches whatever the table's width."""
    from launch_count import count_launches
    from dxa.engine.column import PrimColumn, strings_from_pylist
    dev = torch.device("cuda")
    n = 100_000
    cols = [PrimColumn("long", torch.arange(n, device=dev) * k) for k in range(12)]
    cols.append(PrimColumn("double", torch.rand(n, dtype=torch.float64, device=dev), torch.rand(n, device=dev) > 0.1))
    cols.append(strings_from_pylist([f"s{i % 977}" for i in range(n)], dev))
    t = Table([f"c{i}" for i in range(len(cols))], cols, n, dev)
    dest = torch.randint(0, 8, (n,), device=dev)
    torch.cuda.synchronize()
    lay = PK.Layout(t)
    with count_launches() as log:
        ext, state = PK.plan(lay, dest, 8, extra=lay.flags())
    sz = ext.tolist()                                       # the exchange's one host read-back
    with count_launches() as log2:
        PK.scatter(lay, state, [r[0] for r in sz], [[r[1 + s] for r in sz] for s in range(lay.S)])
    # dxa_xchg_plan = histogram + scan kernels
    assert log == ["dxa_xchg_plan"] and log2 == ["dxa_xchg_scatter"], (log, log2)


def test_crc_placement_rule():
    """check.crcs=auto (dxa.parallel.affinity.crc_placement): host while the planner threads keep up with the ingest
    and the node's host memory budget covers every local rank's CRC + DMA reads; the same answer on every local
    rank (lockstep ranks run at the slowest one's pace); device otherwise (profiles/round6/host8/README.md)."""
    from dxa.parallel.affinity import crc_placement
    assert crc_placement(0, 1, 16) == "host"
    assert [crc_placement(r, 8, 16) for r in range(8)] == ["host"] * 8          # 8 x 2 x 57 = 912 <= 1000 GB/s
    assert [crc_placement(r, 8, 16, budget_gbs=600) for r in range(8)] == ["device"] * 8
    assert crc_placement(0, 1, 4) == "device"                                    # 4 x 9 GB/s < 57 GB/s
