"""Differential tests: every hand-written HIP kernel vs the plain CPU/PyTorch reference of the same op."""
import json
import random

import pytest
import torch

from dxa.engine.column import PrimColumn, Table, column_from_pylist, strings_from_pylist
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql
from dxa.engine.serialize import table_to_json_lines
from dxa.engine.types import schema_from_json
from dxa.ops import groupby as G
from dxa.ops import join as J
from dxa.ops import strings as S
from dxa.ops.hashing import hash_columns
from dxa.ops.jsonparse import ParsePlan, frame_records, parse

pytestmark = pytest.mark.gpu

SCHEMA = schema_from_json(json.dumps({"type": "struct", "fields": [
    {"name": "deviceDetails", "type": {"type": "struct", "fields": [
        {"name": "deviceId", "type": "long"}, {"name": "deviceType", "type": "string"},
        {"name": "homeId", "type": "long"}, {"name": "status", "type": "long"},
        {"name": "temperature", "type": "double"}, {"name": "ok", "type": "boolean"},
        {"name": "eventTime", "type": "timestamp"}, {"name": "tags", "type": {"type": "array", "elementType": "string",
                                                                             "containsNull": True}}]}},
    {"name": "note", "type": "string"}, {"name": "small", "type": "integer"}]}))


def _records(n, seed=0):
    rnd = random.Random(seed)
    out = []
    for i in range(n):
        d = {"deviceId": rnd.randint(1, 40), "deviceType": rnd.choice(["DoorLock", "WindowLock", "Heating", "Gar\"age"]),
             "homeId": rnd.choice([150, 32, 25, 81]), "status": rnd.randint(0, 1),
             "temperature": round(rnd.uniform(-40, 120), rnd.randint(0, 6)), "ok": rnd.random() < 0.5,
             "eventTime": rnd.choice(["2019-02-28T22:45:00Z", "2019-03-01 01:02:03.5", 1551394800]),
             "tags": ["a", "b"][:rnd.randint(0, 2)]}
        if rnd.random() < 0.1:
            d["deviceId"] = None
        if rnd.random() < 0.05:
            d["status"] = "oops"          # type mismatch → null
        if rnd.random() < 0.05:
            del d["temperature"]
        rec = {"deviceDetails": d, "note": rnd.choice(["hello", "tab\there", "unié", "q\"uote", ""]),
               "small": rnd.choice([1, 2**40, -5])}
        s = json.dumps(rec, ensure_ascii=rnd.random() < 0.5)
        if rnd.random() < 0.03:
            s = s[: len(s) // 2]             # malformed
        out.append(s.encode())
    return out


def _parse_both(gpu, n=3000, seed=0):
    recs = _records(n, seed)
    plan = ParsePlan(SCHEMA)
    b, o = frame_records(recs)
    cpu_raw, cpu_ok = parse(b, o, plan)
    bg, og = frame_records(recs, device=gpu)
    gpu_raw, gpu_ok = parse(bg, og, plan)
    return cpu_raw, cpu_ok, gpu_raw, gpu_ok


def test_json_parse_matches_cpu(gpu):
    cpu_raw, cpu_ok, gpu_raw, gpu_ok = _parse_both(gpu)
    assert torch.equal(cpu_ok, gpu_ok.cpu())
    a, b = cpu_raw.to_pylist(), gpu_raw.to_pylist()
    for x, y in zip(a, b):
        if x is not None and y is not None:
            # raw JSON columns may differ in whitespace only
            x["deviceDetails"] and x["deviceDetails"].pop("tags", None)
            y["deviceDetails"] and y["deviceDetails"].pop("tags", None)
        assert x == y


def test_hash_matches_cpu(gpu):
    ints = column_from_pylist([1, None, -7, 2**62, 0], "long")
    dbl = column_from_pylist([0.0, -0.0, 1.5, None, float("nan")], "double")
    st = strings_from_pylist(["", "a", None, "hello world, this is long", "x" * 17], "cpu")
    h_cpu = hash_columns([ints, dbl, st])
    h_gpu = hash_columns([ints.to(gpu), dbl.to(gpu), st.to(gpu)])
    assert torch.equal(h_cpu, h_gpu.cpu())


@pytest.mark.parametrize("ngroups", [3, 500, 20000])
def test_groupby_matches_cpu(gpu, ngroups):
    rnd = random.Random(ngroups)
    n = 50000
    k1 = [rnd.randrange(ngroups) for _ in range(n)]
    k2 = [f"t{x % 7}" for x in k1]
    v = [None if rnd.random() < 0.02 else rnd.uniform(-5, 5) for _ in range(n)]
    iv = [rnd.randint(-100, 100) for _ in range(n)]
    cols = [column_from_pylist(k1, "long"), strings_from_pylist(k2, "cpu")]
    vc, ic = column_from_pylist(v, "double"), column_from_pylist(iv, "long")
    gc = G.group_rows(cols)
    gg = G.group_rows([c.to(gpu) for c in cols])
    assert gc.ngroups == gg.ngroups
    assert torch.equal(gc.rep, gg.rep.cpu())
    assert torch.equal(gc.gid.to(torch.int64), gg.gid.cpu().to(torch.int64))
    for func, col in [("sum", vc), ("min", vc), ("max", vc), ("avg", vc), ("count", vc), ("sum", ic), ("min", ic),
                      ("max", ic), ("count_star", None)]:
        a = G.aggregate(gc, col, func, n).to_pylist()
        b = G.aggregate(gg, None if col is None else col.to(gpu), func, n).to_pylist()
        for x, y in zip(a, b):
            if isinstance(x, float):
                assert y == pytest.approx(x, rel=1e-9, abs=1e-9)
            else:
                assert x == y, func


@pytest.mark.parametrize("ngroups", [5000, 30000])
def test_fused_aggregates_match_cpu(gpu, ngroups):
    """aggregate_many (one fused pass, [group][slot] lines per atomic kind) against the CPU aggregates: nulls,
    negative / mixed-sign doubles (ordered-bits MIN/MAX), ints, booleans, shared validity masks, >8 slots per kind."""
    rnd = random.Random(ngroups)
    n = 60000
    k = [rnd.randrange(ngroups) for _ in range(n)]
    v = [None if rnd.random() < 0.03 else rnd.uniform(-1e6, 1e6) * rnd.choice([1, 1e-9]) for _ in range(n)]
    w = [rnd.choice([-0.5, -3.25, 7.0, 1e300, -1e-300]) for _ in range(n)]
    iv = [None if rnd.random() < 0.01 else rnd.randint(-2**62, 2**62) for _ in range(n)]
    bv = [rnd.random() < 0.5 for _ in range(n)]
    kc = column_from_pylist(k, "long")
    cols = {"v": column_from_pylist(v, "double"), "w": column_from_pylist(w, "double"),
            "i": column_from_pylist(iv, "long"), "b": column_from_pylist(bv, "boolean")}
    reqs = [(None, "count_star")]
    for nm in ("v", "w", "i"):
        reqs += [(nm, f) for f in ("sum", "min", "max", "avg", "count")]
    reqs += [("b", "min"), ("b", "max"), ("v", "sum"), ("w", "max")] + [("w", "sum")] * 9
    gc = G.group_rows([kc])
    gg = G.group_rows([kc.to(gpu)])
    got = G.aggregate_many(gg, [(None if c is None else cols[c].to(gpu), f) for c, f in reqs], n)
    for (c, f), col in zip(reqs, got):
        want = G.aggregate(gc, None if c is None else cols[c], f, n).to_pylist()
        have = col.to_pylist()
        assert len(want) == len(have) == gc.ngroups
        for x, y in zip(want, have):
            if isinstance(x, float):
                assert y == pytest.approx(x, rel=1e-9, abs=1e-6), (c, f)
            else:
                assert x == y, (c, f)


@pytest.mark.parametrize("kind", ["inner", "left", "semi", "anti", "full"])
def test_join_matches_cpu(gpu, kind):
    rnd = random.Random(1)
    lk = [rnd.randrange(300) for _ in range(4000)]
    rk = [rnd.randrange(400) for _ in range(900)] + [None]
    lc, rc = [column_from_pylist(lk, "long")], [column_from_pylist(rk, "long")]
    a = J.hash_join(lc, rc, kind)
    b = J.hash_join([c.to(gpu) for c in lc], [c.to(gpu) for c in rc], kind)
    pa = sorted(zip(a[0].tolist(), a[1].tolist()))
    pb = sorted(zip(b[0].cpu().tolist(), b[1].cpu().tolist()))
    assert pa == pb


@pytest.mark.parametrize("kind", ["inner", "left", "semi", "anti"])
@pytest.mark.parametrize("unique", [True, False])
def test_cached_build_join_matches_cpu(gpu, kind, unique):
    """A cached build side (stream–static join): a keyed table takes the positional one-candidate path
    (join.py _unique_join), a table with duplicate keys the count / write path; both against the CPU join."""
    rnd = random.Random(2)
    lk = [rnd.randrange(500) for _ in range(3000)] + [None]
    rk = (rnd.sample(range(400), 350) if unique else [rnd.randrange(400) for _ in range(700)]) + [None]
    lc = [column_from_pylist(lk, "long"), strings_from_pylist([None if k is None else f"s{k}" for k in lk], "cpu")]
    rc = [column_from_pylist(rk, "long"), strings_from_pylist([None if k is None else f"s{k}" for k in rk], "cpu")]
    a = J.hash_join(lc, rc, kind)
    glc, grc = [c.to(gpu) for c in lc], [c.to(gpu) for c in rc]
    built = J.build_side(grc)
    for _ in range(2):                              # the multiplicity is read on first use, then reused
        b = J.hash_join(glc, grc, kind, built)
        assert (built.max_mult <= 1) == unique
        assert sorted(zip(a[0].tolist(), a[1].tolist())) == sorted(zip(b[0].cpu().tolist(), b[1].cpu().tolist()))


def test_string_ops_match_cpu(gpu):
    vals = ["DoorLock", "Door", "", "Heating", None, "doorlock", "Zebra", "DoorLocks"]
    c = strings_from_pylist(vals, "cpu")
    g = c.to(gpu)
    for op in ["=", "!=", "<", "<=", ">", ">=", "startswith", "endswith", "contains"]:
        assert torch.equal(S.cmp_literal(c, "DoorLock", op), S.cmp_literal(g, "DoorLock", op).cpu()), op
    assert S.case_map(c, True).to_pylist() == S.case_map(g, True).to_pylist()
    ints = column_from_pylist([0, -1, 123456789012, None, 7], "long")
    assert S.from_int64(ints.data, ints.valid).to_pylist() == S.from_int64(ints.data.to(gpu),
                                                                          ints.valid.to(gpu)).to_pylist()
    parts = ["n: ", c, "/", S.from_int64(column_from_pylist(list(range(8)), "long").data, None)]
    gparts = ["n: ", g, "/", S.from_int64(column_from_pylist(list(range(8)), "long").data.to(gpu), None)]
    assert S.concat_strings(parts, 8, "cpu").to_pylist() == S.concat_strings(gparts, 8, gpu).to_pylist()
    ts = strings_from_pylist(["2019-02-28 22:45:00", "2019-02-28T22:45:00Z", "02/28/2019 22:45:00", "bad",
                              "2019-02-28 22:45:00.123", None, "1551394800000", "2019-2-8 1:2:3"], "cpu")
    assert S.to_timestamp(ts).to_pylist() == S.to_timestamp(ts.to(gpu)).to_pylist()
    # fixed-width fast path (aligned-word reads): every arena alignment, 0-10 fraction digits, near misses
    forms = ["2019-02-28 22:45:00", "2019-02-28T22:45:00Z", "2019-02-28T22:45:00.5Z", "2019-13-01 00:00:00",
             "2019-02-28 24:00:00", "2019-02-28X22:45:00", "2019-02-28 22:45:0a", "2019-02-28 22:45:00.",
             "2019-02-28T22:45:00", "2019-02-28 22:45:00Z", "0001-01-01 00:00:00", "9999-12-31T23:59:59Z"]
    forms += ["2019-02-28 22:45:00." + "123456789a"[:k] for k in range(1, 11)]
    vals = []
    for k, f in enumerate(forms * 8):
        vals += ["y" * (k % 8), f]
    ts = strings_from_pylist(vals, "cpu")
    assert S.to_timestamp(ts).to_pylist() == S.to_timestamp(ts.to(gpu)).to_pylist()


def test_full_query_matches_cpu(gpu):
    cpu_raw, _, gpu_raw, _ = _parse_both(gpu, n=5000, seed=3)
    outs = []
    for raw in (cpu_raw, gpu_raw):
        cat = Catalog()
        ctx = EvalContext(now_us=1551394800_000000)
        base = Catalog()
        base.register("T", Table(["Raw"], [raw]))
        cat.register("DataXProcessedInput", run_sql("SELECT Raw.*, current_timestamp() AS eventTimeStamp FROM T",
                                                     base, ctx))
        q1 = run_sql("SELECT deviceDetails.deviceId, deviceDetails.deviceType, deviceDetails.homeId, "
                     "MAX(deviceDetails.eventTime) AS MaxEventTime, MIN(deviceDetails.status) AS MinReading, "
                     "AVG(deviceDetails.temperature) AS t, COUNT(*) AS c FROM DataXProcessedInput "
                     "GROUP BY deviceId, deviceType, homeId ORDER BY deviceId, deviceType, homeId", cat, ctx)
        q2 = run_sql("SELECT deviceDetails.deviceId AS id, CONCAT('Door: ', deviceDetails.deviceType, ' at ', "
                     "deviceDetails.homeId) AS p FROM DataXProcessedInput WHERE deviceDetails.homeId = 150 AND "
                     "deviceDetails.deviceType = 'DoorLock' AND deviceDetails.status = 0", cat, ctx)
        outs.append((table_to_json_lines(q1), table_to_json_lines(q2)))
    for a, b in zip(outs[0], outs[1]):
        assert len(a) == len(b)
        for x, y in zip(a, b):
            x, y = json.loads(x), json.loads(y)
            assert x.keys() == y.keys()
            for k in x:
                if isinstance(x[k], float):
                    assert y[k] == pytest.approx(x[k], rel=1e-12)   # float sums: atomic order differs
                else:
                    assert x[k] == y[k]


def _serializer_table(device):
    from dxa.engine.column import ArrayColumn, ConstColumn, StructColumn
    from dxa.engine.types import MapType
    rnd = random.Random(5)
    n = 3000
    longs = column_from_pylist([None if rnd.random() < 0.1 else rnd.randint(-2**62, 2**62) for _ in range(n)], "long")
    specials = [0.0, -0.0, 1e7, 9999999.999, 1e-3, 0.00099, 5e-324, 1.7976931348623157e308, 100.0, 0.1, 1e22,
                float("inf"), float("-inf"), float("nan")]
    dbl = [rnd.choice(specials) if rnd.random() < 0.2 else rnd.uniform(-1, 1) * 10 ** rnd.randint(-20, 20)
           for _ in range(n)]
    dbls = column_from_pylist([None if rnd.random() < 0.05 else d for d in dbl], "double")
    strs = strings_from_pylist([None if rnd.random() < 0.1 else rnd.choice(["plain", 'q"uote', "back\\slash",
                                "tab\tnl\n", "ctl\x01\x1f", "unié", ""]) for _ in range(n)], "cpu")
    bools = column_from_pylist([None if rnd.random() < 0.1 else rnd.random() < 0.5 for _ in range(n)], "boolean")
    ts = column_from_pylist([None if rnd.random() < 0.1 else rnd.randint(-10**15, 4 * 10**15) for _ in range(n)],
                            "timestamp")
    struct = StructColumn(["a", "b"], [longs, strs], n, None)
    mp = StructColumn(["k1", "k2"], [strs, dbls], n, None, True, MapType("string", "string"))
    arr = ArrayColumn([longs, dbls], n, None, True)
    const = ConstColumn("x\"y", "string", n, "cpu")
    t = Table(["l", "d", "s", "b", "t", "st", "m", "arr", "c", "nul"],
              [longs, dbls, strs, bools, ts, struct, mp, arr, const, ConstColumn(None, "string", n, "cpu")], n)
    return t


def test_gpu_serializer_matches_host(gpu, monkeypatch):
    from dxa.ops import serialize as ser
    t = _serializer_table("cpu")
    host = ser.Staged(t).render()                     # CPU table → host serializer
    gt = t.to(gpu)
    st = ser.Staged(gt)
    assert st.gpu
    dev = st.render()
    assert dev.blob == host.blob
    assert dev.lens.tolist() == host.lens.tolist()


def test_gpu_serializer_render_group_matches_host(gpu):
    """Several output tables of a batch (different schemas and row counts, one of 300 rows so a workgroup would
    straddle segments if the kernel did not pad them) render in one launch pair; each slice equals the table's own
    host rendering."""
    from dxa.ops import serialize as ser
    t = _serializer_table("cpu")
    parts = [t, t.take(torch.arange(0, 300)), Table(["s", "l"], [t.columns[2], t.columns[0]], t.length),
             t.take(torch.arange(1000, 1257))]
    hosts = [ser.Staged(p).render() for p in parts]
    staged = [ser.Staged(p.to(gpu)) for p in parts]
    ser.link_render_groups(staged)
    assert staged[0].group is not None and all(s.group is staged[0].group for s in staged)
    before = ser.STATS["launch_pairs"]
    for k in (2, 0, 3, 1):                               # any member may trigger the render
        dev = staged[k].render()
        assert dev.blob == hosts[k].blob, k
        assert dev.lens.tolist() == hosts[k].lens.tolist()
    assert ser.STATS["launch_pairs"] == before + 1


def test_gpu_java_double_matches_host(gpu):
    import ctypes
    import numpy as np
    from dxa.ops import native as N
    from dxa.ops.serialize import java_double
    rng = np.random.default_rng(3)
    vals = np.concatenate([rng.standard_normal(50000) * 10.0 ** rng.integers(-300, 300, 50000),
                           rng.integers(0, 2**63, 50000, dtype=np.int64).view(np.float64)])
    vals = vals[np.isfinite(vals)]
    d = torch.from_numpy(vals).to(gpu)
    out = torch.zeros(32 * len(vals), dtype=torch.uint8, device=gpu)
    lens = torch.zeros(len(vals), dtype=torch.int32, device=gpu)
    N.call("dxa_java_double_dev", N.ptr(d), len(vals), N.ptr(out), N.ptr(lens), N.stream_handle(gpu))
    o, l = out.cpu().numpy(), lens.cpu().numpy()
    bad = [v for i, v in enumerate(vals) if bytes(o[32 * i:32 * i + l[i]]).decode() != java_double(float(v))]
    assert not bad, bad[:5]


def test_byte_map_kernel_matches_cpu(gpu):
    from dxa.udf.api import apply_byte_map
    from dxa.udf.samples import RemoveInvalidChars
    table = RemoveInvalidChars().byte_map()
    for n in (0, 5, 16, 1000, 1 << 20, (1 << 20) + 7):
        buf = torch.randint(0, 256, (n,), dtype=torch.uint8)
        want = apply_byte_map(buf, table)
        got = apply_byte_map(buf.to(gpu), table).cpu()
        assert torch.equal(got, want), n


def test_json_parse_key_order_speculation(gpu):
    """Keys out of schema order, unknown keys, escaped key text and prefix-sharing names must all resolve exactly
    like the CPU reference (the kernel predicts the next key and falls back to hashing on a miss)."""
    rnd = random.Random(11)
    schema = schema_from_json(json.dumps({"type": "struct", "fields": [
        {"name": "a", "type": "long"}, {"name": "ab", "type": "string"}, {"name": "abcdefgh", "type": "double"},
        {"name": "abcdefghi", "type": "long"},
        {"name": "s", "type": {"type": "struct", "fields": [{"name": "x", "type": "long"},
                                                             {"name": "y", "type": "string"}]}}]}))
    recs = []
    for i in range(4000):
        items = [("a", i), ("ab", f"v{i}"), ("abcdefgh", i * 0.5), ("abcdefghi", -i),
                 ("s", {"y": "q", "x": i}), ("zz_unknown", [1, 2])]
        if rnd.random() < 0.5:
            rnd.shuffle(items)
        d = "{" + ",".join(json.dumps(k) + ":" + json.dumps(v) for k, v in items) + "}"
        if rnd.random() < 0.1:
            d = d.replace('"ab":', '"a\\u0062":')          # escaped key text
        recs.append(d.encode())
    plan = ParsePlan(schema)
    b, o = frame_records(recs)
    cpu_raw, cpu_ok = parse(b, o, plan)
    bg, og = frame_records(recs, device=gpu)
    gpu_raw, gpu_ok = parse(bg, og, plan)
    assert torch.equal(cpu_ok.cpu(), gpu_ok.cpu())
    assert cpu_raw.to_pylist() == gpu_raw.to_pylist()


def _gen_programs():
    from dxa.models import iot
    from dxa.simulate.datagen import compile_simulated, compile_spark
    spark = schema_from_json(json.dumps({"type": "struct", "fields": [
        {"name": "id", "type": "long", "nullable": True, "metadata": {"minValue": -5, "maxValue": 10 ** 12}},
        {"name": "name", "type": "string", "nullable": True, "metadata": {"maxLength": 19}},
        {"name": "kind", "type": "string", "nullable": False, "metadata": {"allowedValues": ["a", "bb", "a\"c", ""]}},
        {"name": "v", "type": "double", "nullable": True, "metadata": {"minValue": -1e6, "maxValue": 1e6,
                                                                        "decimals": 3}},
        {"name": "w", "type": "double", "nullable": False, "metadata": {"minValue": 0, "maxValue": 1, "decimals": 0}},
        {"name": "ok", "type": "boolean", "nullable": True, "metadata": {}},
        {"name": "t", "type": "long", "nullable": False, "metadata": {"useCurrentTimeMillis": True}},
        {"name": "ts", "type": "string", "nullable": False, "metadata": {"datetimeStringFormat": "MM/dd/yyyy HH:mm:ss"}},
        {"name": "nested", "type": {"type": "struct", "fields": [
            {"name": "x", "type": "integer", "nullable": True, "metadata": {}},
            {"name": "arr", "type": {"type": "array", "elementType": "double", "containsNull": True},
             "nullable": True, "metadata": {"maxLength": 3}}]}, "nullable": True, "metadata": {}}]}))
    sim = compile_simulated([
        {"name": "deviceId", "type": "long", "minRange": 1, "maxRange": 1000},
        {"name": "temp", "type": "double", "minRange": -40.5, "maxRange": 120.25},
        {"name": "kind", "type": "string", "valueList": ["DoorLock", "WindowLock", "Heating"]},
        {"name": "when", "type": "datetime", "datetimeStringFormat": "yyyy-MM-ddTHH:mm:ssZ", "utcAddSeconds": -30},
        {"name": "const", "type": "string", "value": "fixed"},
        {"name": "s", "type": "struct", "properties": [
            {"name": "arr", "type": "array", "minRange": 0, "maxRange": 1, "length": 4, "castAsString": True}]}])
    return {"iot": iot.program(), "iot_nl": iot.program(newline=True), "spark": compile_spark(spark),
            "simulated": sim}


@pytest.mark.parametrize("name", ["iot", "iot_nl", "spark", "simulated"])
def test_datagen_matches_cpu(gpu, name):
    """The GPU event generator renders byte-for-byte what the host reference renders (word-packed emitter: records
    start at every alignment, so the first/last partial words of each record are exercised)."""
    from dxa.simulate.datagen import generate, generate_cpu
    prog = _gen_programs()[name]
    for seed, row0, n, step in ((1, 0, 2000, 0), (77, 123457, 1531, 997), (2**63 + 5, 10 ** 9, 700, 1000)):
        base = 1_700_000_000_123
        gb, go = generate(prog, n, gpu, seed=seed, row0=row0, base_ms=base, step_us=step)
        cb, co = generate_cpu(prog, n, seed=seed, row0=row0, base_ms=base, step_us=step)
        assert go.cpu().tolist() == co.tolist()
        total = int(co[-1])
        assert bytes(gb[:total].cpu().numpy()) == bytes(cb[:total].numpy())
        assert not gb[total:].cpu().any()


@pytest.mark.parametrize("name", ["iot", "spark", "simulated"])
def test_datagen_slotted_matches_cpu(gpu, name):
    """The one-pass slotted generator (fixed-size 16-B aligned slots, no length pass) renders the host reference's
    records byte for byte; slot starts and record ends describe them, and the JSON parser reads the gapped batch to
    the same columns as the packed one."""
    from dxa.simulate.datagen import generate_cpu, generate_slotted
    prog = _gen_programs()[name]
    for seed, row0, n, step in ((1, 0, 2000, 0), (2**63 + 5, 10 ** 9, 700, 1000)):
        base = 1_700_000_000_123
        gb, go, ge = generate_slotted(prog, n, gpu, seed=seed, row0=row0, base_ms=base, step_us=step)
        cb, co = generate_cpu(prog, n, seed=seed, row0=row0, base_ms=base, step_us=step)
        go, ge, gbh = go.cpu().tolist(), ge.cpu().tolist(), bytes(gb.cpu().numpy())
        stride = go[1] - go[0]
        assert stride % 16 == 0 and stride >= prog.max_len()
        cbh, co = bytes(cb.numpy()), co.tolist()
        for i in range(n):
            assert go[i] == i * stride
            assert gbh[go[i]:ge[i]] == cbh[co[i]:co[i + 1]], i
        assert go[n] == n * stride and not any(gbh[n * stride:])


def test_order_by_and_string_ordering_match_cpu(gpu):
    """ORDER BY over strings (device dense ranks), doubles with NaN/-0.0, nulls first/last, DESC — one device radix
    argsort — and string < / >= predicates (device compare kernel) give the CPU engine's rows in the same order."""
    rnd = random.Random(11)
    n = 20000
    words = ["", "a", "ab", "abcdefghij", "abcdefghik", "Zeta", "éclair", "door lock", "DoorLock"]
    s1 = [None if rnd.random() < 0.08 else rnd.choice(words) + rnd.choice(["", "x", "yy"]) for _ in range(n)]
    s2 = [rnd.choice(words) for _ in range(n)]
    d = [None if rnd.random() < 0.05 else rnd.choice([float("nan"), -0.0, 0.0, 1.5, -2.5, rnd.uniform(-9, 9)])
         for _ in range(n)]
    k = [rnd.randint(0, 50) for _ in range(n)]
    outs = []
    for dev in ("cpu", gpu):
        t = Table(["s1", "s2", "d", "k", "i"],
                  [strings_from_pylist(s1, dev), strings_from_pylist(s2, dev), column_from_pylist(d, "double", dev),
                   column_from_pylist(k, "long", dev), column_from_pylist(list(range(n)), "long", dev)], n)
        cat = Catalog()
        cat.register("T", t)
        ctx = EvalContext(now_us=0)
        q1 = run_sql("SELECT i FROM T ORDER BY s1 DESC NULLS LAST, d, k DESC, i", cat, ctx)
        q2 = run_sql("SELECT i FROM T WHERE s1 < s2 OR s2 >= 'abcdefghij' ORDER BY i", cat, ctx)
        q3 = run_sql("SELECT i, RANK() OVER (PARTITION BY s2 ORDER BY d DESC, s1) AS r FROM T ORDER BY i", cat, ctx)
        outs.append([table_to_json_lines(q) for q in (q1, q2, q3)])
    for a, b in zip(outs[0], outs[1]):
        assert a == b


def test_multi_column_take_matches_cpu(gpu):
    """Table.take on the GPU gathers every leaf (data, validity, string views, nested validity) in one
    multi-column launch; rows must equal the CPU take, negative indices included."""
    t_cpu = _serializer_table("cpu")
    t_gpu = t_cpu.to(gpu)
    g = torch.Generator().manual_seed(4)
    idx = torch.randint(-t_cpu.length, t_cpu.length, (7001,), generator=g)
    a = t_cpu.take(idx).to_pylist()
    b = t_gpu.take(idx.to(gpu)).to_pylist()
    assert json.dumps(a, default=str) == json.dumps(b, default=str)
    assert t_gpu.take(torch.empty(0, dtype=torch.int64, device=gpu)).length == 0


def test_string_gather_lengths_and_alignments(gpu):
    """Compaction (lane-per-string gather with unaligned 8/4/2/1-byte copies; > 128-byte strings by the whole
    wave) against the CPU gather: every length 0..300, every source alignment, nulls, views in random order."""
    rnd = random.Random(7)
    words = []
    for k in range(2000):
        L = k % 301 if k % 7 else rnd.choice([0, 1, 7, 8, 9, 129, 300, 1000])
        words.append("".join(chr(97 + rnd.randint(0, 25)) for _ in range(L)) if rnd.random() > 0.05 else None)
    c = strings_from_pylist(words, "cpu")
    # views in shuffled order into the same arena (non-contiguous, unaligned starts)
    perm = torch.tensor(rnd.sample(range(len(words)), len(words)), dtype=torch.int64)
    view = c.take(perm)
    want = [words[i] for i in perm.tolist()]
    assert S.compact(view).to_pylist() == want
    gv = c.to(gpu).take(perm.to(gpu))
    got = S.compact(gv)
    assert got.to_pylist() == want
    assert S.compact_known(gv, int(gv.lens.to(torch.int64).sum())).to_pylist() == want
    assert [x.to_pylist() for x in S.compact_many([gv, gv.take(torch.arange(5, device=gpu))])] == [want, want[:5]]


def test_sdma_device_to_host_copy(gpu):
    """dxa_copy_sdma (ROCr async copy on a DMA engine) copies a device range into pinned host memory."""
    from dxa.ops import native as N
    src = torch.randint(0, 256, (3_000_001,), dtype=torch.uint8, device=gpu)
    host = torch.empty(3_000_001, dtype=torch.uint8, pin_memory=True)
    torch.cuda.synchronize()
    assert N.lib().dxa_copy_sdma(host.data_ptr(), src.data_ptr() + 1, 3_000_000) == 0
    assert torch.equal(host[:3_000_000], src[1:].cpu())


def test_parse_ahead_matches_parse(gpu):
    """jsonparse.parse_async (Processor.prepare's parse-ahead) = parse, including the null-mask decisions."""
    from dxa.ops.jsonparse import parse_async
    recs = _records(4000, seed=9)
    plan = ParsePlan(SCHEMA)
    bg, og = frame_records(recs, device=gpu)
    a, ok_a = parse(bg, og, plan)
    bg, og = frame_records(recs, device=gpu)                 # a parse un-escapes strings in place: fresh bytes
    pend = parse_async(bg, og, plan)
    filler = torch.randn(1 << 22, device=gpu).sort()        # later work on the stream does not disturb the result
    b, ok_b = pend.result()
    assert pend.result()[0] is b
    del filler
    assert torch.equal(ok_a, ok_b)
    assert a.to_pylist() == b.to_pylist()


@pytest.mark.parametrize("variant", ["groupby", "window"])
def test_processor_prepare_same_outputs(gpu, variant, tmp_path):
    """A Processor fed prepared batches (parse queued one batch ahead) produces the same views as one that parses
    inside process_batch."""
    from dxa.engine.processor import Processor, RawBatch
    from dxa.models import iot
    from dxa.simulate.datagen import generate
    prog = iot.program()
    n, t0 = 20000, 1_700_000_000_000_000
    bufs = [generate(prog, n, gpu, seed=i + 1, row0=i * n, base_ms=t0 // 1000 + i * 1000 - 1000, step_us=50)
            for i in range(3)]
    views = []
    side = torch.cuda.Stream(gpu)
    for ahead in (False, True, "side"):
        proc = Processor(iot.flow_settings(workdir=str(tmp_path / f"w{ahead}"), variant=variant), gpu)
        proc.keep_views = True
        raws = [RawBatch(b.clone(), o, n) for b, o in bufs]      # a parse consumes its bytes (in-place unescape)
        side.wait_stream(torch.cuda.current_stream(gpu))
        got = []
        for i, rb in enumerate(raws):
            if ahead == "side" and i + 1 < len(raws):
                proc.prepare(raws[i + 1], stream=side)           # overlaps batch i's query kernels
                assert raws[i + 1].pending is not None
            proc.process_batch(rb, t0 + i * 1_000_000, 1_000_000)
            if ahead is True and i + 1 < len(raws):
                proc.prepare(raws[i + 1])
                assert raws[i + 1].pending is not None
            name = "DeviceSummary" if variant == "groupby" else "DeviceWindow"
            v = proc.last_views[name]
            got.append(sorted(zip(*[c.to_pylist() for c in v.columns]), key=lambda r: tuple(map(str, r[:3]))))
        proc.drain()
        views.append(got)
    for x, y in [(a, b) for v in views[1:] for a, b in zip(views[0], v)]:    # per batch, vs parse-in-process
        assert len(x) == len(y)
        for rx, ry in zip(x, y):
            for a, b in zip(rx, ry):
                if isinstance(a, float):
                    assert b == pytest.approx(a, rel=1e-9)      # float sums: atomic order differs between runs
                else:
                    assert a == b


def test_string_concat_and_compact_many_parts(gpu):
    """strings.concat / compact_many go through one multi-part gather launch per 32 parts: 45 parts (empty ones,
    strings longer than the 128-byte lane path, views into shared arenas) against the CPU reference."""
    rnd = random.Random(11)

    def col(k):
        vals = [None if rnd.random() < 0.1 else "".join(rnd.choice("abcé\"xyz") for _ in range(rnd.choice(
            [0, 1, 7, 40, 129, 300]))) for _ in range(k)]
        return vals

    lists = [col(rnd.choice([0, 1, 5, 60, 300])) for _ in range(45)]
    cpu_cols = [strings_from_pylist(v, "cpu") for v in lists]
    gpu_cols = [c.to(gpu) for c in cpu_cols]
    # views: every other part is a take (starts into a bigger arena, not compact)
    for i in range(0, 45, 2):
        if gpu_cols[i].length:
            idx = torch.arange(gpu_cols[i].length - 1, -1, -1)
            cpu_cols[i] = cpu_cols[i].take(idx)
            gpu_cols[i] = gpu_cols[i].take(idx.to(gpu))
    want = [x for c in cpu_cols for x in c.to_pylist()]
    nn = sum(c.length for c in gpu_cols)
    valid = torch.tensor([x is not None for x in want], dtype=torch.bool, device=gpu)
    got = S.concat(gpu_cols, valid)
    assert got.to_pylist() == want
    many = S.compact_many(gpu_cols)
    assert [c.to_pylist() for c in many] == [c.to_pylist() for c in cpu_cols]
    assert nn == got.length


@pytest.mark.gpu
def test_parser_timestamp_shadow_matches_string_kernel(gpu):
    """A string field a projection feeds to stringToTimestamp is converted by the parser from the same bytes
    (ParsePlan ts_shadow, dxa_ts.h): the shadow column equals the string kernel's conversion of the parsed column
    for every accepted form, escapes, nulls, type mismatches and rejects."""
    from dxa.engine.types import StructField, StructType
    from dxa.ops import strings as S
    sch = StructType((StructField("a", StructType((StructField("t", "string"), StructField("k", "long")))),
                      StructField("u", "string")))
    forms = ["2023-11-14T22:13:20Z", "2023-11-14 22:13:20", "2023-11-14 22:13:20.123456", "2023-1-4 2:3:4",
             "11/14/2023 22:13:20", "2023-11-14T22:13:20", "2023-13-14 22:13:20", "bad", "", "2023-11-14",
             "2023-11-14T22:13:20Z ", "\\u0032023-11-14T22:13:20Z", "1999-12-31 23:59:59.9"]
    recs = []
    for i in range(3000):
        f = forms[i % len(forms)]
        t = "null" if i % 17 == 0 else (str(i) if i % 23 == 0 else f'"{f}"')
        recs.append(('{"a":{"t":%s,"k":%d},"u":"x%d"}' % (t, i, i)).encode())
    # a repeated key: the last occurrence decides the string and its shadow alike (a junk, null, numeric or valid
    # second value after a valid first one)
    for i, second in enumerate(['"junk"', "null", "17", '"2020-02-02 02:02:02"', '{"x":1}'] * 40):
        recs.append(('{"a":{"t":"2023-11-14T22:13:20Z","k":%d,"t":%s},"u":"d"}' % (i, second)).encode())
    bg, og = frame_records(recs, device=gpu)
    plan = ParsePlan(sch, ts_shadow={("a", "t")})
    col, ok = parse(bg, og, plan)
    t = col.child("a").child("t")
    assert getattr(t, "_parsed_ts", None) is not None
    want = S.to_timestamp(t)
    got = t._parsed_ts
    wv = want.valid_mask().cpu()
    gv = got.valid_mask().cpu()
    assert torch.equal(wv, gv)
    assert torch.equal(want.data.cpu()[wv], got.data.cpu()[gv])
    assert int(wv.sum()) > 1000


@pytest.mark.gpu
def test_parser_null_strings_are_empty_views(gpu):
    """The parse kernel zeroes every assembled string's (start, length) per row itself (no fill kernels): a
    missing, null, mistyped or malformed-row string is an empty view at offset 0, also for decimal text and raw
    JSON fields, with kept and dropped (column-pruned) fields mixed in the plan."""
    from dxa.engine.decimal import parse_decimal_type
    from dxa.engine.types import StructField, StructType
    sch = StructType((StructField("a", StructType((StructField("s", "string"),
                                                   StructField("d", parse_decimal_type("decimal(10,2)")),
                                                   StructField("k", "long")))),
                      StructField("u", "string"), StructField("v", "string")))
    recs = []
    for i in range(4000):
        parts = []
        if i % 3:
            parts.append('"a":{"s":%s,"d":%s,"k":%d}' % ("null" if i % 7 == 0 else f'"s{i}"',
                                                           "1.25" if i % 5 else "null", i))
        if i % 4:
            parts.append('"u":%s' % ("7" if i % 11 == 0 else f'"u{i}"'))
        parts.append('"v":"w%d"' % i)
        recs.append(("{" + ",".join(parts) + "}" if i % 97 else "{bad").encode())
    bg, og = frame_records(recs, device=gpu)
    for keep in (None, {("a", "s"), ("a", "d"), ("u",)}):
        plan = ParsePlan(sch, keep)
        junk = torch.full((1 << 22,), -1, dtype=torch.int64, device=gpu)   # the allocator hands this back dirty
        del junk
        col, ok = parse(bg, og, plan)
        for path in (("a", "s"), ("u",)):
            c = col
            for p in path:
                c = c.child(p)
            null = ~c.valid_mask().cpu()
            assert int(null.sum()) > 100
            assert int(c.lens.cpu()[null].abs().sum()) == 0
            assert int(c.starts.cpu()[null].abs().sum()) == 0


def test_prefiltered_where_matches_plain_filter(gpu):
    """query.prefilter: the filters over one present table have their WHERE masks evaluated together when the first
    runs, with one count copy; the later ones take their rows without a stream drain; results equal plain filters."""
    from dxa.engine.query import execute, prefilter
    from dxa.sql.parser import parse_query
    rnd = random.Random(3)
    n = 5000
    a = [None if rnd.random() < 0.05 else rnd.randint(0, 20) for _ in range(n)]
    b = [rnd.choice(["x", "yy", None, "zzz"]) for _ in range(n)]
    t = Table(["a", "b"], [column_from_pylist(a, "long", gpu), strings_from_pylist(b, gpu)], n, gpu)
    qs = [parse_query("SELECT a, b FROM T WHERE a > 5 AND b IS NOT NULL"),
          parse_query("SELECT b, a * 2 AS a2 FROM T WHERE length(b) = 2 OR a IS NULL"),
          parse_query("SELECT COUNT(*) AS c FROM T WHERE a < 3"),
          parse_query("SELECT a FROM T WHERE a IN (SELECT a FROM T WHERE a = 1)")]     # sub-query: not early
    cat = Catalog()
    cat.register("T", t)
    ctx = EvalContext(device=gpu)
    prefilter(qs, cat, ctx)
    assert [c[0] for c in ctx.prefilter_cands[id(t)]] == [q.body for q in qs[:3]]   # the sub-query filter: not
    got = [execute(qs[0], cat, ctx)]
    assert {id(q.body) for q in qs[1:3]} == set(ctx.prefilter)   # the first ran all three masks, one count copy
    got += [execute(q, cat, ctx) for q in qs[1:]]
    assert not ctx.prefilter and not ctx.prefilter_cands          # every early mask was consumed
    want = [execute(q, cat, EvalContext(device=gpu)) for q in qs]
    for g, w in zip(got, want):
        assert g.names == w.names and g.length == w.length
        assert [c.to_pylist() for c in g.columns] == [c.to_pylist() for c in w.columns]
