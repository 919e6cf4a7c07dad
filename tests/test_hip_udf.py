"""HIP-source UDFs (dxa.udf.hip): generated elementwise kernel around a user __device__ function.  CPU tests build
the same source with g++; the GPU test compiles it with hipRTC for gfx950 and compares with the torch UDF."""
import random

import pytest
import torch

from dxa.config.settings import SettingDictionary
from dxa.engine.column import column_from_pylist
from dxa.engine.expr import EvalContext
from dxa.engine.query import Catalog, run_sql
from dxa.engine.column import Table
from dxa.udf.hip import HipUDF, HipUdfError
from dxa.udf.registry import build_udfs
from dxa.udf.samples import HEALTH_SCORE_HIP, HealthScore, HealthScoreHip


def _cols(n, device, seed=3):
    rnd = random.Random(seed)
    bat = [None if rnd.random() < 0.1 else rnd.uniform(-10, 120) for _ in range(n)]
    sig = [None if rnd.random() < 0.1 else rnd.randint(-130, -20) for _ in range(n)]
    return column_from_pylist(bat, "double", device), column_from_pylist(sig, "long", device)


def _close(a, b):
    return all((x is None and y is None) or (x is not None and y is not None and abs(x - y) < 1e-12)
               for x, y in zip(a, b))


def test_hip_udf_matches_torch_udf_on_host():
    b, s = _cols(2000, "cpu")
    want = HealthScore()([b, s], None, 2000, torch.device("cpu")).to_pylist()
    got = HealthScoreHip()([b, s], None, 2000, torch.device("cpu")).to_pylist()
    assert _close(got, want) and sum(v is None for v in got) > 0


def test_null_safe_and_boolean_udfs():
    src = "__device__ long long pick(long long a, long long b, bool oka, bool okb) { return oka ? a : (okb ? b : -1); }"
    u = HipUDF(source=src, entry="pick", return_type="long", arg_types=["long", "long"], null_safe=True)
    a = column_from_pylist([1, None, None, 4], "long", "cpu")
    b = column_from_pylist([10, 20, None, None], "long", "cpu")
    out = u([a, b], None, 4, torch.device("cpu"))
    assert out.to_pylist() == [1, 20, -1, 4] and out.valid is None
    neg = HipUDF(source="__device__ bool neg(double x) { return x < 0; }", entry="neg", return_type="boolean",
                 arg_types=["double"])
    assert neg([column_from_pylist([-1.0, 2.0, None], "double", "cpu")], None, 3,
               torch.device("cpu")).to_pylist() == [True, False, None]


def test_bad_declarations():
    with pytest.raises(HipUdfError):
        HipUDF(source="__device__ double f(double x) { return x; }", entry="f(", arg_types=["double"])
    with pytest.raises(HipUdfError):
        HipUDF(source="__device__ double f(double x) { return x; }", entry="f", arg_types=["string"])
    u = HipUDF(source="__device__ double f(double x) { return x; }", entry="f", arg_types=["double"])
    with pytest.raises(HipUdfError):
        u([], None, 0, torch.device("cpu"))


def test_hipudf_from_settings_in_sql(tmp_path):
    p = tmp_path / "hs.hip"
    p.write_text(HEALTH_SCORE_HIP)
    d = SettingDictionary({"datax.job.process.hipudf.healthScore.source": str(p),
                           "datax.job.process.hipudf.healthScore.entry": "health_score",
                           "datax.job.process.hipudf.healthScore.returntype": "double",
                           "datax.job.process.hipudf.healthScore.argtypes": "double;long"})
    udfs, _, _ = build_udfs(d, {}, {})
    b, s = _cols(500, "cpu", seed=9)
    cat = Catalog()
    cat.register("T", Table(["battery", "rssi"], [b, s], 500, torch.device("cpu")))
    out = run_sql("SELECT healthScore(battery, rssi) AS h FROM T WHERE rssi > -100", cat, EvalContext(udfs=udfs))
    rows = [(x, y) for x, y in zip(b.to_pylist(), s.to_pylist()) if y is not None and y > -100]
    want = HealthScore()([column_from_pylist([r[0] for r in rows], "double", "cpu"),
                          column_from_pylist([r[1] for r in rows], "long", "cpu")], None, len(rows),
                         torch.device("cpu")).to_pylist()
    assert _close(out.column("h").to_pylist(), want)


@pytest.mark.gpu
def test_hip_udf_on_gpu_matches_torch(gpu):
    b, s = _cols(300_000, "cpu", seed=11)
    want = HealthScore()([b, s], None, 300_000, torch.device("cpu")).to_pylist()
    gb, gs = b.to(gpu), s.to(gpu)
    got = HealthScoreHip()([gb, gs], None, 300_000, gpu)
    assert got.data.is_cuda
    assert _close(got.to_pylist(), want)


def test_hipudf_flow_function_through_configgen(tmp_path):
    """A flow's ``hipUDF`` function → datax.job.process.hipudf.* in the generated .conf → a callable UDF."""
    from dxa.config.settings import read_conf_file
    from dxa.flow import configgen
    src = tmp_path / "hs.hip"
    src.write_text(HEALTH_SCORE_HIP)
    flow = {"name": "hipflow", "gui": {
        "name": "hipflow", "displayName": "hipflow", "owner": "t",
        "input": {"type": "local", "mode": "streaming", "properties": {
            "inputSchemaFile": '{"type":"struct","fields":[{"name":"b","type":"double"},{"name":"r","type":"long"}]}',
            "normalizationSnippet": "Raw.*", "windowDuration": "1", "maxRate": "10", "timestampColumn": "",
            "watermarkValue": "0", "watermarkUnit": "second"}, "referenceData": []},
        "process": {"queries": ["--DataXQuery--\nT = SELECT healthScore(b, r) AS h FROM DataXProcessedInput;\n"
                                "OUTPUT T TO Metrics;"],
                    "functions": [{"id": "healthScore", "type": "hipUDF", "properties": {
                        "source": str(src), "entry": "health_score", "returnType": "double",
                        "argTypes": ["double", "long"]}}]},
        "outputs": [{"id": "Metrics", "type": "metric", "properties": {}}], "rules": []}}
    res = configgen.generate(flow, str(tmp_path / "runtime"))
    conf = open(res.conf_path).read()
    assert "datax.job.process.hipudf.healthScore.entry=health_score" in conf
    assert "datax.job.process.hipudf.healthScore.argtypes=double;long" in conf
    d = SettingDictionary(read_conf_file(res.conf_path))
    udfs, _, _ = build_udfs(d, {}, {})
    b, s = _cols(50, "cpu", seed=5)
    assert _close(udfs["healthscore"]([b, s], None, 50, torch.device("cpu")).to_pylist(),
                  HealthScore()([b, s], None, 50, torch.device("cpu")).to_pylist())


def _last_by_time_reference(keys, ts, vals):
    best = {}
    for k, t, v in zip(keys, ts, vals):
        if t is None or v is None:
            continue
        if k not in best or best[k][0] <= t:
            best[k] = (t, v)
    return best


def _udaf_table(n, device, seed=4):
    rnd = random.Random(seed)
    keys = [rnd.randint(0, 40) for _ in range(n)]
    ts = [None if rnd.random() < 0.05 else rnd.randint(0, 50) for _ in range(n)]     # many ties
    vals = [None if rnd.random() < 0.05 else rnd.uniform(0, 10) for _ in range(n)]
    t = Table(["k", "t", "v"], [column_from_pylist(keys, "long", device), column_from_pylist(ts, "timestamp", device),
                                column_from_pylist(vals, "double", device)], n, torch.device(device))
    return t, keys, ts, vals


def test_hip_udaf_group_by_on_host():
    from dxa.udf.samples import LastByTimeHip
    t, keys, ts, vals = _udaf_table(3000, "cpu")
    cat = Catalog()
    cat.register("T", t)
    out = run_sql("SELECT k, lastByTime(t, v) AS lv, COUNT(*) AS n FROM T GROUP BY k", cat,
                  EvalContext(udafs={"lastbytime": LastByTimeHip()}))
    best = _last_by_time_reference(keys, ts, vals)
    got = dict(zip(out.column("k").to_pylist(), out.column("lv").to_pylist()))
    assert got == {k: (best[k][1] if k in best else None) for k in set(keys)}


def test_hipudaf_settings():
    from dxa.udf.samples import LAST_BY_TIME_HIP
    d = SettingDictionary({"datax.job.process.hipudaf.lastByTime.source": LAST_BY_TIME_HIP,
                           "datax.job.process.hipudaf.lastByTime.returntype": "double",
                           "datax.job.process.hipudaf.lastByTime.argtypes": "timestamp;double"})
    _, udafs, _ = build_udfs(d, {}, {})
    t, keys, ts, vals = _udaf_table(400, "cpu", seed=8)
    cat = Catalog()
    cat.register("T", t)
    out = run_sql("SELECT k, lastByTime(t, v) AS lv FROM T GROUP BY k", cat, EvalContext(udafs=udafs))
    best = _last_by_time_reference(keys, ts, vals)
    assert dict(zip(out.column("k").to_pylist(), out.column("lv").to_pylist())) == \
        {k: (best[k][1] if k in best else None) for k in set(keys)}


@pytest.mark.gpu
def test_hip_udaf_on_gpu(gpu):
    from dxa.udf.samples import LastByTimeHip
    t, keys, ts, vals = _udaf_table(200_000, gpu, seed=12)
    cat = Catalog()
    cat.register("T", t)
    out = run_sql("SELECT k, lastByTime(t, v) AS lv FROM T GROUP BY k", cat,
                  EvalContext(udafs={"lastbytime": LastByTimeHip()}))
    assert out.column("lv").data.is_cuda
    best = _last_by_time_reference(keys, ts, vals)
    assert dict(zip(out.column("k").to_pylist(), out.column("lv").to_pylist())) == \
        {k: (best[k][1] if k in best else None) for k in set(keys)}
