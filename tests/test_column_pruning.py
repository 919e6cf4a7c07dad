"""Column pruning through ``Raw.*`` (Processor._raw_paths_read_by_sql): the JSON parser extracts, and windows retain,
only the raw fields a live statement names — outputs are identical to the unpruned run, and any ``SELECT *`` (or an
output of the projected table itself) keeps every field."""
import json

import torch

from dxa.models import iot
from dxa.ops.jsonparse import FT_SKIP


def _run(variant, prune, tmp_path):
    from dxa.engine.processor import Processor, RawBatch
    from dxa.io import sinks
    from dxa.simulate.datagen import generate
    extra = {"datax.job.process.pipelineoutputs": "false"}
    if variant in ("window", "full"):
        extra["datax.job.process.timewindow.DataXProcessedInput_5minutes.windowduration"] = "3 seconds"
    s = iot.flow_settings(workdir=str(tmp_path / f"{variant}{prune}"), variant=variant, sink="memory", extra=extra,
                          ref_rows=100)
    proc = Processor(s, "cpu", parse_prune=prune)
    sinks.MEMORY_SINKS.clear()
    out = []
    t0 = 1_700_000_000_000_000
    for i in range(3):
        bt = t0 + i * 1_000_000
        buf, offs = generate(iot.program(), 800, "cpu", seed=i + 1, row0=i * 800, base_ms=bt // 1000 - 1000,
                             step_us=1000)
        proc.clock = lambda bt=bt: bt / 1e6
        proc.process_batch(RawBatch(buf, offs, 800), bt, 1_000_000)
        proc.drain()
        out.append({k: sorted(v) for k, v in sinks.MEMORY_SINKS.items()})
        sinks.MEMORY_SINKS.clear()
    return proc, out


def test_pruned_outputs_equal_unpruned(tmp_path):
    for variant in ("groupby", "window", "full"):
        p1, a = _run(variant, True, tmp_path)
        p0, b = _run(variant, False, tmp_path)
        assert a == b, variant
        # unread fields are parsed and dropped when the struct is assembled (the faster form on MI355X), so the
        # pruned plan assembles fewer leaves than the unpruned one
        def assembled(plan):
            return sum(1 for nd in plan.nodes[1:] if nd.code != 0 and not nd.dropped and nd.code != FT_SKIP)
        assert p1.parse_plan.keep and assembled(p1.parse_plan) < assembled(p0.parse_plan)
        leaves = {path[-1] for path in p1.parse_plan.keep}
        assert "deviceType" in leaves and "temperature" in leaves and "firmware" not in leaves
        if variant == "window":
            pane = next(iter(p1.window_store.past.values()))
            raw_cols = {c for c in pane.table.column("deviceDetails").names}
            assert "firmware" not in raw_cols and "deviceId" in raw_cols


def test_star_keeps_every_field(tmp_path):
    p, _ = _run("passthrough", True, tmp_path)
    assert p.parse_plan.keep is None


def test_window_timestamp_column_survives_pruning(tmp_path):
    """``Raw.*`` projection, windowed SQL that never names the timestamp column: the column the settings name
    (datax.job.process.timestampcolumn) is still parsed, so the window store can bucket the rows."""
    from dxa.config.settings import SettingDictionary
    from dxa.engine.processor import Processor
    from dxa.io import sinks
    from dxa.ops.jsonparse import frame_records
    from dxa.engine.processor import RawBatch
    schema = {"type": "struct", "fields": [
        {"name": "id", "type": "long", "nullable": True, "metadata": {}},
        {"name": "ts", "type": "timestamp", "nullable": True, "metadata": {}},
        {"name": "v", "type": "double", "nullable": True, "metadata": {}},
        {"name": "junk", "type": "string", "nullable": True, "metadata": {}}]}
    (tmp_path / "s.json").write_text(json.dumps(schema))
    (tmp_path / "p.txt").write_text("Raw.*\n")
    (tmp_path / "t.txt").write_text("--DataXQuery--\nW = SELECT id, SUM(v) AS sv, COUNT(*) AS c "
                                    "FROM DataXProcessedInput_3seconds GROUP BY id\n")
    d = SettingDictionary({
        "datax.job.name": "tsprune", "datax.job.input.default.blobschemafile": str(tmp_path / "s.json"),
        "datax.job.process.projection": str(tmp_path / "p.txt"),
        "datax.job.process.transform": str(tmp_path / "t.txt"),
        "datax.job.process.timewindow.DataXProcessedInput_3seconds.windowduration": "3 seconds",
        "datax.job.process.watermark": "1 second", "datax.job.process.timestampcolumn": "ts",
        "datax.job.process.pipelineoutputs": "false", "datax.job.output.W.memory.enabled": "true"})
    def run(prune):
        proc = Processor(d, "cpu", parse_prune=prune)
        sinks.MEMORY_SINKS.clear()
        t0 = 1_700_000_000
        got = []
        for b in range(3):
            bt = (t0 + b) * 1_000_000
            recs = [json.dumps({"id": i % 2, "ts": f"2023-11-14T22:13:{19 + b:02d}.{500 + i:03d}Z", "v": 1.0,
                                "junk": "x"}).encode() for i in range(4)]
            buf, offs = frame_records(recs)
            proc.clock = lambda bt=bt: bt / 1e6
            proc.process_batch(RawBatch(buf, offs, len(recs)), bt, 1_000_000)
            proc.drain()
            got.append(sorted(json.loads(l)["c"] for l in sinks.MEMORY_SINKS.get("W", [])))
            sinks.MEMORY_SINKS.clear()
        return proc, got
    proc, got = run(True)
    assert proc.parse_plan.keep is not None
    leaves = {p[-1] for p in proc.parse_plan.keep}
    assert "ts" in leaves and "junk" not in leaves
    _, want = run(False)
    assert got == want and got[-1] and got[-1][0] >= 4     # the window holds more than one batch of rows
