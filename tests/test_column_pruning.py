"""Column pruning through ``Raw.*`` (Processor._raw_paths_read_by_sql): the JSON parser extracts, and windows retain,
only the raw fields a live statement names — outputs are identical to the unpruned run, and any ``SELECT *`` (or an
output of the projected table itself) keeps every field."""
import json

import torch

from dxa.models import iot


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
        assert p1.parse_plan.keep and len(p1.parse_plan.nodes) < len(p0.parse_plan.nodes)
        leaves = {path[-1] for path in p1.parse_plan.keep}
        assert "deviceType" in leaves and "temperature" in leaves and "firmware" not in leaves
        if variant == "window":
            pane = next(iter(p1.window_store.past.values()))
            raw_cols = {c for c in pane.table.column("deviceDetails").names}
            assert "firmware" not in raw_cols and "deviceId" in raw_cols


def test_star_keeps_every_field(tmp_path):
    p, _ = _run("passthrough", True, tmp_path)
    assert p.parse_plan.keep is None
