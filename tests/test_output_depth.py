"""Output pipeline depth (datax.job.process.outputdepth / DXA_OUTPUT_DEPTH): with two batches' outputs in flight the
sinks receive the same rows, batches complete in order (metrics, state flips) and the accumulator ends the same as
with synchronous outputs."""
import json

import pytest

from dxa.models import iot

N_EVENTS = 2000
INTERVAL_US = 1_000_000


def _run(tmp_path, extra, batches, clock0):
    from dxa.engine.processor import Processor, RawBatch
    from dxa.io import sinks
    extra = dict(extra)
    extra["datax.job.process.timewindow.DataXProcessedInput_5minutes.windowduration"] = "3 seconds"
    settings = iot.flow_settings(workdir=str(tmp_path), variant="full", sink="memory", extra=extra, ref_rows=500)
    sinks.MEMORY_SINKS.clear()
    proc = Processor(settings, "cpu")
    done = []
    proc.on_batch_complete = lambda bt, m: done.append(bt)
    for i, (buf, offs) in enumerate(batches):
        bt = clock0 + i * INTERVAL_US
        proc.clock = lambda bt=bt: bt / 1e6 + 0.25
        proc.process_batch(RawBatch(buf.clone(), offs.clone(), N_EVENTS), bt, INTERVAL_US)
    proc.drain()
    rows = {k: sorted(json.dumps(json.loads(l), sort_keys=True) for l in v) for k, v in sinks.MEMORY_SINKS.items()}
    state = sorted(json.dumps(r, sort_keys=True, default=str) for r in proc.state_tables["DeviceState"].active.to_pylist())
    return rows, state, done, proc


def test_two_batches_in_flight_same_outputs_in_order(tmp_path):
    import time
    from dxa.simulate.datagen import generate
    clock0 = (int(time.time()) - 3600) * 1_000_000
    prog = iot.program()
    batches = []
    for i in range(5):
        bt = clock0 + i * INTERVAL_US
        buf, offs = generate(prog, N_EVENTS, "cpu", seed=11 + i, row0=i * N_EVENTS, base_ms=bt // 1000 - 1000,
                             step_us=INTERVAL_US // N_EVENTS)
        batches.append((buf, offs))
    sync = _run(tmp_path / "sync", {"datax.job.process.pipelineoutputs": "false"}, batches, clock0)
    deep = _run(tmp_path / "deep", {"datax.job.process.pipelineoutputs": "true",
                                    "datax.job.process.outputdepth": "2"}, batches, clock0)
    assert deep[3].output_depth == 2
    assert deep[0] == sync[0] and any(sync[0].values())
    assert deep[1] == sync[1] and sync[1]
    assert deep[2] == sync[2] == sorted(sync[2])           # completed in batch order
