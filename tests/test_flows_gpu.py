"""End-to-end GPU-vs-CPU differential of the five benchmark flows (bench.py --flow …, BASELINE configs 1-5): the
same SimulatedData batches run through the Processor on the MI355X (HIP kernels) and on the CPU (the PyTorch /
Python reference paths), for enough batches to fill a (shortened) window and update the accumulator, and every
output's rows must agree — exactly for strings / integers / timestamps, to 1e-9 relative for floating aggregates
(summation order differs).  Outputs per OutputManager.scala:81-160 (to_json of every row, per sink)."""
import json
import math

import pytest
import torch

from dxa.models import iot

N_EVENTS = 20_000
N_BATCHES = 6
INTERVAL_US = 1_000_000


def _settings(variant, workdir):
    extra = {"datax.job.process.pipelineoutputs": "false"}
    if variant in ("window", "full"):
        # the flows' 5-minute window shortened to 3 s so a few batches fill it (view name unchanged)
        extra["datax.job.process.timewindow.DataXProcessedInput_5minutes.windowduration"] = "3 seconds"
    return iot.flow_settings(workdir=str(workdir), variant=variant, sink="memory", extra=extra, ref_rows=5000)


def _batches(device, clock0_us):
    """The bench's gpu-sim batches: event times inside each batch's second."""
    from dxa.simulate.datagen import generate
    prog = iot.program()
    out = []
    for i in range(N_BATCHES):
        bt = clock0_us + i * INTERVAL_US
        buf, offs = generate(prog, N_EVENTS, device, seed=7919 + i, row0=i * N_EVENTS, base_ms=bt // 1000 - 1000,
                             step_us=max(1, INTERVAL_US // N_EVENTS))
        out.append((bt, buf.cpu().clone(), offs.cpu().clone()))
    return out


def _run(variant, device, batches, workdir):
    from dxa.engine.processor import Processor, RawBatch
    from dxa.io import sinks
    if variant == "join":
        path = _settings(variant, workdir).get("datax.job.input.default.referencedata.RefDevices.path")
        import os
        if not os.path.exists(path):
            iot.write_reference_csv(path, 5000, "cpu")
    sinks.MEMORY_SINKS.clear()
    proc = Processor(_settings(variant, workdir), device)
    per_batch = []
    for bt, buf, offs in batches:
        proc.clock = lambda bt=bt: bt / 1e6 + 0.25         # current_timestamp() (alert EventTime) pinned per batch
        raw = RawBatch(buf.clone().to(device), offs.clone().to(device), N_EVENTS)
        proc.process_batch(raw, bt, INTERVAL_US)
        proc.drain()
        per_batch.append({k: list(v) for k, v in sinks.MEMORY_SINKS.items()})
        sinks.MEMORY_SINKS.clear()
    state = {n: st.active.to_pylist() for n, st in proc.state_tables.items()}
    return per_batch, state


def _key(row):
    """Sort key: every non-float leaf (floats may differ in the last bits)."""
    def strip(v):
        if isinstance(v, dict):
            return tuple((k, strip(x)) for k, x in sorted(v.items()))
        if isinstance(v, list):
            return tuple(strip(x) for x in v)
        if isinstance(v, float):
            return "<f>"
        return v
    return repr(strip(row))


def _close(a, b, path=""):
    if isinstance(a, float) or isinstance(b, float):
        assert isinstance(a, (int, float)) and isinstance(b, (int, float)), (path, a, b)
        if math.isnan(a) and math.isnan(b):
            return
        assert math.isclose(a, b, rel_tol=1e-9, abs_tol=1e-9), (path, a, b)
        return
    if isinstance(a, dict):
        assert isinstance(b, dict) and a.keys() == b.keys(), (path, a, b)
        for k in a:
            _close(a[k], b[k], f"{path}.{k}")
        return
    if isinstance(a, list):
        assert isinstance(b, list) and len(a) == len(b), (path, a, b)
        for i, (x, y) in enumerate(zip(a, b)):
            _close(x, y, f"{path}[{i}]")
        return
    assert a == b, (path, a, b)


def _compare_outputs(gpu_out, cpu_out):
    assert len(gpu_out) == len(cpu_out)
    for bi, (g, c) in enumerate(zip(gpu_out, cpu_out)):
        assert g.keys() == c.keys(), (bi, g.keys(), c.keys())
        for name in g:
            rg = sorted((json.loads(l) for l in g[name]), key=_key)
            rc = sorted((json.loads(l) for l in c[name]), key=_key)
            assert len(rg) == len(rc), (bi, name, len(rg), len(rc))
            for x, y in zip(rg, rc):
                _close(x, y, f"batch{bi}.{name}")


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["groupby", "window", "join", "full", "passthrough"])
def test_flow_outputs_gpu_match_cpu(gpu, variant, tmp_path):
    import time
    clock0 = (int(time.time()) - 3600) * 1_000_000
    batches = _batches(gpu, clock0)
    got_gpu, state_gpu = _run(variant, gpu, batches, tmp_path / "gpu" / "w")
    got_cpu, state_cpu = _run(variant, "cpu", batches, tmp_path / "cpu" / "w")
    _compare_outputs(got_gpu, got_cpu)
    assert any(v for b in got_gpu for v in b.values()), "no output rows at all"
    for name in state_gpu:
        _close(sorted(state_gpu[name], key=_key), sorted(state_cpu[name], key=_key), f"state.{name}")
    if variant in ("full",):
        assert state_gpu["DeviceState"], "accumulator never updated"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["streams", "threads"])
@pytest.mark.parametrize("variant", ["full", "window"])
def test_concurrent_views_match_sequential(gpu, variant, mode, tmp_path, monkeypatch):
    """Independent views on side HIP streams (DXA_VIEW_STREAMS=streams / threads) give the same outputs and
    accumulator as the statement-order run on one stream; the schedule really has a concurrent step."""
    import time
    from dxa.engine.processor import Processor
    clock0 = (int(time.time()) - 3600) * 1_000_000
    batches = _batches(gpu, clock0)
    monkeypatch.setenv("DXA_VIEW_STREAMS", mode)
    p = Processor(_settings(variant, tmp_path / "probe"), gpu)
    steps = p._view_schedule(p._live_statements())
    if variant == "full":
        assert any(len(s) > 1 for s in steps), steps
    got_c, state_c = _run(variant, gpu, batches, tmp_path / "conc" / "w")
    monkeypatch.setenv("DXA_VIEW_STREAMS", "0")
    got_s, state_s = _run(variant, gpu, batches, tmp_path / "seq" / "w")
    _compare_outputs(got_c, got_s)
    for name in state_c:
        _close(sorted(state_c[name], key=_key), sorted(state_s[name], key=_key), f"state.{name}")
