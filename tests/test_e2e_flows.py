"""End to end on CPU: the reference's onebox sample flows (DeploymentLocal/sample/{BasicLocal,HomeAutomationLocal}.json,
BASELINE config 1) go through config generation, then the generated job runs micro-batches through the streaming
host (local generator source → parse → projection → windows/state/rules/UDF/refdata SQL → metric outputs), and the
engine entry point ``python -m dxa.app`` runs the same conf in a subprocess."""
import json
import os
import shutil
import subprocess
import sys

import pytest

from tests.fixtures import ref_path

SAMPLES = ref_path("DeploymentLocal/sample")
DEVICES = ref_path("DeploymentCloud/Deployment.DataX/Samples/usercontent/devices.csv")
pytestmark = pytest.mark.skipif(not os.path.isdir(SAMPLES), reason="reference samples not mounted")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _flow(name, tmp_path):
    flow = json.load(open(os.path.join(SAMPLES, f"{name}.json"), encoding="utf-8-sig"))
    for rd in flow["gui"]["input"].get("referenceData") or []:
        dst = tmp_path / os.path.basename(rd["properties"]["path"])
        shutil.copy(DEVICES, dst)
        rd["properties"]["path"] = str(dst)
    return flow


@pytest.mark.parametrize("name", ["BasicLocal", "HomeAutomationLocal"])
def test_sample_flow_runs(name, tmp_path, monkeypatch):
    monkeypatch.setenv("DXA_SECRETS_DIR", str(tmp_path / "secrets"))
    from dxa.config.settings import load_config, settings_from_arguments
    from dxa.engine.host import StreamingHost
    from dxa.engine.processor import Processor
    from dxa.flow import configgen
    from dxa.io.sources import build_source
    res = configgen.generate(_flow(name, tmp_path), str(tmp_path / "runtime"))
    d = load_config(settings_from_arguments([f"conf={res.conf_path}"]))
    proc = Processor(d, "cpu")
    src = build_source(d, "cpu", "local")
    # realtime: HomeAutomationLocal stamps events with current_timestamp(), so batch time must track the wall clock
    hist = StreamingHost(proc, src, 1.0, max_batches=3, realtime=True).run()
    assert len(hist) == 3
    m = hist[-1]
    assert m["Input_DataXProcessedInput_Events_Count"] > 0
    outs = [k for k in m if k.startswith("Output_") and k.endswith("_InputEvents")]
    assert outs, m
    # metric outputs land in the flow's metrics file (the dashboard feed)
    metrics_dir = os.path.join(os.path.dirname(res.conf_path), "metrics")
    assert os.path.isdir(metrics_dir) and os.listdir(metrics_dir)
    if name == "HomeAutomationLocal":
        # TIMEWINDOW('5 minutes') views are backed by the window store's retained panes
        assert proc.window_store is not None and proc.window_store.past


def test_app_entry_point(tmp_path):
    env = dict(os.environ, DXA_SECRETS_DIR=str(tmp_path / "secrets"), PYTHONPATH=ROOT)
    from dxa.flow import configgen
    os.environ["DXA_SECRETS_DIR"] = env["DXA_SECRETS_DIR"]
    res = configgen.generate(_flow("BasicLocal", tmp_path), str(tmp_path / "runtime"))
    r = subprocess.run([sys.executable, "-m", "dxa.app", f"conf={res.conf_path}", "app=local", "maxBatches=2",
                        "realtime=false"], capture_output=True, text=True, env=env, timeout=240, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    last = json.loads(r.stdout.strip().splitlines()[-1])
    assert last["batches"] == 2 and last["last"]["Input_DataXProcessedInput_Events_Count"] > 0


def test_input_normalizer_and_preprojection(tmp_path):
    """``datax.job.process.inputnormalizer`` (RemoveInvalidChars: control chars → '#') runs before parsing and
    ``datax.job.process.preprojection`` gets the raw table before projection."""
    from dxa.config.settings import SettingDictionary
    from dxa.engine.processor import Processor
    from dxa.ops.jsonparse import frame_records
    from dxa.engine.processor import RawBatch
    schema = json.dumps({"type": "struct", "fields": [{"name": "s", "type": "string", "nullable": True,
                                                       "metadata": {}}]})
    (tmp_path / "schema.json").write_text(schema)
    (tmp_path / "proj.txt").write_text("Raw.s AS s")
    (tmp_path / "t.txt").write_text("--DataXQuery--\nOut = SELECT s FROM DataXProcessedInput")
    d = SettingDictionary({
        "datax.job.name": "norm", "datax.job.input.default.blobschemafile": str(tmp_path / "schema.json"),
        "datax.job.process.projection": str(tmp_path / "proj.txt"),
        "datax.job.process.transform": str(tmp_path / "t.txt"),
        "datax.job.process.inputnormalizer": "datax.sample.normalizer.RemoveInvalidChars",
        "datax.job.output.Out.memory.enabled": "true"})
    proc = Processor(d, "cpu")
    buf, offs = frame_records([b'{"s":"a\x01b"}', b'{"s":"ok"}'])
    proc.keep_views = True
    proc.process_batch(RawBatch(buf, offs, 2), 0, 1_000_000)
    assert proc.last_views["Out"].column("s").to_pylist() == ["a#b", "ok"]
