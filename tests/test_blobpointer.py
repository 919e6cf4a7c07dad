"""Blob-pointer input (BlobPointerInput.scala:28-162): source-id / file-time / output-name regexes, out-of-scope
paths dropped, per-row FileInternal, InputBlobs / Latency-Blobs metrics, ${target} in blob output folders."""
import json
import os

from dxa.config.settings import SettingDictionary


def _write_blob(root, account, rel, lines):
    p = os.path.join(root, "wasbs", "data", f"{account}.blob.core.windows.net", rel)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        f.write("\n".join(json.dumps(l) for l in lines) + "\n")
    return f"wasbs://data@{account}.blob.core.windows.net/{rel}"


def test_blob_pointer_metadata_and_scoping(tmp_path, monkeypatch):
    monkeypatch.setenv("DXA_FS_ROOT", str(tmp_path / "fs"))
    from dxa.io.sources import BlobPointerSource, QueueSource
    root = str(tmp_path / "fs")
    a = _write_blob(root, "acct1", "2024-05-06T07_08_09/devA/part1.json", [{"v": 1}, {"v": 2}])
    b = _write_blob(root, "acct1", "2024-05-06T07_00_00/devB/part2.json", [{"v": 3}])
    c = _write_blob(root, "other", "2024-05-06T07_08_09/devC/part3.json", [{"v": 9}])
    d = SettingDictionary({
        "datax.job.input.default.source.acct1.target": "T1",
        "datax.job.input.default.source.acct1.catalogprefix": "cat",
        "datax.job.input.default.filetimeregex": r"/(\d{4}-\d{2}-\d{2}T\d{2}_\d{2}_\d{2})/",
        "datax.job.input.default.blobpathregex": r"/([^/]+)/([^/.]+)\.json$"})
    q = QueueSource("cpu")
    src = BlobPointerSource(q, "cpu", settings=d)
    q.push_many([json.dumps({"BlobPath": p}) for p in (a, b, c, a)])        # duplicate + out of scope
    raw = src.next_batch(0)
    assert raw.n == 3
    infos = [(i, n) for i, n in raw.file_rows]
    assert [n for _i, n in infos] == [2, 1]
    i0 = infos[0][0]
    assert i0["target"] == "T1" and i0["ruleIndexPrefix"] == "cat" and i0["fileTime"] == "2024-05-06 07:08:09"
    assert i0["outputFileName"] == "devA-part1"
    assert raw.source_metrics["InputBlobs"] == 2 and raw.source_metrics["Latency-Blobs"] > 0


def test_blob_pointer_through_processor_targets_output_folder(tmp_path, monkeypatch):
    monkeypatch.setenv("DXA_FS_ROOT", str(tmp_path / "fs"))
    from dxa.engine.processor import Processor
    from dxa.io.sources import build_source
    root = str(tmp_path / "fs")
    paths = [_write_blob(root, "acct1", f"2024-05-06T07_08_0{i}/dev/p{i}.json", [{"v": i}, {"v": 10 + i}])
             for i in range(3)]
    (tmp_path / "s.json").write_text('{"type":"struct","fields":[{"name":"v","type":"long","nullable":true,'
                                     '"metadata":{}}]}')
    (tmp_path / "p.txt").write_text("Raw.*\n")
    (tmp_path / "t.txt").write_text("--DataXQuery--\nT = SELECT v FROM DataXProcessedInput\n")
    d = SettingDictionary({
        "datax.job.name": "bp", "datax.job.input.default.blobschemafile": str(tmp_path / "s.json"),
        "datax.job.process.projection": str(tmp_path / "p.txt"), "datax.job.process.transform": str(tmp_path / "t.txt"),
        "datax.job.input.default.source.acct1.target": "TGT",
        "datax.job.output.T.blob.group.main.folder": str(tmp_path / "out" / "${target}") + "/",
        "datax.job.output.T.blob.compressiontype": "none"})
    proc = Processor(d, "cpu")
    src = build_source(d, "cpu", "blobpointer")
    src.inner.push_many([json.dumps({"BlobPath": p}) for p in paths])
    m = proc.process_batch(src.next_batch(0), 1_000_000, 1_000_000)
    assert m["InputBlobs"] == 3 and m["Input_DataXProcessedInput_Events_Count"] == 6
    written = [f for dp, _d, fs_ in os.walk(tmp_path / "out") for f in fs_]
    assert written and os.path.isdir(tmp_path / "out" / "TGT")
