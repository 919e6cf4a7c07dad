"""Output operators and sinks against the reference's semantics (DataProcessing/datax-host/src/main/scala/datax/sink/
OutputManager.scala, BlobSinker.scala, datax-utility/.../SinkerUtil.scala)."""
import datetime as dt
import glob
import gzip
import json
import os

import pytest


from dxa.config.settings import SettingDictionary
from dxa.engine.column import Table
from dxa.engine.types import StructField, StructType
from dxa.io.sinks import build_outputs

SCHEMA = StructType((StructField("id", "long"), StructField("v", "double")))
ROWS = [{"id": i, "v": float(i - 5)} for i in range(10)]


def _read_all(folder):
    out = []
    for p in sorted(glob.glob(os.path.join(folder, "**", "*.json*"), recursive=True)):
        data = gzip.open(p).read() if p.endswith(".gz") else open(p, "rb").read()
        out += [json.loads(l) for l in data.decode().splitlines() if l.strip()]
    return sorted(out, key=lambda r: r["id"])


def test_blob_groups_by_flag_expression(tmp_path):
    pos, neg = tmp_path / "pos", tmp_path / "neg"
    d = SettingDictionary({
        "datax.job.output.Out.blob.groupevaluation": "CASE WHEN v > 0 THEN 'pos' WHEN v < 0 THEN 'neg' ELSE 'zero' END",
        "datax.job.output.Out.blob.group.pos.folder": str(pos) + "/",
        "datax.job.output.Out.blob.group.neg.folder": str(neg) + "/",
        "datax.job.output.Out.blob.compressiontype": "gzip"})
    op, = build_outputs(d)
    t = Table.from_pylist(ROWS, SCHEMA)
    m = op.output(t, dt.datetime(2024, 1, 1))
    assert [r["id"] for r in _read_all(pos)] == [6, 7, 8, 9]
    assert [r["id"] for r in _read_all(neg)] == [0, 1, 2, 3, 4]
    # 'zero' has no folder: dropped (BlobSinker.sinkDataGroups); per-group metrics, one file per written group
    assert m["Sink_InputEvents"] == 10
    assert m["Sink_Blobs_Events_pos"] == 4 and m["Sink_Blobs_Count_pos"] == 1
    assert m["Sink_Blobs_Events_neg"] == 5 and m["Sink_Blobs_Count_neg"] == 1
    # the metric key set does not depend on the data (ranks all-reduce one vector)
    empty = op.output(Table.from_pylist([], SCHEMA), dt.datetime(2024, 1, 1))
    assert set(empty) == set(m)


def test_blob_without_flag_goes_to_main(tmp_path):
    main = tmp_path / "main"
    d = SettingDictionary({"datax.job.output.Out.blob.group.main.folder": str(main) + "/",
                           "datax.job.output.Out.blob.compressiontype": "none"})
    op, = build_outputs(d)
    m = op.output(Table.from_pylist(ROWS, SCHEMA), dt.datetime(2024, 1, 1))
    assert [r["id"] for r in _read_all(main)] == list(range(10))
    assert m["Sink_Blobs_Events_main"] == 10 and m["Sink_Blobs_Count_main"] == 1


def test_filtered_sink_metric_names(tmp_path):
    d = SettingDictionary({"datax.job.output.Out.file.path": str(tmp_path / "o.jsonl"),
                           "datax.job.output.Out.file.filter": "v >= 3"})
    op, = build_outputs(d)
    m = op.output(Table.from_pylist(ROWS, SCHEMA), dt.datetime(2024, 1, 1))
    assert m["Sink_File_Filtered"] == 2


def test_gzip_parallel_is_one_valid_stream():
    """Blob / Event Hubs payloads are gzip members compressed in parallel and concatenated: one valid gzip
    stream for any reader."""
    import gzip
    import zlib
    from dxa.io.fs import gzip_parallel
    data = b"".join(b'{"i":%d,"s":"%s"}\n' % (i, b"x" * (i % 37)) for i in range(300000))
    z = gzip_parallel(data, chunk=1 << 20)
    assert gzip.decompress(z) == data
    d = zlib.decompressobj(16 + zlib.MAX_WBITS)            # a streaming reader that walks member by member
    out, rest = [], z
    while rest:
        out.append(d.decompress(rest))
        rest = d.unused_data
        d = zlib.decompressobj(16 + zlib.MAX_WBITS) if rest else d
    assert b"".join(out) == data
    assert gzip.decompress(gzip_parallel(b"small")) == b"small"


@pytest.mark.gpu
def test_blob_gzip_compressed_on_device(tmp_path, gpu):
    """A gzip blob sink on a GPU table: the device compresses (ops/deflate.py) and the file inflates to exactly the
    text the uncompressed path writes."""
    rows = [{"id": i, "s": f"device-{i % 97}", "v": i * 0.25} for i in range(60000)]
    schema = StructType((StructField("id", "long"), StructField("s", "string"), StructField("v", "double")))
    outs = {}
    for comp in ("gzip", "none"):
        folder = tmp_path / comp
        d = SettingDictionary({"datax.job.output.Out.blob.group.main.folder": str(folder) + "/",
                               "datax.job.output.Out.blob.compressiontype": comp})
        op, = build_outputs(d)
        staged = op.stage(Table.from_pylist(rows, schema, gpu))
        if comp == "gzip":
            assert staged.items[0][1]["main"].compress
        m = staged.finish(dt.datetime(2024, 1, 1))
        assert m["Sink_Blobs_Events_main"] == len(rows)
        p, = glob.glob(os.path.join(folder, "**", "*.json*"), recursive=True)
        outs[comp] = gzip.open(p).read() if comp == "gzip" else open(p, "rb").read()
    assert outs["gzip"] == outs["none"]
    assert [json.loads(l)["id"] for l in outs["gzip"].splitlines()] == list(range(60000))
