"""Reference data (CSV → device string table): Spark 2.4 CSV semantics on the host oracle, the device tokenizer
(csv.hip) against it, the optional schema cast, and loading through the job settings
(ReferenceDataHandler.scala:42-60, CSVUtil.scala:15-41)."""
import random

import pytest
import torch

from dxa.io.refdata import load_csv, tokenize_line

TRICKY = ('id,name,city\r\n'
          '1,alice,paris\r\n'
          '2,"bob, jr","new\\"york"\n'
          '\n'
          '3,,\n'
          '4,"","x"junk,extra,fields\n'
          '5,"say ""hi""",\n'
          '\r\n'
          '6\n'
          '7,ünï,çødé\n'
          '8,"a\\\\b",last')


def test_tokenize_line_semantics():
    assert tokenize_line("a,b,c") == ["a", "b", "c"]
    assert tokenize_line("a,,") == ["a", None, None]
    assert tokenize_line('"x,y",""') == ["x,y", ""]
    assert tokenize_line('"a""b","c\\"d"') == ['a"b', 'c"d']
    assert tokenize_line('"q"tail,z') == ["q", "z"]
    assert tokenize_line("a\tb", "\t") == ["a", "b"]


def test_host_loader(tmp_path):
    p = tmp_path / "r.csv"
    p.write_bytes(TRICKY.encode())
    t = load_csv(str(p), ",", True, "cpu")
    assert t.names == ["id", "name", "city"]
    rows = t.to_pylist()
    assert [r["id"] for r in rows] == [str(i) for i in range(1, 9)]
    assert rows[1] == {"id": "2", "name": "bob, jr", "city": 'new"york'}
    assert rows[2] == {"id": "3", "name": None, "city": None}
    assert rows[3] == {"id": "4", "name": "", "city": "x"}
    assert rows[4]["name"] == 'say "hi"' and rows[5] == {"id": "6", "name": None, "city": None}
    assert rows[7]["name"] == "a\\b" and rows[6]["name"] == "ünï"
    typed = load_csv(str(p), ",", True, "cpu", schema="id long")
    assert typed.column("id").dtype == "long" and typed.column("id").to_pylist()[:2] == [1, 2]


def _random_csv(n, seed):
    rnd = random.Random(seed)
    words = ["plain", "with space", "comma,inside", 'quote"inside', "", "ünicode", "tab\tx", "back\\slash"]
    lines = ["k,a,b,c"]
    for i in range(n):
        cells = [str(i)]
        for _ in range(rnd.randint(0, 4)):
            w = rnd.choice(words)
            if rnd.random() < 0.5 or "," in w or '"' in w:
                w = '"' + w.replace('"', '""' if rnd.random() < 0.5 else '\\"') + '"'
            cells.append(w)
        lines.append(",".join(cells) + ("\r" if rnd.random() < 0.1 else ""))
        if rnd.random() < 0.05:
            lines.append("")
    return "\n".join(lines) + ("\n" if seed % 2 else "")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_device_tokenizer_matches_host(gpu, tmp_path, seed):
    p = tmp_path / "r.csv"
    p.write_bytes((TRICKY if seed == 1 else _random_csv(20000, seed)).encode())
    host = load_csv(str(p), ",", True, "cpu")
    stats = {}
    dev = load_csv(str(p), ",", True, gpu, stats=stats)
    assert dev.names == host.names and dev.length == host.length == stats["rows"]
    assert dev.to_pylist() == host.to_pylist()
    typed = load_csv(str(p), ",", True, gpu, schema="k long" if seed != 1 else "id long")
    assert typed.columns[0].dtype == "long"


@pytest.mark.gpu
def test_device_tsv_no_header(gpu, tmp_path):
    p = tmp_path / "r.tsv"
    p.write_bytes(b"1\ta\n2\t\n3\t\"q\"\n")
    assert load_csv(str(p), "\t", False, gpu).to_pylist() == \
        [{"_c0": "1", "_c1": "a"}, {"_c0": "2", "_c1": None}, {"_c0": "3", "_c1": "q"}]


def test_reference_data_through_job_settings(tmp_path):
    """datax.job.input.default.referencedata.<name>.{path,format,delimiter,header,schema} → a resident table the
    transform joins against."""
    from dxa.config.settings import SettingDictionary
    from dxa.engine.processor import Processor, RawBatch
    from dxa.ops.jsonparse import frame_records
    (tmp_path / "s.json").write_text('{"type":"struct","fields":[{"name":"dev","type":"long","nullable":true,'
                                     '"metadata":{}}]}')
    (tmp_path / "p.txt").write_text("Raw.*\n")
    (tmp_path / "t.txt").write_text("--DataXQuery--\nJ = SELECT d.dev, r.name FROM DataXProcessedInput d "
                                    "JOIN Devs r ON d.dev = r.id\n")
    (tmp_path / "devs.csv").write_text("id,name\n1,one\n2,two\n003,three\n")
    base = {"datax.job.name": "ref", "datax.job.input.default.blobschemafile": str(tmp_path / "s.json"),
            "datax.job.process.projection": str(tmp_path / "p.txt"),
            "datax.job.process.transform": str(tmp_path / "t.txt"), "datax.job.output.J.null.enabled": "true",
            "datax.job.input.default.referencedata.Devs.path": str(tmp_path / "devs.csv"),
            "datax.job.input.default.referencedata.Devs.format": "csv",
            "datax.job.input.default.referencedata.Devs.header": "true"}
    for extra in ({}, {"datax.job.input.default.referencedata.Devs.schema": "id long"}):
        proc = Processor(SettingDictionary(dict(base, **extra)), "cpu")
        proc.keep_views = True
        buf, offs = frame_records([b'{"dev":1}', b'{"dev":3}', b'{"dev":9}'])
        proc.process_batch(RawBatch(buf, offs, 3), 1_000_000, 1_000_000)
        got = sorted((r["dev"], r["name"]) for r in proc.last_views["J"].to_pylist())
        # long = string compares numerically (Spark casts the string side): "003" matches 3
        assert got == [(1, "one"), (3, "three")], extra
        assert proc.reference_stats["Devs"]["rows"] == 3
