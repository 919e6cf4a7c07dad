"""Ports of the reference's own unit tests and golden fixtures (CPU):

* TransformSQLParserTests.scala — exact parsed statements + view reference counts;
* RedisTests.scala — connection-string parsing with the reference defaults;
* ConcurrentDateFormatTests.scala — ``stringToTimestamp`` of a single-digit-seconds string;
* DataGeneratorTests.scala — schema-metadata-driven random JSON (minValue/maxValue, useCurrentTimeMillis,
  allowedValues, maxLength);
* the flattener golden files (Resource/flattenerConfig.json + jobConfig.json → jobConfig.conf, and
  Resource/Flattener/{config,input}.json → output.conf).
"""
import datetime as dt
import json
import os
import time

import pytest
import torch

from tests.fixtures import ref_path

CFG = ref_path("Services/DataX.Config/DataX.Config.Test/Resource")
need_ref = pytest.mark.skipif(not os.path.isdir(CFG), reason="reference fixtures not mounted")


def test_transform_sql_parser():
    from dxa.sql.transform import COMMAND_QUERY, parse_transform
    sql = ("--DataXQuery--\niottestbatch5s = \nSELECT MIN(myTime) AS __receivedtime,\n      "
           "'00000000-0000-0000-0000-000000000000' AS __ruleid,\n\tIoTDeviceId AS __deviceid,\n        "
           "MAP('avg', AVG(temperature), 'max', MAX(temperature), 'min', MIN(temperature), 'count', "
           "COUNT(temperature)) AS temperature\nFROM DataXProcessedInput\nGROUP BY IoTDeviceId\n--DataXQuery--\n"
           "iottestbatch5salert = \nSELECT 1 AS `doc.schemaversion`,\n\t'alarm' AS `doc.schema`,\n\t'open' AS status,"
           "\n\t'1Rule-1Device-NMessage' AS logic,\n\tunix_timestamp()*1000 AS created,\n\tunix_timestamp()*1000 AS "
           "modified,\n\t'Temperature > 80 degrees' AS `rule.description`,\n\t'Critical' AS `rule.severity`,\n\t"
           "__ruleid AS `rule.id`,\n\t__deviceid AS `device.id`,\n\tSTRUCT(__ruleid, __deviceid, temperature) AS "
           "__aggregates,\n   \t__receivedtime AS `device.msg.received`\nFROM iottestbatch5s\nWHERE "
           "temperature.avg>0")
    r = parse_transform(sql.split("\n"))
    assert [(c.name, c.command_type) for c in r.commands] == [("iottestbatch5s", COMMAND_QUERY),
                                                              ("iottestbatch5salert", COMMAND_QUERY)]
    assert r.commands[0].text == (
        "SELECT MIN(myTime) AS __receivedtime, '00000000-0000-0000-0000-000000000000' AS __ruleid, IoTDeviceId AS "
        "__deviceid, MAP('avg', AVG(temperature), 'max', MAX(temperature), 'min', MIN(temperature), 'count', "
        "COUNT(temperature)) AS temperature FROM DataXProcessedInput GROUP BY IoTDeviceId")
    assert r.commands[1].text == (
        "SELECT 1 AS `doc.schemaversion`, 'alarm' AS `doc.schema`, 'open' AS status, '1Rule-1Device-NMessage' AS "
        "logic, unix_timestamp()*1000 AS created, unix_timestamp()*1000 AS modified, 'Temperature > 80 degrees' AS "
        "`rule.description`, 'Critical' AS `rule.severity`, __ruleid AS `rule.id`, __deviceid AS `device.id`, "
        "STRUCT(__ruleid, __deviceid, temperature) AS __aggregates, __receivedtime AS `device.msg.received` FROM "
        "iottestbatch5s WHERE temperature.avg>0")
    assert r.view_reference_count == {"iottestbatch5s": 1, "iottestbatch5salert": 0}


def test_transform_duplicate_name_is_an_error():
    from dxa.sql.transform import parse_transform
    with pytest.raises(Exception):
        parse_transform("--DataXQuery--\nA = SELECT 1\n--DataXQuery--\nA = SELECT 2")


def test_redis_connection_string():
    from dxa.telemetry.metrics import RedisServerConf, parse_redis_connection_string
    conf = parse_redis_connection_string(
        "asdfasdf.asdfasd.com:6380,password=insertpasswordhere=,ssl=True,abortConnect=False")
    assert conf == RedisServerConf(name="asdfasdf.asdfasd.com", host="asdfasdf.asdfasd.com", port=6380,
                                   key="insertpasswordhere=", timeout=3000, use_ssl=True, is_cluster=True)
    assert parse_redis_connection_string("") is None
    with pytest.raises(ValueError):
        parse_redis_connection_string("nohostport,password=x")


def test_string_to_timestamp():
    from dxa.engine.column import strings_from_pylist
    from dxa.ops.strings import py_string_to_timestamp_us, to_timestamp
    want = int((dt.datetime(2018, 8, 10, 22, 55, 3) - dt.datetime(1970, 1, 1)).total_seconds() * 1e6)
    assert py_string_to_timestamp_us("08/10/2018 22:55:3") == want
    col = to_timestamp(strings_from_pylist(["08/10/2018 22:55:3", "2018-08-10T22:55:03Z", "garbage"], "cpu"))
    assert col.data[:2].tolist() == [want, want]
    assert col.valid_mask().tolist() == [True, True, False]


def test_data_generator_metadata():
    from dxa.engine.types import ArrayType, MapType, StructField, StructType
    from dxa.simulate.datagen import compile_spark, generate_cpu
    schema = StructType((
        StructField("doubleField", "double", False, {"minValue": 5.0, "maxValue": 100.0}),
        StructField("timeField", "long", False, {"useCurrentTimeMillis": True}),
        StructField("intField", "int", False, {"allowedValues": [3, 9]}),
        StructField("stringField", "string", False, {"maxLength": 5}),
        StructField("mapField", MapType("string", "float"), False, {"maxLength": 5}),
        StructField("arrayField", ArrayType("string"), False, {"maxLength": 5}),
    ))
    prog = compile_spark(schema)
    now_ms = int(time.time() * 1000)
    buf, offs = generate_cpu(prog, 50, seed=11, base_ms=now_ms)
    data = bytes(buf.numpy())
    for i in range(50):
        rec = json.loads(data[int(offs[i]):int(offs[i + 1])].decode())
        assert 5.0 <= rec["doubleField"] < 100.0
        assert now_ms - 60_000 <= rec["timeField"] <= int(time.time() * 1000)
        assert rec["intField"] in (3, 9)
        assert len(rec["stringField"]) <= 5
        assert len(rec["mapField"]) <= 5
        assert len(rec["arrayField"]) <= 5


def _props(path):
    out = {}
    with open(path, encoding="utf-8-sig") as f:
        for line in f:
            line = line.strip()
            if line and not line.startswith("#") and "=" in line:
                k, v = line.split("=", 1)
                out[k] = v
    return out


@need_ref
@pytest.mark.parametrize("spec,doc,expected", [
    ("flattenerConfig.json", "jobConfig.json", "jobConfig.conf"),
    ("Flattener/config.json", "Flattener/input.json", "Flattener/output.conf"),
])
def test_flattener_golden(spec, doc, expected):
    from dxa.flow.flattener import flatten
    spec_obj = json.load(open(os.path.join(CFG, spec), encoding="utf-8-sig"))
    doc_obj = json.load(open(os.path.join(CFG, doc), encoding="utf-8-sig"))
    assert flatten(spec_obj, doc_obj) == _props(os.path.join(CFG, expected))


@need_ref
def test_default_spec_is_a_superset_of_reference_spec():
    """Every key the reference's flattener spec emits for its golden job config is emitted by ours too."""
    from dxa.flow.flattener import DEFAULT_SPEC, flatten
    doc_obj = json.load(open(os.path.join(CFG, "jobConfig.json"), encoding="utf-8-sig"))
    ours = flatten(DEFAULT_SPEC, doc_obj)
    ref = _props(os.path.join(CFG, "jobConfig.conf"))
    missing = [k for k in ref if k not in ours]
    assert not missing, missing[:10]


def test_utility_helpers():
    from concurrent.futures import ThreadPoolExecutor
    from dxa import utils as U
    assert U.named_args(["conf=a=b", "x=1", "bad"]) == {"conf": "a=b", "x": "1"}
    assert U.sanitize_column_name("a.b") == "`a.b`" and U.sanitize_column_name("ab") == "ab"
    assert U.inflate(U.deflate("hello\nworld")) == "hello\nworld"
    assert U.inflate_bytes(U.deflate_lines(["a", "b"])) == "a\nb"
    assert U.merge_map_of_counts({"a": 1}, {"a": 2, "b": 3}) == {"a": 3, "b": 3}
    assert U.flatten_map_of_counts({"o": {"x": 1}}) == {"o_x": 1}
    assert U.add_property(None, "k", "v") == {"k": "v"} and U.add_property({"a": "1"}, "k", None) == {"a": "1"}
    assert U.ip_octet("10.1.2.3", 2) == 2 and U.ip_octet("", 0) == 0
    with ThreadPoolExecutor(2) as ex:
        assert U.fail_fast([ex.submit(lambda: 1), ex.submit(lambda: 2)]) == [1, 2]
        with pytest.raises(ZeroDivisionError):
            U.fail_fast([ex.submit(lambda: 1 / 0)])


def test_device_double_formatter_on_host():
    """The __host__ __device__ Ryu/Java formatter of the GPU serializer, run on the CPU, equals the host formatter."""
    import ctypes
    import numpy as np
    from dxa.ops import native as N
    from dxa.ops.serialize import java_double
    try:
        L = N.lib()
    except Exception:
        pytest.skip("kernel library not built")
    rng = np.random.default_rng(7)
    vals = np.concatenate([rng.standard_normal(20000) * 10.0 ** rng.integers(-300, 300, 20000),
                           rng.integers(0, 2**63, 20000, dtype=np.int64).view(np.float64),
                           np.array([0.0, -0.0, 1e7, 9999999.0, 1e-3, 0.00099, 5e-324, 2.2250738585072014e-308,
                                     1.7976931348623157e308, 0.1, 0.3, 1e22, 1e23, 2.0 ** 53])])
    vals = vals[np.isfinite(vals)]
    out = np.zeros(32 * len(vals), dtype=np.uint8)
    lens = np.zeros(len(vals), dtype=np.int32)
    L.dxa_java_double_hostcheck(vals.ctypes.data, len(vals), out.ctypes.data, lens.ctypes.data)
    bad = [v for i, v in enumerate(vals) if bytes(out[32 * i:32 * i + lens[i]]).decode() != java_double(float(v))]
    assert not bad, bad[:5]
