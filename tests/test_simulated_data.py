"""SimulatedData service: ports DataGenUnitTests.cs (seeded .NET Random → the reference's golden events, byte-level
parity), rule-trigger events, the periodic service loop and its outputs (Kafka via the fake broker, files)."""
import json
import os

import pytest

from dxa.simulate.simulated_data import DataGen, DotNetRandom, SimulatedDataService, dotnet_g15, file_output

from tests.fixtures import ref_path

D = ref_path("Services/DataX.SimulatedData/DataX.SimulatedData.DataGenServiceTest")
need_ref = pytest.mark.skipif(not os.path.isdir(D), reason="reference fixtures not mounted")


def _load(name):
    return json.load(open(os.path.join(D, name), encoding="utf-8-sig"))


def test_dotnet_random_known_sequence():
    r = DotNetRandom(0)
    # System.Random(0): first Next() values (well-known): 1559595546, 1755192844, 1649316166
    assert [r._internal() for _ in range(3)] == [1559595546, 1755192844, 1649316166]
    assert dotnet_g15(19781906739.707066) == "19781906739.7071"
    assert dotnet_g15(1e20) == "1E+20"


@need_ref
@pytest.mark.parametrize("inp,expected", [("testinput1.json", "testrandomexpecteddata1.json"),
                                          ("testinput2Array.json", "testrandomexpecteddata2.json")])
def test_random_data_matches_reference(inp, expected):
    ds = _load(inp)["dataSchema"][0]
    dg = DataGen(1345678)
    got = dg.generate_random_data(dict(ds, numEventsPerBatch=1))[0]
    want = _load(expected)
    got["sensordetails"]["timestamp"] = want["sensordetails"]["timestamp"] = "now"
    assert got == want


@need_ref
def test_rules_data_matches_reference():
    ds = _load("testinput1.json")["dataSchema"][0]
    dg = DataGen(1345678)
    streams = dg.generate_random_data(ds)
    streams += dg.generate_data_rules(ds, 1)
    want = _load("testrulesexpecteddata1.json")
    got = streams[0]
    got["sensordetails"]["timestamp"] = want["sensordetails"]["timestamp"] = "now"
    assert got == want
    assert len(streams) == ds["numEventsPerBatch"] + len(ds.get("rulesData") or [])


def _schema():
    return {"rulesCounterRefreshInMinutes": 3, "dataSchema": [{
        "dataTypeName": "dev", "simulationPeriodInMinute": 1, "numEventsPerBatch": 5,
        "fields": [{"name": "d", "type": "struct", "properties": [
            {"name": "id", "type": "int", "minRange": 1, "maxRange": 4},
            {"name": "kind", "type": "string", "valueList": ["a", "b"]},
            {"name": "t", "type": "double", "minRange": 0, "maxRange": 1}]}],
        "rulesData": [{"dataStream": '{"d":{"id":99,"kind":"a","t":0}}',
                       "triggerConditions": [{"parentJsonPropertyPath": "$.d", "propertyName": "t",
                                              "propertyType": "double", "ruleTriggerValue": "42",
                                              "ruleNotTriggerValue": "1", "ruleNotTriggerTimeInMinutes": [2]}]}]}]}


def test_trigger_conditions_follow_the_minute_counter():
    svc = SimulatedDataService([_schema()], [], period_s=0, seed=5)
    t = []
    for minute in range(4):
        evs = [json.loads(e) for e in svc.events_for_tick(minute)]
        assert len(evs) == 6
        t.append(evs[-1]["d"]["t"])
    # counter 1 → fire, 2 → not-trigger minute, then refresh back to 1 (rulesCounterRefreshInMinutes = 3)
    assert t == [42.0, 1.0, 42.0, 1.0]


def test_service_outputs(tmp_path):
    from dxa.io.kafka import EARLIEST, LATEST, KafkaClient
    from dxa.simulate.simulated_data import kafka_output
    from tests.kafka_fake import FakeBroker
    b = FakeBroker(["sim"], partitions=2)
    try:
        svc = SimulatedDataService([_schema()], [kafka_output(f"127.0.0.1:{b.port}", ["sim"]),
                                                 file_output(str(tmp_path / "out"))], period_s=0, seed=1)
        svc.run(ticks=3)
        assert svc.sent == 18
        c = KafkaClient(f"127.0.0.1:{b.port}")
        assert sum(c.list_offset("sim", p, LATEST) for p in (0, 1)) == 18
        files = os.listdir(tmp_path / "out")
        assert files and sum(len(open(tmp_path / "out" / f).read().splitlines()) for f in files) == 18
    finally:
        b.close()


def test_gpu_program_path_on_cpu():
    svc = SimulatedDataService([_schema()], [], period_s=0, gpu=True, device="cpu", emit_rules=False)
    evs = [json.loads(e) for e in svc.events_for_tick(0)]
    assert len(evs) == 5 and all(1 <= e["d"]["id"] < 4 and e["d"]["kind"] in ("a", "b") for e in evs)


def test_program_length_bound_covers_rendered_events():
    """``GenProgram.max_len`` (the slot size of the one-pass generator) bounds every rendered event, including
    nullable Spark fields, arrays, alphanumerics and extreme seeds."""
    from dxa.models import iot
    from dxa.simulate.datagen import compile_spark, generate_cpu
    from dxa.engine.types import from_json_obj
    spark = from_json_obj({"type": "struct", "fields": [
        {"name": "a", "type": "long", "nullable": True, "metadata": {"minValue": -5, "maxValue": 10 ** 12}},
        {"name": "d", "type": "double", "nullable": True, "metadata": {"minValue": -999.5, "maxValue": 999.5}},
        {"name": "s", "type": "string", "nullable": False, "metadata": {"maxLength": 13}},
        {"name": "t", "type": "string", "nullable": True, "metadata": {"datetimeStringFormat": "MM/dd/yyyy HH:mm:ss"}},
        {"name": "b", "type": "boolean", "nullable": True, "metadata": {}},
        {"name": "arr", "type": {"type": "array", "elementType": "double", "containsNull": True}, "nullable": True,
         "metadata": {"maxLength": 3}}]})
    for prog in (iot.program(), compile_spark(spark)):
        bound = prog.max_len()
        for seed in (1, 2**63 + 5):
            _, offs = generate_cpu(prog, 3000, seed=seed, row0=10 ** 9, base_ms=1_700_000_000_123, step_us=997)
            lens = (offs[1:] - offs[:-1])
            assert int(lens.max()) <= bound
