"""The flagship benchmark flow: SimulatedData IoT stream → SQL group-by aggregate (BASELINE.json config 2,
"SimulatedData IoT stream, SQL group-by aggregate on 1×MI355X (1M ev/s, 32-col JSON)").

The event shape follows the reference's IoT sample (DeploymentCloud/Deployment.DataX/Samples/samples/iotDevice/
iotsample.json — ``deviceDetails.{deviceId, deviceType, eventTime, homeId, status}``) widened to 32 leaf columns with
telemetry and location sensors; the SQL is the reference's ``DeviceInfoTimeWindow`` aggregate
(Services/DataX.Config/DataX.Config.Test/Resource/configgentest-combined.txt:22-34) plus sensor statistics and an
alert view built on it.
"""
from __future__ import annotations

import json
import os
import tempfile
from typing import Dict, Optional

import torch

from ..config.settings import SettingDictionary
from ..engine.types import StructField, StructType
from ..udf.samples import HEALTH_SCORE_HIP

N_DEVICES = 50
N_HOMES = 50

IOT_FIELDS = [
    {"name": "deviceDetails", "type": "struct", "properties": [
        {"name": "deviceId", "type": "int", "minRange": 1, "maxRange": N_DEVICES + 1},
        {"name": "deviceType", "type": "string", "valueList": ["DoorLock", "Heating", "WindowLock",
                                                                "GarageDoorLock"]},
        {"name": "homeId", "type": "int", "minRange": 1, "maxRange": N_HOMES + 1},
        {"name": "status", "type": "int", "minRange": 0, "maxRange": 2},
        {"name": "eventTime", "type": "dateTime", "utcAddSeconds": "0",
         "datetimeStringFormat": "yyyy-MM-ddTHH:mm:ssZ"},
        {"name": "firmware", "type": "string", "valueList": ["1.0.3", "1.1.0", "2.0.1", "2.1.4"]},
        {"name": "region", "type": "string", "valueList": ["westus", "eastus", "northeurope", "westeurope",
                                                            "southeastasia", "japaneast"]},
        {"name": "floor", "type": "int", "minRange": 0, "maxRange": 30},
    ]},
    {"name": "telemetry", "type": "struct", "properties": [
        {"name": "temperature", "type": "double", "minRange": -20, "maxRange": 45},
        {"name": "humidity", "type": "double", "minRange": 0, "maxRange": 100},
        {"name": "pressure", "type": "double", "minRange": 950, "maxRange": 1050},
        {"name": "co2", "type": "int", "minRange": 350, "maxRange": 2000},
        {"name": "pm25", "type": "double", "minRange": 0, "maxRange": 250},
        {"name": "noise", "type": "double", "minRange": 20, "maxRange": 110},
        {"name": "light", "type": "int", "minRange": 0, "maxRange": 100000},
        {"name": "motion", "type": "int", "minRange": 0, "maxRange": 2},
        {"name": "batteryLevel", "type": "double", "minRange": 0, "maxRange": 100},
        {"name": "voltage", "type": "double", "minRange": 3.0, "maxRange": 4.2},
        {"name": "current", "type": "double", "minRange": 0, "maxRange": 2.5},
        {"name": "power", "type": "double", "minRange": 0, "maxRange": 10},
        {"name": "energy", "type": "double", "minRange": 0, "maxRange": 100000},
        {"name": "signalStrength", "type": "int", "minRange": -110, "maxRange": -40},
        {"name": "rssi", "type": "int", "minRange": -100, "maxRange": -30},
        {"name": "vibration", "type": "double", "minRange": 0, "maxRange": 5},
        {"name": "rpm", "type": "int", "minRange": 0, "maxRange": 6000},
    ]},
    {"name": "location", "type": "struct", "properties": [
        {"name": "latitude", "type": "double", "minRange": -90, "maxRange": 90},
        {"name": "longitude", "type": "double", "minRange": -180, "maxRange": 180},
        {"name": "altitude", "type": "double", "minRange": 0, "maxRange": 4000},
        {"name": "speed", "type": "double", "minRange": 0, "maxRange": 120},
        {"name": "heading", "type": "int", "minRange": 0, "maxRange": 360},
    ]},
    {"name": "sequenceNumber", "type": "long", "minRange": 0, "maxRange": 1000000000},
    {"name": "errorCode", "type": "int", "minRange": 0, "maxRange": 16},
]

IOT_SIM_SCHEMA = {"rulesCounterRefreshInMinutes": 15, "dataSchema": [
    {"dataTypeName": "DeviceTelemetry", "simulationPeriodInMinute": 1, "numEventsPerBatch": 1_000_000,
     "fields": IOT_FIELDS, "rulesData": []}]}

TRANSFORM = """--DataXQuery--
DeviceSummary = SELECT deviceDetails.deviceId,
        deviceDetails.deviceType,
        deviceDetails.homeId,
        COUNT(*) AS EventCount,
        MAX(eventTimeStamp) AS MaxEventTime,
        MIN(deviceDetails.status) AS MinReading,
        MAX(deviceDetails.status) AS MaxReading,
        AVG(telemetry.temperature) AS AvgTemperature,
        MAX(telemetry.temperature) AS MaxTemperature,
        AVG(telemetry.humidity) AS AvgHumidity,
        SUM(telemetry.power) AS TotalPower,
        MIN(telemetry.batteryLevel) AS MinBattery
    FROM DataXProcessedInput
    GROUP BY deviceId, deviceType, homeId

--DataXQuery--
HotDeviceAlerts = SELECT MaxEventTime AS EventTime,
        'HotDevice' AS MetricName,
        MaxTemperature AS Metric,
        'iotbench' AS Product,
        CONCAT('device ', deviceId, ' home ', homeId) AS Pivot1
    FROM DeviceSummary
    WHERE MaxTemperature > 44.99
"""

PROJECTION = "stringToTimestamp(Raw.deviceDetails.eventTime) AS eventTimeStamp\nRaw.*\n"


def _spark_type(f):
    t = f["type"].lower()
    if t == "struct":
        return StructType(tuple(StructField(p["name"], _spark_type(p)) for p in f["properties"]))
    return {"int": "long", "long": "long", "double": "double", "decimal": "double", "string": "string",
            "datetime": "string"}[t]


def _generator_metadata(f) -> dict:
    """DataGenerator-style field metadata (minValue/maxValue, allowedValues, datetimeStringFormat) so the Spark
    schema alone drives realistic synthetic events (local source, LiveQuery samples)."""
    md = {}
    if "valueList" in f:
        md["allowedValues"] = f["valueList"]
    if "minRange" in f:
        md["minValue"], md["maxValue"] = f["minRange"], f["maxRange"]
    if f["type"].lower() == "datetime":
        md["datetimeStringFormat"] = f.get("datetimeStringFormat", "yyyy-MM-ddTHH:mm:ssZ")
    return md


def iot_spark_schema() -> StructType:
    def field(f):
        return StructField(f["name"], _spark_type(f), True, _generator_metadata(f)) \
            if f["type"] != "struct" else StructField(f["name"], StructType(tuple(field(p) for p in f["properties"])))
    return StructType(tuple(field(f) for f in IOT_FIELDS))


def leaf_count(fields=IOT_FIELDS) -> int:
    return sum(leaf_count(f["properties"]) if f["type"] == "struct" else 1 for f in fields)


WINDOW_TRANSFORM = """--DataXQuery--
DeviceWindow = SELECT deviceDetails.deviceId,
        deviceDetails.deviceType,
        deviceDetails.homeId,
        COUNT(*) AS EventCount,
        MAX(eventTimeStamp) AS MaxEventTime,
        MIN(deviceDetails.status) AS MinReading,
        MAX(deviceDetails.status) AS MaxReading,
        AVG(telemetry.temperature) AS AvgTemperature,
        MAX(telemetry.temperature) AS MaxTemperature,
        AVG(telemetry.humidity) AS AvgHumidity,
        SUM(telemetry.power) AS TotalPower,
        MIN(telemetry.batteryLevel) AS MinBattery
    FROM DataXProcessedInput TIMEWINDOW('5 minutes')
    GROUP BY deviceId, deviceType, homeId

--DataXQuery--
HotDeviceAlerts = SELECT MaxEventTime AS EventTime,
        'HotDevice5min' AS MetricName,
        MaxTemperature AS Metric,
        'iotbench' AS Product,
        CONCAT('device ', deviceId, ' home ', homeId) AS Pivot1
    FROM DeviceWindow
    WHERE MaxTemperature > 44.99
"""

REF_ROWS = 100_000_000

JOIN_TRANSFORM = """--DataXQuery--
Enriched = SELECT r.zone AS zone,
        r.tier AS tier,
        deviceDetails.deviceType AS deviceType,
        telemetry.power AS power,
        telemetry.temperature AS temperature
    FROM DataXProcessedInput
    JOIN RefDevices r ON sequenceNumber % {ref_rows} = r.refKey

--DataXQuery--
ZoneSummary = SELECT zone, tier, deviceType,
        COUNT(*) AS EventCount,
        SUM(power) AS TotalPower,
        AVG(temperature) AS AvgTemperature,
        MAX(temperature) AS MaxTemperature
    FROM Enriched
    GROUP BY zone, tier, deviceType
"""

FULL_USER_CODE = """--DataXStates--
CREATE TABLE DeviceState (deviceId long, homeId long, deviceType string, LastSeen timestamp, EventCount long,
    MaxTemperature double);

--DataXQuery--
DeviceWindow = SELECT deviceDetails.deviceId AS deviceId,
        deviceDetails.homeId AS homeId,
        deviceDetails.deviceType AS deviceType,
        COUNT(*) AS EventCount,
        MAX(eventTimeStamp) AS LastSeen,
        AVG(telemetry.temperature) AS AvgTemperature,
        MAX(telemetry.temperature) AS MaxTemperature,
        AVG(healthScore(telemetry.batteryLevel, telemetry.signalStrength)) AS AvgHealth
    FROM DataXProcessedInput TIMEWINDOW('5 minutes')
    GROUP BY deviceId, homeId, deviceType;

--DataXQuery--
DeviceNamed = SELECT w.deviceId, w.homeId, w.deviceType, w.EventCount, w.LastSeen, w.MaxTemperature, w.AvgHealth,
        d.deviceName
    FROM DeviceWindow w
    JOIN myDevicesRefdata d ON w.deviceId = d.deviceId AND w.homeId = d.homeId;

--DataXQuery--
DeviceState = SELECT deviceId, homeId, deviceType,
        MAX(LastSeen) AS LastSeen,
        MAX(EventCount) AS EventCount,
        MAX(MaxTemperature) AS MaxTemperature
    FROM (SELECT deviceId, homeId, deviceType, LastSeen, EventCount, MaxTemperature FROM DeviceWindow
          UNION ALL
          SELECT deviceId, homeId, deviceType, LastSeen, EventCount, MaxTemperature FROM DeviceState) s
    GROUP BY deviceId, homeId, deviceType;

--DataXQuery--
Tagged = ProcessRules(DataXProcessedInput);

--DataXQuery--
UnhealthyDevices = SELECT deviceName, deviceType, homeId, AvgHealth
    FROM DeviceNamed
    WHERE AvgHealth < 49.8;

OUTPUT UnhealthyDevices TO Metrics;
"""

FULL_RULES = [
    {"$ruleId": "hot", "$productId": "iotbench", "$ruleType": "SimpleRule", "$ruleDescription": "hot device",
     "$severity": "Critical", "$condition": "telemetry.temperature > 44.5", "$tagname": "Tag", "$tag": "Hot",
     "$isAlert": True, "$alertsinks": ["Metrics"], "schemaTableName": "DataXProcessedInput"},
    {"$ruleId": "lowbat", "$productId": "iotbench", "$ruleType": "SimpleRule", "$ruleDescription": "battery low",
     "$severity": "Medium", "$condition": "telemetry.batteryLevel < 1.0 AND deviceDetails.status = 1",
     "$tagname": "Tag", "$tag": "LowBattery", "$isAlert": True, "$alertsinks": ["Metrics"],
     "schemaTableName": "DataXProcessedInput"},
    {"$ruleId": "noisy", "$productId": "iotbench", "$ruleType": "SimpleRule", "$ruleDescription": "noisy room",
     "$severity": "Low", "$condition": "telemetry.noise > 109.9", "$tagname": "Tag", "$tag": "Noisy",
     "$isAlert": False, "schemaTableName": "DataXProcessedInput"},
]

PASSTHROUGH_USER_CODE = """--DataXQuery--
Tagged = ProcessRules(DataXProcessedInput);

OUTPUT Tagged TO Events;
"""

VARIANTS = ("groupby", "window", "join", "full", "passthrough")


def flow_settings(workdir: Optional[str] = None, sink: str = "null", extra: Optional[Dict[str, str]] = None,
                  name: str = "iotbench", variant: str = "groupby", ref_rows: int = REF_ROWS) -> SettingDictionary:
    """Job settings for one of the benchmark flows (BASELINE.json configs 2-5):

    * ``groupby`` — per-batch GROUP BY + alert view (config 2);
    * ``window``  — the same aggregate over a 5-minute sliding window, 1-s slide (config 3);
    * ``join``    — stream–static join against a ``ref_rows``-row reference table resident in HBM (config 4;
      the table itself is built on device by ``reference_table``);
    * ``full``    — rules (codegen'd ProcessRules + alerts) + windowed SQL with a device UDF + reference-data join +
      accumulator state table (config 5);
    * ``passthrough`` — the hello-world shape of config 1 at full rate: tag rules on every event, every tagged
      event serialised to JSON and written (exercises the device JSON serializer).
    """
    from ..engine.types import schema_to_json
    if variant not in VARIANTS:
        raise ValueError(f"unknown flow variant {variant}")
    workdir = workdir or tempfile.mkdtemp(prefix="dxa_iot_")
    os.makedirs(workdir, exist_ok=True)
    paths = {"schema": os.path.join(workdir, "inputschema.json"),
             "projection": os.path.join(workdir, "projection.txt"),
             "transform": os.path.join(workdir, f"{name}-combined.txt")}
    if variant == "join":
        # the 100M-row reference table goes through the real referencedata path: a CSV file, loaded on the device
        # (rank 0 reads, RCCL broadcast, line framing + tokenizer kernels); written once per size
        ref_csv = os.path.join(os.path.dirname(workdir.rstrip("/")) or workdir, f"dxa_refdevices_{ref_rows}.csv")
        extra = dict(extra or {})
        extra.setdefault("datax.job.input.default.referencedata.RefDevices.path", ref_csv)
        extra.setdefault("datax.job.input.default.referencedata.RefDevices.format", "csv")
        extra.setdefault("datax.job.input.default.referencedata.RefDevices.header", "true")
        extra.setdefault("datax.job.input.default.referencedata.RefDevices.schema", REF_SCHEMA)
    outputs = {"groupby": ["DeviceSummary", "HotDeviceAlerts"], "window": ["DeviceWindow", "HotDeviceAlerts"],
               "join": ["ZoneSummary"], "full": ["DeviceNamed", "DeviceState"], "passthrough": ["Tagged"]}[variant]
    d = {
        "datax.job.name": name,
        "datax.job.input.default.blobschemafile": paths["schema"],
        "datax.job.input.default.streaming.intervalinseconds": "1",
        "datax.job.process.projection": paths["projection"],
        "datax.job.process.transform": paths["transform"],
    }
    if variant == "groupby":
        transform = TRANSFORM
    elif variant == "window":
        transform = WINDOW_TRANSFORM
    elif variant == "join":
        transform = JOIN_TRANSFORM.format(ref_rows=ref_rows)
    elif variant == "passthrough":
        from ..sql.codegen import generate_code
        transform = generate_code(PASSTHROUGH_USER_CODE, [dict(r, **{"$isAlert": False}) for r in FULL_RULES],
                                  "iotbench").code
    else:
        from ..sql.codegen import generate_code
        rc = generate_code(FULL_USER_CODE, FULL_RULES, "iotbench")
        transform = rc.code
        for tables, _sink in rc.outputs:
            outputs += [t.strip() for t in tables.split(",") if t.strip() not in outputs]
        ref = os.path.join(workdir, "devices.csv")
        with open(ref, "w") as f:
            f.write("deviceId,homeId,deviceName\n")
            for dv in range(1, N_DEVICES + 1):
                for h in range(1, N_HOMES + 1):
                    f.write(f"{dv},{h},device-{dv}-home-{h}\n")
        d.update({
            "datax.job.input.default.referencedata.myDevicesRefdata.path": ref,
            "datax.job.input.default.referencedata.myDevicesRefdata.format": "csv",
            "datax.job.input.default.referencedata.myDevicesRefdata.header": "true",
            # the flow's "Scala UDF" is a HIP device function here (dxa.udf.hip), compiled with hipRTC at startup
            "datax.job.process.hipudf.healthScore.source": HEALTH_SCORE_HIP,
            "datax.job.process.hipudf.healthScore.entry": "health_score",
            "datax.job.process.hipudf.healthScore.returntype": "double",
            "datax.job.process.hipudf.healthScore.argtypes": "double;long",
            "datax.job.process.statetable.DeviceState.schema":
                "deviceId long, homeId long, deviceType string, LastSeen timestamp, EventCount long, "
                "MaxTemperature double",
            "datax.job.process.statetable.DeviceState.location": os.path.join(workdir, "state", "DeviceState"),
        })
    if variant in ("window", "full"):
        d.update({
            "datax.job.process.timewindow.DataXProcessedInput_5minutes.windowduration": "5 minutes",
            "datax.job.process.watermark": "2 second",
            "datax.job.process.timestampcolumn": "eventTimeStamp",
        })
    for o in dict.fromkeys(outputs):
        d[f"datax.job.output.{o}.{sink}.enabled"] = "true"
        if sink == "blob":                    # gzip JSON files under the work dir (BlobSinker's layout)
            d[f"datax.job.output.{o}.blob.group.main.folder"] = os.path.join(workdir, "out", o) + "/"
            d[f"datax.job.output.{o}.blob.compressiontype"] = "gzip"
    with open(paths["schema"], "w") as f:
        f.write(schema_to_json(iot_spark_schema()))
    with open(paths["projection"], "w") as f:
        f.write(PROJECTION)
    with open(paths["transform"], "w") as f:
        f.write(transform)
    if extra:
        d.update(extra)
    return SettingDictionary(d)


REF_SCHEMA = "refKey long, zone long, tier string"
_TIERS = (b"bronze", b"silver", b"gold", b"platinum")


def write_reference_csv(path: str, n_rows: int, device, chunk: int = 1 << 23) -> int:
    """The device-registry reference data as a CSV file (``refKey,zone,tier`` with a header): the same rows as
    ``reference_table`` (shuffled keys 0..n-1, zone = hash % 1000, one of 4 tiers), rendered on the device 8 M rows
    at a time and written once.  Returns the file size."""
    device = torch.device(device)
    g = torch.Generator(device="cpu").manual_seed(1234)
    keys_all = torch.randperm(n_rows, generator=g).to(device) if n_rows <= 4_000_000 else \
        _device_perm(n_rows, device)
    kw = max(1, len(str(max(n_rows - 1, 0))))
    tw = max(len(t) for t in _TIERS)
    tab = torch.zeros((4, tw), dtype=torch.uint8)
    tmask = torch.zeros((4, tw), dtype=torch.bool)
    for i, t in enumerate(_TIERS):
        tab[i, :len(t)] = torch.tensor(list(t), dtype=torch.uint8)
        tmask[i, :len(t)] = True
    tab, tmask = tab.to(device), tmask.to(device)

    def digits(x, width):
        d = torch.empty((x.shape[0], width), dtype=torch.uint8, device=device)
        v = x.clone()
        for k in range(width - 1, -1, -1):
            d[:, k] = (v % 10).to(torch.uint8) + 48
            v //= 10
        nd = torch.ones_like(x)
        t = x // 10
        for _ in range(width - 1):
            nd += (t > 0).to(nd.dtype)
            t //= 10
        keep = torch.arange(width, device=device).unsqueeze(0) >= (width - nd).unsqueeze(1)
        return d, keep
    size = 0
    with open(path, "wb") as f:
        head = b"refKey,zone,tier\n"
        f.write(head)
        size += len(head)
        for lo in range(0, n_rows, chunk):
            keys = keys_all[lo:lo + chunk]
            n = keys.shape[0]
            zone, tier = (keys * 2654435761) % 1000, keys % 4
            kd, kk = digits(keys, kw)
            zd, zk = digits(zone, 3)
            comma = torch.full((n, 1), 44, dtype=torch.uint8, device=device)
            nl = torch.full((n, 1), 10, dtype=torch.uint8, device=device)
            ones = torch.ones((n, 1), dtype=torch.bool, device=device)
            body = torch.cat([kd, comma, zd, comma, tab[tier], nl], 1)
            keep = torch.cat([kk, ones, zk, ones, tmask[tier], ones], 1)
            data = body[keep].cpu().numpy()
            data.tofile(f)
            size += int(data.size)
    return size


def reference_table(n_rows: int, device):
    """Synthetic device-registry reference table resident in HBM: refKey (0..n-1, shuffled), zone (0..999),
    tier (one of 4 strings, stored as views into a shared 24-byte arena)."""
    from ..engine.column import PrimColumn, StrColumn, Table
    device = torch.device(device)
    g = torch.Generator(device="cpu").manual_seed(1234)
    keys = torch.randperm(n_rows, generator=g).to(device) if n_rows <= 4_000_000 else \
        _device_perm(n_rows, device)
    zone = (keys * 2654435761) % 1000
    tiers = [b"bronze", b"silver", b"gold", b"platinum"]
    arena = torch.tensor(list(b"".join(tiers)), dtype=torch.uint8, device=device)
    tstart = torch.tensor([0, 6, 12, 16], dtype=torch.int64, device=device)
    tlen = torch.tensor([6, 6, 4, 8], dtype=torch.int32, device=device)
    ti = keys % 4
    tier = StrColumn(arena, tstart[ti], tlen[ti])
    t = Table(["refKey", "zone", "tier"], [PrimColumn("long", keys), PrimColumn("long", zone), tier], n_rows,
              device)
    return t


def _device_perm(n: int, device):
    """A bijective shuffle of 0..n-1 without a host round trip: sort by a hash of the index."""
    i = torch.arange(n, dtype=torch.int64, device=device)
    h = (i * -7046029254386353131) ^ ((i >> 29) * 0x632BE59BD9B4E019)
    return torch.argsort(h)


def program(newline: bool = False):
    """Generator program for the IoT event; ``newline=True`` terminates every event with '\\n' (JSON-lines
    payloads: blob files, compressed ingest frames)."""
    from ..simulate.datagen import compile_simulated
    prog = compile_simulated(IOT_FIELDS)
    if newline:
        prog.lit(b"\n")
    return prog


def smoke_batch(device, n: int = 4096):
    """One tiny micro-batch of the IoT flow on ``device`` (driver smoke test)."""
    import time
    from ..engine.processor import Processor, RawBatch
    from ..simulate.datagen import generate
    device = torch.device(device)
    proc = Processor(flow_settings(), device)
    buf, offs = generate(program(), n, device, seed=1)
    now = int(time.time() * 1e6)
    m = proc.process_batch(RawBatch(buf, offs, n), now, 1_000_000)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    assert m["Input_DataXProcessedInput_Events_Count"] == n, m
    assert m["Output_DeviceSummary_Sink_InputEvents"] > 0, m
    return m
