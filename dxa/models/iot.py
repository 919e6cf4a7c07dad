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


def iot_spark_schema() -> StructType:
    return StructType(tuple(StructField(f["name"], _spark_type(f)) for f in IOT_FIELDS))


def leaf_count(fields=IOT_FIELDS) -> int:
    return sum(leaf_count(f["properties"]) if f["type"] == "struct" else 1 for f in fields)


def flow_settings(workdir: Optional[str] = None, sink: str = "null", extra: Optional[Dict[str, str]] = None,
                  name: str = "iotbench") -> SettingDictionary:
    from ..engine.types import schema_to_json
    workdir = workdir or tempfile.mkdtemp(prefix="dxa_iot_")
    os.makedirs(workdir, exist_ok=True)
    paths = {"schema": os.path.join(workdir, "inputschema.json"),
             "projection": os.path.join(workdir, "projection.txt"),
             "transform": os.path.join(workdir, f"{name}-combined.txt")}
    with open(paths["schema"], "w") as f:
        f.write(schema_to_json(iot_spark_schema()))
    with open(paths["projection"], "w") as f:
        f.write(PROJECTION)
    with open(paths["transform"], "w") as f:
        f.write(TRANSFORM)
    d = {
        "datax.job.name": name,
        "datax.job.input.default.blobschemafile": paths["schema"],
        "datax.job.input.default.streaming.intervalinseconds": "1",
        "datax.job.process.projection": paths["projection"],
        "datax.job.process.transform": paths["transform"],
        f"datax.job.output.DeviceSummary.{sink}.enabled": "true",
        f"datax.job.output.HotDeviceAlerts.{sink}.enabled": "true",
    }
    if extra:
        d.update(extra)
    return SettingDictionary(d)


def program():
    from ..simulate.datagen import compile_simulated
    return compile_simulated(IOT_FIELDS)


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
