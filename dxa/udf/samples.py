"""Ports of the reference UDF samples (DataProcessing/datax-udf-samples/src/main/scala/datax/sample/**)."""
from __future__ import annotations

import datetime as _dt

from .api import FunctionUDF, Generator, RowUDF, StringNormalizer, UDAF


class UdfHelloWorld(RowUDF):
    """udf/UdfHelloWorld.scala:9-13 — ``"hello, " + p1``."""
    return_type = "string"

    def call(self, p1):
        return "hello, " + str(p1)


class DynamicUdfHelloWorld(Generator):
    """dynamicudf/DynamicUdfHelloWorld.scala:15-27 — a counter bumped by every on_interval()."""

    def __init__(self):
        self.counter = 1
        self.timestamp = _dt.datetime.utcnow()

    def initialize(self, settings):
        def fn(s):
            return f"Hello {s}, my counter is {self.counter}, timestamp at {self.timestamp}"

        def on_interval(batch_time_us):
            self.timestamp = _dt.datetime(1970, 1, 1) + _dt.timedelta(microseconds=batch_time_us)
            self.counter += 1
        return FunctionUDF(fn, "string"), on_interval


class RemoveInvalidChars(StringNormalizer):
    """normalizer/RemoveInvalidChars.scala:12-17 — control chars [\\x00-\\x08\\x0E-\\x1F] → '#'."""

    def byte_map(self):
        m = list(range(256))
        for c in list(range(0x00, 0x09)) + list(range(0x0E, 0x20)):
            m[c] = ord("#")
        return m

    def normalize(self, s):
        return "".join("#" if (ord(c) <= 0x08 or 0x0E <= ord(c) <= 0x1F) else c for c in s)


class UdafLastThreshold(UDAF):
    """udaf/UdafLastThreshold.scala:11-56 — the row with the latest eventTime (ties → later row)."""
    from ..engine.types import StructField, StructType
    return_type = StructType((StructField("eventTime", "timestamp"), StructField("thresholdType", "string"),
                              StructField("val1", "string"), StructField("val2", "string")))

    def initialize(self):
        return None

    def update(self, buf, event_time, threshold_type=None, val1=None, val2=None):
        if event_time is None:
            return buf
        if buf is None or buf["eventTime"] <= event_time:
            return {"eventTime": event_time, "thresholdType": threshold_type, "val1": val1, "val2": val2}
        return buf

    def merge(self, buf, other):
        if other is None:
            return buf
        return self.update(buf, other["eventTime"], other["thresholdType"], other["val1"], other["val2"])


class HealthScore:
    """Device-side UDF (the MI355X counterpart of a Scala UDF): ``healthScore(batteryLevel, signalStrength)`` →
    0..100 from battery percentage and RSSI in dBm, evaluated on whole columns with torch ops (no host round trip)."""
    return_type = "double"
    deterministic = True          # pure function of its inputs: window partials that use it can be cached

    def __call__(self, cols, ctx, n, device):
        import torch
        from ..engine.column import ConstColumn, PrimColumn
        b, s = [c.materialize() if isinstance(c, ConstColumn) else c for c in cols]
        bat = b.data.to(torch.float64).clamp(0, 100)
        sig = ((s.data.to(torch.float64) + 110.0) * (100.0 / 70.0)).clamp(0, 100)
        valid = None
        for c in (b, s):
            if c.valid is not None:
                valid = c.valid if valid is None else valid & c.valid
        return PrimColumn("double", 0.7 * bat + 0.3 * sig, valid)


HEALTH_SCORE_HIP = r"""
__device__ __forceinline__ double clamp100(double x) { return x < 0.0 ? 0.0 : (x > 100.0 ? 100.0 : x); }
__device__ double health_score(double battery, long long rssi) {
  return 0.7 * clamp100(battery) + 0.3 * clamp100(((double)rssi + 110.0) * (100.0 / 70.0));
}
"""


LAST_BY_TIME_HIP = r"""
// the value at the latest event time of the group (ties: the later row) — UdafLastThreshold.scala:11-56 on numbers
struct State { long long t; double v; bool any; };
__device__ void init(State& s) { s.any = false; s.t = 0; s.v = 0.0; }
__device__ void update(State& s, long long t, double v) {
  if (!s.any || s.t <= t) { s.t = t; s.v = v; s.any = true; }
}
__device__ double finish(const State& s, bool& valid) { valid = s.any; return s.v; }
"""


class LastByTimeHip:
    """``lastByTime(eventTime, value)``: a HIP device UDAF (``dxa.udf.hip.HipUDAF``)."""

    def __new__(cls):
        from .hip import HipUDAF
        return HipUDAF(source=LAST_BY_TIME_HIP, return_type="double", arg_types=["timestamp", "double"])


class HealthScoreHip:
    """``HealthScore`` written as a HIP device function (``dxa.udf.hip``): what a Scala UDF jar becomes here."""

    def __new__(cls):
        from .hip import HipUDF
        return HipUDF(source=HEALTH_SCORE_HIP, entry="health_score", return_type="double",
                      arg_types=["double", "long"])


REFERENCE_CLASS_MAP = {
    "datax.sample.udf.UdfHelloWorld": UdfHelloWorld,
    "datax.sample.dynamicudf.DynamicUdfHelloWorld": DynamicUdfHelloWorld,
    "datax.sample.normalizer.RemoveInvalidChars": RemoveInvalidChars,
    "datax.sample.udaf.UdafLastThreshold": UdafLastThreshold,
}
