"""SimulatedData service — the reference's DataX.SimulatedData.DataGenService (DataGen.cs:17-330,
DataGenService.cs:32-375, Model/DataSchema.cs) rebuilt: a schema file (``rulesCounterRefreshInMinutes`` +
``dataSchema[]`` of ``{dataTypeName, simulationPeriodInMinute, numEventsPerBatch, fields, rulesData}``) drives
random events plus *rule-trigger* events whose trigger conditions fire except in the listed minutes.

Two generators:

* ``DataGen`` — host generator that reproduces the reference byte for byte given the same seed: the .NET
  ``System.Random`` subtractive generator, the same field/RNG visiting order and .NET Framework ``G15`` double
  text (checked against the reference's own golden files).
* ``dxa.simulate.datagen`` — the GPU generator (counter-based RNG) used when ``gpu=True`` for high event rates.

``SimulatedDataService`` wakes every ``period_s`` (60 s in the reference), emits each schema whose period divides
the elapsed minutes, appends the rule-trigger events (rank/node 0 only, as the reference does on SF node 0), and
sends them to Kafka / Event Hubs (Kafka endpoint) / an HTTP ingest endpoint / files / an in-process queue.
"""
from __future__ import annotations

import copy
import datetime as _dt
import json
import logging
import os
import re
import threading
import time
from typing import Any, Callable, Dict, List, Optional

log = logging.getLogger("dxa.simulated")

INT32_MAX = 2147483647


class DotNetRandom:
    """``System.Random(seed)`` (the legacy seeded algorithm, Knuth's subtractive generator) — bit-exact."""
    MBIG = INT32_MAX
    MSEED = 161803398

    def __init__(self, seed: Optional[int] = None):
        if seed is None:
            seed = int(time.time() * 1000) & INT32_MAX
        sub = INT32_MAX if seed == -2147483648 else abs(seed)
        mj = self.MSEED - sub
        a = [0] * 56
        a[55] = mj
        mk = 1
        for i in range(1, 55):
            ii = (21 * i) % 55
            a[ii] = mk
            mk = mj - mk
            if mk < 0:
                mk += self.MBIG
            mj = a[ii]
        for _ in range(1, 5):
            for i in range(1, 56):
                a[i] -= a[1 + (i + 30) % 55]
                if a[i] > INT32_MAX or a[i] < -2147483648:      # Int32 wrap-around (unchecked C# arithmetic)
                    a[i] = (a[i] + 2**31) % 2**32 - 2**31
                if a[i] < 0:
                    a[i] += self.MBIG
        self.a, self.inext, self.inextp = a, 0, 21

    def _internal(self) -> int:
        i = self.inext + 1
        if i >= 56:
            i = 1
        j = self.inextp + 1
        if j >= 56:
            j = 1
        r = self.a[i] - self.a[j]
        if r == self.MBIG:
            r -= 1
        if r < 0:
            r += self.MBIG
        self.a[i] = r
        self.inext, self.inextp = i, j
        return r

    def sample(self) -> float:
        return self._internal() * (1.0 / self.MBIG)

    def next_double(self) -> float:
        return self.sample()

    def next(self, lo: int, hi: int) -> int:
        rng = hi - lo
        if rng <= INT32_MAX:
            return int(self.sample() * rng) + lo
        # large range: two samples (GetSampleForLargeRange)
        result = self._internal()
        if self._internal() % 2 == 0:
            result = -result
        d = (result + 2147483646.0) / 4294967293.0
        return int(d * rng) + lo


def dotnet_g15(v: float) -> str:
    """.NET Framework ``Double.ToString()`` ("G15"): 15 significant digits, exponent form ``E+XX`` when needed."""
    if v != v:
        return "NaN"
    if v in (float("inf"), float("-inf")):
        return "Infinity" if v > 0 else "-Infinity"
    s = format(v, ".15g")
    if "e" in s:
        m, e = s.split("e")
        sign = "-" if e.startswith("-") else "+"
        s = f"{m}E{sign}{abs(int(e)):02d}"
    return s


_NET_FMT = [("yyyy", "%Y"), ("MM", "%m"), ("dd", "%d"), ("HH", "%H"), ("mm", "%M"), ("ss", "%S"), ("fff", "%f")]


def dotnet_datetime(t: _dt.datetime, fmt: Optional[str]) -> str:
    if not fmt:
        return t.strftime("%m/%d/%Y %H:%M:%S")
    out = fmt
    for a, b in _NET_FMT:
        out = out.replace(a, b)
    s = t.strftime(out)
    if "%f" in out:
        s = s.replace(t.strftime("%f"), t.strftime("%f")[:3])
    return s


def _num_text(v: Any) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    return str(v)


class DataGen:
    """Host generator with the reference's exact RNG consumption order (DataGen.cs:38-226)."""

    def __init__(self, seed: Optional[int] = None, now: Optional[Callable[[], _dt.datetime]] = None):
        self.random = DotNetRandom(seed)
        self.now = now or _dt.datetime.utcnow

    def _double(self, lo, hi) -> float:
        return self.random.next_double() * (hi - lo) + lo

    def _int(self, lo, hi) -> int:
        return self.random.next(lo, hi)

    def property_string(self, p: Dict[str, Any], first: bool) -> str:
        name = p.get("name")
        t = (p.get("type") or "").lower()
        pre = ("" if first else ",") + f'"{name}":'
        if t == "struct":
            return pre + "{" + self.properties_string(p.get("properties") or []) + "}"
        value = p.get("value")
        if value not in (None, ""):
            if t in ("long", "int", "double"):
                return pre + _num_text(value)
            if t == "string":
                return pre + f'"{value}"'
            return ""
        lo, hi = p.get("minRange"), p.get("maxRange")
        if lo not in (None, "") and hi not in (None, ""):
            q = '"' if p.get("castAsString") else ""
            if t == "array":
                n = int(p.get("length") or 0)
                vals = [q + dotnet_g15(self._double(float(lo), float(hi))) + q for _ in range(max(0, n))]
                return pre + "[" + ",".join(vals) + "]"
            if t in ("long", "int"):
                return pre + q + str(self._int(int(lo), int(hi))) + q
            if t in ("decimal", "double"):
                return pre + q + dotnet_g15(self._double(float(lo), float(hi))) + q
            raise ValueError(f"Unknown type of data being requested on {name}")
        if t == "datetime":
            ts = self.now() + _dt.timedelta(seconds=float(p.get("utcAddSeconds") or 0))
            return pre + '"' + dotnet_datetime(ts, p.get("datetimeStringFormat")) + '"'
        if p.get("valueList") is not None:
            vl = p["valueList"]
            return pre + '"' + str(vl[self._int(0, len(vl))]) + '"'
        return ""

    def properties_string(self, props: List[Dict[str, Any]]) -> str:
        return "".join(self.property_string(p, i == 0) for i, p in enumerate(props))

    def random_event(self, ds: Dict[str, Any]) -> str:
        parts = []
        for f in ds.get("fields") or []:
            if (f.get("type") or "").lower() == "struct":
                parts.append(f'"{f["name"]}":{{' + self.properties_string(f.get("properties") or []) + "}")
            else:
                parts.append(self.property_string(f, True))
        return "{" + ",".join(parts) + "}"

    def generate_random_data(self, ds: Dict[str, Any]) -> List[Dict[str, Any]]:
        return [json.loads(self.random_event(ds)) for _ in range(int(ds.get("numEventsPerBatch") or 0))]

    def generate_rules_data(self, rule: Dict[str, Any], counter: int) -> Dict[str, Any]:
        doc = json.loads(rule["dataStream"]) if isinstance(rule["dataStream"], str) else copy.deepcopy(
            rule["dataStream"])
        for tc in rule.get("triggerConditions") or []:
            parent = _select(doc, tc.get("parentJsonPropertyPath") or "$")
            name = tc["propertyName"]
            pt = (tc.get("propertyType") or "").lower()
            fire = counter not in (tc.get("ruleNotTriggerTimeInMinutes") or [])
            cast = bool(tc.get("castAsString"))
            if pt == "datetime":
                ts = self.now() + _dt.timedelta(seconds=float(tc.get("utcAddSeconds") or 0))
                parent[name] = dotnet_datetime(ts, tc.get("datetimeStringFormat"))
            elif pt in ("double", "decimal", "int", "long"):
                key = "ruleTrigger" if fire else "ruleNotTrigger"
                fixed = tc.get(key + "Value")
                if fixed not in (None, ""):
                    parent[name] = fixed if cast else (float(fixed) if pt in ("double", "decimal") else int(fixed))
                else:
                    lo, hi = float(tc.get(key + "MinRange") or 0), float(tc.get(key + "MaxRange") or 0)
                    v = self._double(lo, hi) if pt in ("double", "decimal") else self._int(int(lo), int(hi))
                    parent[name] = (dotnet_g15(v) if pt in ("double", "decimal") else str(v)) if cast else v
            elif pt == "string":
                parent[name] = tc.get("ruleTriggerValue") if fire else tc.get("ruleNotTriggerValue")
        return doc

    def generate_data_rules(self, ds: Dict[str, Any], counter: int) -> List[Dict[str, Any]]:
        return [self.generate_rules_data(r, counter) for r in ds.get("rulesData") or []]


def _select(doc, path: str):
    """JSONPath subset used by trigger conditions: ``$``, ``$.a.b``, ``a.b``, ``a[0].b``."""
    cur = doc
    for part in [p for p in re.split(r"\.", path.lstrip("$").lstrip(".")) if p]:
        m = re.match(r"^([^\[]+)((\[\d+\])*)$", part)
        cur = cur[m.group(1)]
        for idx in re.findall(r"\[(\d+)\]", m.group(2) or ""):
            cur = cur[int(idx)]
    return cur


# ---------------------------------------------------------------------------------------------------------------------
class SimulatedDataService:
    """The periodic generator loop (DataGenService.cs:86-116) with pluggable outputs."""

    def __init__(self, schemas: List[Dict[str, Any]], outputs: List[Callable[[List[bytes]], None]],
                 period_s: float = 60.0, seed: Optional[int] = None, emit_rules: bool = True, gpu: bool = False,
                 device=None):
        self.schemas = schemas
        for s in self.schemas:
            s["currentCounter"] = 1
        self.outputs = outputs
        self.period_s = period_s
        self.gen = DataGen(seed)
        self.emit_rules = emit_rules
        self.gpu = gpu
        self.device = device
        self.tick = 0
        self._stop = threading.Event()
        self.sent = 0

    def events_for_tick(self, minute: int) -> List[bytes]:
        out: List[bytes] = []
        for sf in self.schemas:
            if sf["currentCounter"] >= int(sf.get("rulesCounterRefreshInMinutes") or 1):
                sf["currentCounter"] = 1
            for ds in sf.get("dataSchema") or []:
                period = int(ds.get("simulationPeriodInMinute") or 1)
                if minute % period:
                    continue
                if self.gpu:
                    out += self._gpu_events(ds)
                else:
                    out += [self.gen.random_event(ds).encode() for _ in range(int(ds.get("numEventsPerBatch") or 0))]
                if self.emit_rules and ds.get("rulesData"):
                    out += [json.dumps(d, separators=(",", ":")).encode()
                            for d in self.gen.generate_data_rules(ds, sf["currentCounter"])]
            sf["currentCounter"] += 1
        return out

    def _gpu_events(self, ds) -> List[bytes]:
        import torch
        from .datagen import compile_simulated, generate
        prog = ds.get("_prog")
        if prog is None:
            prog = ds["_prog"] = compile_simulated(ds.get("fields") or [])
        n = int(ds.get("numEventsPerBatch") or 0)
        dev = self.device or ("cuda" if torch.cuda.is_available() else "cpu")
        buf, offs = generate(prog, n, dev, seed=self.tick + 1, row0=self.tick * n)
        b = bytes(buf.cpu().numpy())
        o = offs.cpu().tolist()
        return [b[o[i]:o[i + 1]] for i in range(n)]

    def run_once(self) -> int:
        events = self.events_for_tick(self.tick)
        for send in self.outputs:
            send(events)
        self.tick += 1
        self.sent += len(events)
        return len(events)

    def run(self, ticks: Optional[int] = None):
        while not self._stop.is_set() and (ticks is None or self.tick < ticks):
            t0 = time.time()
            try:
                self.run_once()
            except Exception:  # noqa: BLE001 — a failed send must not kill the simulator
                log.exception("simulated data tick failed")
            self._stop.wait(max(1.0 if ticks is None else 0.0, self.period_s - (time.time() - t0)))

    def stop(self):
        self._stop.set()


# -- outputs ---------------------------------------------------------------------------------------------------------
def kafka_output(bootstrap: str, topics: List[str], sasl=None, use_ssl=False):
    from ..io.kafka import KafkaClient
    client = KafkaClient(bootstrap, use_ssl=use_ssl, sasl=sasl)
    meta = client.metadata(topics)
    state = {"i": 0}

    def send(events: List[bytes]):
        if not events:
            return
        for k, t in enumerate(topics):
            parts = meta.get(t) or [0]
            chunk = events[k::len(topics)]
            if chunk:
                client.produce(t, parts[state["i"] % len(parts)], chunk)
        state["i"] += 1
    return send


def eventhub_output(conn: str):
    from ..io.kafka import eventhub_kafka_settings
    es = eventhub_kafka_settings(conn)
    return kafka_output(es["bootstrap"], [es["topic"]], sasl=es["sasl"], use_ssl=True)


def http_output(url: str, chunk: int = 1000):
    import urllib.request

    def send(events: List[bytes]):
        for i in range(0, len(events), chunk):
            body = b"[" + b",".join(events[i:i + chunk]) + b"]"
            req = urllib.request.Request(url, data=body, headers={"Content-Type": "application/json"}, method="POST")
            urllib.request.urlopen(req, timeout=10).read()
    return send


def file_output(folder: str):
    os.makedirs(folder, exist_ok=True)

    def send(events: List[bytes]):
        if events:
            import uuid
            p = os.path.join(folder, f"sim-{int(time.time() * 1000)}-{uuid.uuid4().hex[:8]}.json")
            with open(p + ".tmp", "wb") as f:
                f.write(b"\n".join(events) + b"\n")
            os.replace(p + ".tmp", p)
    return send


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="SimulatedData generator service")
    ap.add_argument("--schema", action="append", required=True, help="data schema file(s) (repeatable)")
    ap.add_argument("--kafka")
    ap.add_argument("--topics", default="")
    ap.add_argument("--eventhub")
    ap.add_argument("--http")
    ap.add_argument("--folder")
    ap.add_argument("--period", type=float, default=60.0)
    ap.add_argument("--ticks", type=int, default=None)
    ap.add_argument("--gpu", action="store_true")
    args = ap.parse_args(argv)
    schemas = [json.load(open(p, encoding="utf-8-sig")) for p in args.schema]
    outs = []
    if args.kafka:
        outs.append(kafka_output(args.kafka, [t for t in args.topics.split(",") if t]))
    if args.eventhub:
        outs.append(eventhub_output(args.eventhub))
    if args.http:
        outs.append(http_output(args.http))
    if args.folder:
        outs.append(file_output(args.folder))
    if not outs:
        raise SystemExit("No output specified; a Kafka topic, Event Hub, HTTP endpoint or folder is needed.")
    svc = SimulatedDataService(schemas, outs, args.period, gpu=args.gpu)
    svc.run(args.ticks)
    print(json.dumps({"sent": svc.sent}))


if __name__ == "__main__":
    main()
