"""Runtime config generation: Flow JSON → job config JSON → flattened ``.conf`` + transform / projection / schema files.

Mirrors the reference's processor chain (Services/DataX.Config/DataX.Config/PublicService/RuntimeConfigGeneration.cs
and ConfigGeneration/Processor/S100…S900) as ordered Python stages over one ``Session``:

  S200 merge defaults → S300 validate → S400 job variables → S450 transform (rules codegen) →
  S500 projection / schema / outputs / reference data / functions / state tables / time windows / timestamp &
       watermark / streaming → S600 job config → S650 flatten → S700 deploy files → S800 job entity →
  S850 metrics config → S900 finalise

Sensitive values (connection strings, function codes) are moved into the local secret store and replaced by
``keyvault://<vault>/<name>`` references (names are ``<flow>-<kind>-<MD5(value)>`` like the reference's).
Stages at the same order number are independent, as in the reference (TaskExtensions.cs:23-37); a per-flow lock
makes generation non-reentrant (GenerationLockDictionary.cs).
"""
from __future__ import annotations

import copy
import hashlib
import json
import re
import os
import threading
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..config import secrets
from ..engine.types import schema_from_json
from ..io import fs
from ..sql.codegen import RulesCode, generate_code
from .flattener import DEFAULT_SPEC, flatten, to_conf

INPUT_TYPES = ("events", "iothub", "kafka", "kafkaeventhub", "blob", "local", "socket", "file")
INPUT_MODES = ("streaming", "batching")
_locks: Dict[str, threading.Lock] = {}
_locks_guard = threading.Lock()


class ConfigGenerationError(Exception):
    pass


@dataclass
class Session:
    flow: Dict[str, Any]
    root: str
    vault: str
    metrics_endpoint: Optional[str]
    tokens: Dict[str, Any] = field(default_factory=dict)
    rules_code: Optional[RulesCode] = None
    files: Dict[str, str] = field(default_factory=dict)        # kind → content
    paths: Dict[str, str] = field(default_factory=dict)        # kind → path
    job_config: Dict[str, Any] = field(default_factory=dict)
    conf: Dict[str, str] = field(default_factory=dict)
    jobs: List[Dict[str, Any]] = field(default_factory=list)

    @property
    def gui(self) -> Dict[str, Any]:
        return self.flow["gui"]

    @property
    def name(self) -> str:
        return self.flow["name"]


def _secret(s: Session, kind: str, value: Optional[str]) -> Optional[str]:
    if value in (None, "") or secrets.is_secret_ref(value):
        return value
    digest = hashlib.md5(str(value).encode("utf-8")).hexdigest().upper()
    return secrets.store(s.vault, f"{s.name}-{kind}-{digest}", str(value))


# ---------------------------------------------------------------------------------------------------------------
# stages
# ---------------------------------------------------------------------------------------------------------------

def _try_resolve(v: str) -> str:
    try:
        return secrets.resolve(v) or ""
    except Exception:  # noqa: BLE001 — unresolvable secret: fall back to the raw reference
        return v or ""


def s200_merge_defaults(s: Session):
    from .templates import default_flow
    base = default_flow(s.name)
    cp = s.flow.setdefault("commonProcessor", {})
    for k, v in base["commonProcessor"].items():
        cp.setdefault(k, copy.deepcopy(v))
    s.flow.setdefault("displayName", s.gui.get("displayName", s.name))
    s.flow.setdefault("metrics", base["metrics"])


def s300_validate(s: Session):
    g = s.gui
    if not s.flow.get("name"):
        raise ConfigGenerationError("flow name is required")
    if not re.match(r"^[A-Za-z0-9]+$", str(s.flow["name"])):
        # names become runtime folder / file names (FlowConfigBuilder.cs:75 keeps only [A-Za-z0-9])
        raise ConfigGenerationError(f"invalid flow name {s.flow['name']!r}: only letters and digits are allowed")
    inp = g.get("input") or {}
    if inp.get("type", "local").lower() not in INPUT_TYPES:
        raise ConfigGenerationError(f"unsupported input type {inp.get('type')}")
    if inp.get("mode", "streaming").lower() not in INPUT_MODES:
        raise ConfigGenerationError(f"unsupported input mode {inp.get('mode')}")
    schema = (inp.get("properties") or {}).get("inputSchemaFile")
    if not schema:
        raise ConfigGenerationError("input schema is required")
    try:
        schema_from_json(schema)
    except Exception as e:  # noqa: BLE001
        raise ConfigGenerationError(f"invalid input schema: {e}") from e


def s400_variables(s: Session):
    base = os.path.join(s.root, s.name)
    s.tokens.update({
        "name": s.name, "runtimeFolder": base,
        "checkpointDir": os.path.join(base, "checkpoints"),
        "stateTableRoot": os.path.join(base, "statetables"),
        "outputRoot": os.path.join(base, "outputs"),
    })


def s450_transform(s: Session):
    queries = s.gui.get("process", {}).get("queries") or []
    code = "\n".join(queries)
    rules = []
    for r in s.gui.get("rules") or []:
        props = r.get("properties", r)
        # the designer stores rule fields with a "_S_" prefix for "$" (DeploymentLocal/sample/*.json)
        rules.append({("$" + k[3:]) if k.startswith("_S_") else k: v for k, v in props.items()})
    product = s.name
    s.rules_code = generate_code(code, rules, "")
    s.files["transform"] = s.rules_code.code
    del product


def s500_projection(s: Session):
    props = s.gui.get("input", {}).get("properties", {})
    snippet = props.get("normalizationSnippet") or "Raw.*"
    lines = [l.strip() for l in snippet.replace("\r\n", "\n").split("\n") if l.strip()]
    s.files["projection"] = "\n".join(lines)          # byte-identical to the reference (no trailing newline)


def s500_schema(s: Session):
    s.files["schema"] = s.gui["input"]["properties"]["inputSchemaFile"]


def s500_outputs(s: Session):
    rc = s.rules_code
    gui_outputs = {o["id"]: o for o in (s.gui.get("outputs") or [])}
    per_table: Dict[str, List[str]] = {}
    for tables, sink in rc.outputs:
        if sink not in gui_outputs:
            continue
        for t in tables.split(","):
            per_table.setdefault(t.strip(), []).append(sink)
    specs = []
    for table, sinks in per_table.items():
        spec: Dict[str, Any] = {"name": table}
        for sid in sinks:
            o = gui_outputs[sid]
            kind = o.get("type", "").lower()
            p = o.get("properties") or {}
            key = None
            if kind == "metric":
                key = "httpPost"
                val = {"endpoint": s.metrics_endpoint or "", "filter": None} if s.metrics_endpoint else None
                if val is None:
                    key = "file"
                    val = {"path": os.path.join(s.tokens["runtimeFolder"], "metrics", f"{table}.jsonl")}
            elif kind in ("blob", "local"):
                key = "blob"
                prefix = p.get("blobPrefix") or sid
                part = p.get("blobPartitionFormat") or "yyyy/MM/dd/HH"
                fmt = part.replace("yyyy", "%1$tY").replace("MM", "%1$tm").replace("dd", "%1$td").replace(
                    "HH", "%1$tH")
                folder = os.path.join(p.get("folder") or s.tokens["outputRoot"], prefix, fmt,
                                      "${quarterBucket}", "${minuteBucket}")
                val = {"groups": {"main": {"folder": _secret(s, "output", folder) if p.get("connectionString")
                                           else folder}},
                       "compressionType": p.get("compressionType", "gzip"), "format": p.get("format", "json")}
            elif kind == "eventhub":
                key = "eventhub"
                val = {"connectionStringRef": _secret(s, "output", p.get("connectionString")),
                       "compressionType": p.get("compressionType", "gzip"), "format": p.get("format", "json")}
            elif kind == "cosmosdb":
                key = "cosmosdb"
                val = {"connectionStringRef": _secret(s, "output", p.get("connectionString")),
                       "database": p.get("db"), "collection": p.get("collection")}
            elif kind in ("sqlserver", "sql"):
                key = "sql"
                val = {"connectionStringRef": _secret(s, "output", p.get("connectionString")),
                       "databaseName": p.get("databaseName"), "table": p.get("tableName") or table,
                       "writeMode": p.get("writeMode", "append")}
            elif kind in ("httppost", "http"):
                key = "httpPost"
                val = {"endpoint": p.get("endpoint"), "filter": p.get("filter")}
            elif kind in ("console", "file", "memory"):
                key = kind
                val = {"path": p.get("path")} if kind == "file" else ({"maxRows": p.get("maxRows", 20)}
                                                                      if kind == "console" else {"enabled": "true"})
            else:
                raise ConfigGenerationError(f"{o.get('type')} output type not supported")
            if key in spec:
                raise ConfigGenerationError(f"Multiple target {key} output for same dataset not supported.")
            spec[key] = val
        specs.append(spec)
    s.tokens["outputs"] = specs


def s500_reference_data(s: Session):
    out = []
    for rd in s.gui.get("input", {}).get("referenceData") or []:
        p = rd.get("properties") or {}
        out.append({"name": rd["id"], "format": rd.get("type", "csv"), "path": p.get("path"),
                    "delimiter": p.get("delimiter", ","), "header": p.get("header", True)})
    s.tokens["inputReferenceData"] = out


def s500_functions(s: Session):
    udfs, udafs, azf, hip, hipa = [], [], [], [], []
    for f in s.gui.get("process", {}).get("functions") or []:
        p = dict(f.get("properties") or {})
        t = f.get("type", "").lower()
        if t == "jarudf":
            udfs.append({"name": f["id"], "class": p.get("class"), "path": p.get("path"), "libs": p.get("libs") or []})
        elif t == "jarudaf":
            udafs.append({"name": f["id"], "class": p.get("class"), "path": p.get("path"),
                          "libs": p.get("libs") or []})
        elif t == "hipudf":
            # a HIP __device__ function (dxa.udf.hip): the MI355X form of a jar UDF
            hip.append({"name": f["id"], "source": p.get("source") or p.get("path"), "entry": p.get("entry") or f["id"],
                        "returnType": p.get("returnType") or "double", "argTypes": p.get("argTypes") or [],
                        "nullSafe": str(bool(p.get("nullSafe"))).lower()})
        elif t == "hipudaf":
            hipa.append({"name": f["id"], "source": p.get("source") or p.get("path"), "prefix": p.get("prefix") or "",
                         "returnType": p.get("returnType") or "double", "argTypes": p.get("argTypes") or [],
                         "nullSafe": str(bool(p.get("nullSafe"))).lower()})
        elif t == "azurefunction":
            azf.append({"name": f["id"], "serviceEndpoint": p.get("serviceEndpoint"), "api": p.get("api"),
                        "code": _secret(s, "azurefunc", p.get("code")), "methodType": p.get("methodType", "get"),
                        "params": p.get("params") or []})
        else:
            raise ConfigGenerationError(f"unsupported function type {f.get('type')}")
    s.tokens.update(processJarUDFs=udfs, processJarUDAFs=udafs, processAzureFunctions=azf, processHipUDFs=hip,
                    processHipUDAFs=hipa)


def s500_state_tables(s: Session):
    s.tokens["processStateTables"] = [
        {"name": n, "schema": schema.strip(), "location": os.path.join(s.tokens["stateTableRoot"], n) + "/"}
        for n, schema in s.rules_code.accumulation_tables.items()]


def s500_time_windows(s: Session):
    s.tokens["processTimeWindows"] = [{"name": n, "windowDuration": d}
                                      for n, d in s.rules_code.time_windows.items()]


def s500_timestamp(s: Session):
    proc = s.gui.get("process", {})
    props = s.gui.get("input", {}).get("properties", {})
    ts = proc.get("timestampColumn") or props.get("timestampColumn") or None
    wm = proc.get("watermark")
    if not wm and props.get("watermarkValue"):
        wm = f"{props.get('watermarkValue')} {props.get('watermarkUnit', 'second')}"
    s.tokens["processTimestampColumn"] = ts or None
    s.tokens["processWatermark"] = wm or None


def s500_streaming(s: Session):
    props = s.gui.get("input", {}).get("properties", {})
    s.tokens["inputStreamingIntervalInSeconds"] = str(props.get("windowDuration") or 60)
    s.tokens["inputMaxRate"] = str(props.get("maxRate") or "")


def s600_job_config(s: Session):
    t = s.tokens
    inp = s.gui["input"]
    props = inp.get("properties", {})
    kind = inp.get("type", "local").lower()
    base = t["runtimeFolder"]
    s.paths = {"transform": os.path.join(base, f"{s.name}-combined.txt"),
               "projection": os.path.join(base, "projection.txt"),
               "schema": os.path.join(base, "inputschema.json"),
               "conf": os.path.join(base, f"{s.name}.conf")}
    job = {"name": s.name, "input": {
        "blobSchemaFile": s.paths["schema"],
        "streaming": {"checkpointDir": os.path.join(t["checkpointDir"], "streaming"),
                      "intervalInSeconds": t["inputStreamingIntervalInSeconds"]},
        "referenceData": t["inputReferenceData"]}}
    if kind in ("events", "iothub", "kafkaeventhub"):
        job["input"]["eventhub"] = {
            "connectionString": _secret(s, "input-eventhubconnectionstring", props.get("inputEventhubConnection")),
            "consumerGroup": s.name, "checkpointDir": os.path.join(t["checkpointDir"], "eventhub"),
            "checkpointInterval": "60", "maxRate": t["inputMaxRate"] or None, "flushExistingCheckpoints": True}
    elif kind == "kafka":
        job["input"]["kafka"] = {"bootstrapServers": props.get("inputEventhubConnection"),
                                 "topics": props.get("inputEventhubName"), "groupId": s.name,
                                 "checkpointDir": os.path.join(t["checkpointDir"], "kafka"),
                                 "maxRate": t["inputMaxRate"] or None}
    if inp.get("mode", "streaming").lower() == "batching":
        from ..service.scheduler import partition_increment
        blobs = []
        for i, b in enumerate(inp.get("batch") or []):
            bp = b.get("properties") or {}
            path = bp.get("path") or ""
            blobs.append({"name": f"input{i}", "path": path, "format": bp.get("formatType") or "json",
                          "compressiontype": bp.get("compressionType") or "none",
                          "partitionincrement": str(partition_increment(_try_resolve(path)))})
        job["input"]["blob"] = blobs
    elif kind == "local":
        job["input"]["local"] = {"schemaFile": s.paths["schema"],
                                 "eventsPerBatch": str(props.get("eventsPerBatch") or t["inputMaxRate"] or 100)}
    job["process"] = {
        "metric": ({"httppost": s.metrics_endpoint} if s.metrics_endpoint else
                   {"file": os.path.join(base, "metrics", "batch_metrics.jsonl")}),
        "timestampColumn": t["processTimestampColumn"], "watermark": t["processWatermark"],
        "jarUDAFs": t["processJarUDAFs"], "jarUDFs": t["processJarUDFs"], "hipUDFs": t.get("processHipUDFs", []),
        "hipUDAFs": t.get("processHipUDAFs", []),
        "azureFunctions": t["processAzureFunctions"], "projections": [s.paths["projection"]],
        "timeWindows": t["processTimeWindows"], "transform": s.paths["transform"], "appendEventTags": {},
        "accumulationTables": t["processStateTables"]}
    job["outputs"] = t["outputs"]
    s.job_config = job


def s650_flatten(s: Session):
    s.conf = flatten(DEFAULT_SPEC, s.job_config)


def s700_deploy(s: Session):
    for kind in ("transform", "projection", "schema"):
        fs.write_atomic(s.paths[kind], s.files[kind])
    header = f"# Configuration settings for the job {s.name} (generated)\n"
    fs.write_atomic(s.paths["conf"], header + to_conf(s.conf))


def s800_jobs(s: Session):
    inp = s.gui["input"]
    app = {"local": "local", "blob": "batch", "kafka": "kafka", "socket": "socket", "file": "file"}.get(
        inp.get("type", "local").lower(), "eventhub")
    if inp.get("mode", "streaming").lower() == "batching":
        app = "batch"
    cfg = s.gui.get("process", {}).get("jobconfig") or {}
    n = int(cfg.get("jobNumGpus") or 1)
    s.jobs = [{"name": s.name, "flow": s.name, "confPath": s.paths["conf"], "app": app, "gpus": max(1, n),
               "state": "Idle"}]


def s850_metrics(s: Session):
    m = s.flow.setdefault("metrics", {"sources": [], "widgets": []})
    rm = s.rules_code.metrics
    names = {x["name"] for x in m.get("sources", [])}
    for src in rm["sources"]:
        if src["name"] not in names:
            src = json.loads(json.dumps(src).replace("_FLOW_", s.name))
            m.setdefault("sources", []).append(src)
    wnames = {x["name"] for x in m.get("widgets", [])}
    for w in rm["widgets"]:
        if w["name"] not in wnames:
            m.setdefault("widgets", []).append(w)


def s900_finalise(s: Session):
    s.flow["jobNames"] = [j["name"] for j in s.jobs]
    s.flow.setdefault("commonProcessor", {})["sparkJobConfigFolder"] = s.tokens["runtimeFolder"]


STAGES: List[Tuple[int, Callable[[Session], None]]] = [
    (200, s200_merge_defaults), (300, s300_validate), (400, s400_variables), (450, s450_transform),
    (500, s500_projection), (500, s500_schema), (500, s500_outputs), (500, s500_reference_data),
    (500, s500_functions), (500, s500_state_tables), (500, s500_time_windows), (500, s500_timestamp),
    (500, s500_streaming), (600, s600_job_config), (650, s650_flatten), (700, s700_deploy), (800, s800_jobs),
    (850, s850_metrics), (900, s900_finalise),
]


@dataclass
class GenerationResult:
    flow: Dict[str, Any]
    conf: Dict[str, str]
    conf_path: str
    job_config: Dict[str, Any]
    files: Dict[str, str]
    paths: Dict[str, str]
    jobs: List[Dict[str, Any]]
    rules_code: RulesCode


def generate(flow: Dict[str, Any], root: str, vault: str = "dxa", metrics_endpoint: Optional[str] = None,
             extra_stages: Optional[List[Tuple[int, Callable[[Session], None]]]] = None) -> GenerationResult:
    flow = copy.deepcopy(flow)
    if "gui" not in flow:
        flow = {"name": flow.get("name"), "gui": flow}
    flow["name"] = flow.get("name") or flow["gui"].get("name")
    with _locks_guard:
        lock = _locks.setdefault(flow["name"], threading.Lock())
    if not lock.acquire(blocking=False):
        raise ConfigGenerationError(f"config generation for flow '{flow['name']}' is already in progress")
    try:
        s = Session(flow, root, vault, metrics_endpoint)
        stages = sorted(STAGES + list(extra_stages or []), key=lambda x: x[0])
        for _, stage in stages:
            stage(s)
        return GenerationResult(s.flow, s.conf, s.paths["conf"], s.job_config, s.files, s.paths, s.jobs,
                                s.rules_code)
    finally:
        lock.release()
