"""Nested job-config JSON → flat ``datax.job.*`` properties.

Semantics of the reference flattener (Services/DataX.Config/DataX.Config/ConfigDataModel/Flattener/*.cs) driven by a
mapping spec:  ``object`` (fixed fields, each either a property name or a nested spec), ``map`` (every key becomes a
namespace, values mapped by ``fields``), ``array`` of ``scopedObject`` (each element scoped by its
``namespaceField``), ``stringList`` (``;``-joined), ``mapProps`` (key → value), ``excludeDefaultValue`` (omitted when
equal to the default).  A key starting with ``^`` is absolute.  Scalars render like Newtonsoft's ``JToken.ToString``
(booleans ``True``/``False``).
"""
from __future__ import annotations

import json
from typing import Any, Dict, Iterator, List, Optional, Tuple


def _text(v: Any) -> Optional[str]:
    if v is None:
        return None
    if isinstance(v, bool):
        return "True" if v else "False"
    if isinstance(v, (dict, list)):
        return json.dumps(v, indent=2)
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    return str(v)


def _prop(ns: Optional[str], key: Optional[str]) -> str:
    if key is not None and key.startswith("^"):
        return key[1:]
    return (ns + "." if ns is not None else "") + (key or "")


def _flatten(spec: Dict, value: Any) -> Iterator[Tuple[str, Optional[str]]]:
    kind = spec.get("type")
    ns = spec.get("namespace")
    if kind == "object":
        if value is None or not spec.get("fields"):
            return
        for field, sub in spec["fields"].items():
            v = value.get(field) if isinstance(value, dict) else None
            if isinstance(sub, dict):
                for k, val in _flatten(sub, v):
                    yield _prop(ns, k), val
            else:
                yield _prop(ns, sub), _text(v)
    elif kind == "map":
        if value is None or not spec.get("fields"):
            return
        inner = {"type": "object", "fields": spec["fields"]}
        for key, v in value.items():
            sub_ns = _prop(ns, key)
            for k, val in _flatten(inner, v):
                yield _prop(sub_ns, k), val
    elif kind == "array":
        if value is None or not spec.get("element"):
            return
        if not isinstance(value, list):
            raise ValueError(f"expected array but encounter json:'{value}'")
        for el in value:
            for k, val in _flatten(spec["element"], el):
                yield _prop(ns, k), val
    elif kind == "scopedObject":
        if value is None or not spec.get("fields"):
            return
        inner = {"type": "object", "fields": spec["fields"], "namespace": _text(value[spec["namespaceField"]])}
        for k, val in _flatten(inner, value):
            yield _prop(ns, k), val
    elif kind == "stringList":
        if value is None:
            return
        if not isinstance(value, list):
            raise ValueError(f"Expecting an array but encounter json:{value}")
        if value:
            yield ns, ";".join(_text(v) for v in value)
    elif kind == "mapProps":
        if value is None:
            return
        for key, v in value.items():
            yield _prop(ns, key), _text(v)
    elif kind == "excludeDefaultValue":
        if value is None:
            return
        if _text(value) != _text(spec.get("defaultValue")):
            yield ns, _text(value)
    elif kind is None:
        return
    else:
        raise ValueError(f"Unknown mapping type '{kind}' in flattening the config.")


def flatten(spec: Dict, config: Dict) -> Dict[str, str]:
    """Flatten ``config`` with ``spec``; null-valued properties are dropped."""
    out: Dict[str, str] = {}
    for k, v in _flatten(spec, config):
        if v is not None:
            out[k] = v
    return out


def to_conf(props: Dict[str, str]) -> str:
    return "".join(f"{k}={v}\n" for k, v in props.items())


def _blob(): return {"type": "object", "namespace": "blob", "fields": {
    "groupEvaluation": "groupevaluation",
    "compressionType": {"type": "excludeDefaultValue", "namespace": "compressiontype", "defaultValue": "gzip"},
    "format": {"type": "excludeDefaultValue", "namespace": "format", "defaultValue": "json"},
    "groups": {"type": "map", "namespace": "group", "fields": {"folder": "folder"}}}}


def _output_fields():
    return {
        "blob": _blob(),
        "eventhub": {"type": "object", "namespace": "eventhub", "fields": {
            "connectionStringRef": "connectionstring",
            "compressionType": {"type": "excludeDefaultValue", "namespace": "compressiontype", "defaultValue": "gzip"},
            "format": {"type": "excludeDefaultValue", "namespace": "format", "defaultValue": "json"},
            "appendProperties": {"type": "mapProps", "namespace": "appendproperty"}}},
        "cosmosdb": {"type": "object", "namespace": "cosmosdb", "fields": {
            "connectionStringRef": "connectionstring", "database": "database", "collection": "collection"}},
        "httpPost": {"type": "object", "namespace": "httppost", "fields": {
            "endpoint": "endpoint", "filter": "filter",
            "appendHeaders": {"type": "mapProps", "namespace": "header"}}},
        "sql": {"type": "object", "namespace": "sql", "fields": {
            "connectionStringRef": "connectionstring", "databaseName": "databasename", "table": "table",
            "writeMode": "writemode", "userName": "user", "password": "password", "url": "url",
            "encrypt": "encrypt", "trustServerCertificate": "trustservercertificate",
            "hostNameInCertificate": "hostnameincertificate", "useBulkInsert": "usebulkinsert"}},
        "file": {"type": "object", "namespace": "file", "fields": {"path": "path", "filter": "filter"}},
        "console": {"type": "object", "namespace": "console", "fields": {"maxRows": "maxrows"}},
        "memory": {"type": "object", "namespace": "memory", "fields": {"enabled": "enabled"}},
    }


def _scoped(ns, fields):
    return {"type": "array", "namespace": ns, "element": {"type": "scopedObject", "namespaceField": "name",
                                                          "fields": fields}}


def _jar():
    return {"class": "class", "path": "path", "libs": {"type": "stringList", "namespace": "libs"}}


# The job-config → properties mapping (same key space as the reference's CommonData.Templates/flattenerConfig.json).
DEFAULT_SPEC: Dict = {
    "type": "object", "namespace": "datax.job",
    "fields": {
        "name": "name",
        "input": {"type": "object", "namespace": "input.default", "fields": {
            "blobSchemaFile": "blobschemafile", "sourceIdRegex": "sourceidregex", "blobPathRegex": "blobpathregex",
            "fileTimeRegex": "filetimeregex", "fileTimeFormat": "filetimeformat",
            "eventhub": {"type": "object", "namespace": "eventhub", "fields": {
                "connectionString": "connectionstring", "consumerGroup": "consumergroup",
                "checkpointDir": "checkpointdir", "checkpointInterval": "checkpointinterval", "maxRate": "maxrate",
                "flushExistingCheckpoints": "flushexistingcheckpoints"}},
            "kafka": {"type": "object", "namespace": "kafka", "fields": {
                "connectionString": "connectionstring", "topics": "topics", "groupId": "groupid",
                "checkpointDir": "checkpointdir", "checkpointInterval": "checkpointinterval", "maxRate": "maxrate",
                "bootstrapServers": "bootstrapservers"}},
            "local": {"type": "object", "namespace": "local", "fields": {
                "schemaFile": "schemafile", "eventsPerBatch": "eventsperbatch", "seed": "seed"}},
            "streaming": {"type": "object", "namespace": "streaming", "fields": {
                "checkpointDir": "checkpointdir", "intervalInSeconds": "intervalinseconds"}},
            "blob": _scoped("blob", {"path": "path", "format": "format", "compressiontype": "compressiontype",
                                     "processstarttime": "processstarttime", "processendtime": "processendtime",
                                     "partitionincrement": "partitionincrement"}),
            "sources": {"type": "map", "namespace": "source", "fields": {"target": "target",
                                                                          "catalogPrefix": "catalogprefix"}},
            "referenceData": _scoped("referencedata", {"path": "path", "format": "format", "header": "header",
                                                        "delimiter": "delimiter"}),
        }},
        "process": {"type": "object", "namespace": "process", "fields": {
            "metric": {"type": "object", "namespace": "metric", "fields": {"eventhub": "eventhub",
                                                                            "httppost": "httppost",
                                                                            "redis": "redis", "file": "file"}},
            "projections": {"type": "stringList", "namespace": "projection"},
            "transform": "transform", "timestampColumn": "timestampcolumn", "watermark": "watermark",
            "timeWindows": _scoped("timewindow", {"windowDuration": "windowduration"}),
            "jarUDFs": _scoped("jar.udf", _jar()),
            "jarUDAFs": _scoped("jar.udaf", _jar()),
            "hipUDFs": _scoped("hipudf", {"source": "source", "entry": "entry", "returnType": "returntype",
                                          "argTypes": {"type": "stringList", "namespace": "argtypes"},
                                          "nullSafe": "nullsafe"}),
            "hipUDAFs": _scoped("hipudaf", {"source": "source", "prefix": "prefix", "returnType": "returntype",
                                            "argTypes": {"type": "stringList", "namespace": "argtypes"},
                                            "nullSafe": "nullsafe"}),
            "accumulationTables": _scoped("statetable", {"schema": "schema", "location": "location"}),
            "azureFunctions": _scoped("azurefunction", {
                "serviceEndpoint": "serviceendpoint", "api": "api", "code": "code", "methodType": "methodtype",
                "params": {"type": "stringList", "namespace": "params"}}),
            "appendEventTags": {"type": "mapProps", "namespace": "appendproperty"},
        }},
        "output": {"type": "scopedObject", "namespace": "output", "namespaceField": "name",
                   "fields": _output_fields()},
        "outputs": {"type": "array", "element": {"type": "scopedObject", "namespace": "output",
                                                 "namespaceField": "name", "fields": _output_fields()}},
    },
}
