"""Schema inference: sample JSON events → union Spark ``StructType`` JSON + conflict report.

Reference: Services/DataX.Flow/DataX.Flow.SchemaInference/Engine.cs:13-312 — every event's shape is merged into one
struct; a key whose values have different JSON types is reported as a conflict ("Conflict in schema. Key with path
'…' has different types") and the first type is kept; empty arrays default to array<string>.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional, Tuple


def _leaf_type(v) -> str:
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, int):
        return "long"
    if isinstance(v, float):
        return "double"
    return "string"


class SchemaInferrer:
    def __init__(self):
        self.errors: List[str] = []

    def _conflict(self, path: str):
        msg = f"Conflict in schema. Key with path '{path}' has different types"
        if msg not in self.errors:
            self.errors.append(msg)

    def _merge(self, cur, v, path: str):
        """cur: existing type node (None = unseen); returns merged node."""
        if v is None:
            return cur if cur is not None else {"__null__": True}
        if isinstance(v, dict):
            if cur is None or cur == {"__null__": True}:
                cur = {"type": "struct", "fields": {}}
            if not (isinstance(cur, dict) and cur.get("type") == "struct"):
                self._conflict(path)
                return cur
            for k, x in v.items():
                cur["fields"][k] = self._merge(cur["fields"].get(k), x, f"{path}.{k}" if path else k)
            return cur
        if isinstance(v, list):
            if cur is None or cur == {"__null__": True}:
                cur = {"type": "array", "elementType": None}
            if not (isinstance(cur, dict) and cur.get("type") == "array"):
                self._conflict(path)
                return cur
            for x in v:
                cur["elementType"] = self._merge(cur["elementType"], x, path + ".array")
            return cur
        t = _leaf_type(v)
        if cur is None or cur == {"__null__": True}:
            return t
        if cur != t:
            if {cur, t} == {"long", "double"} if isinstance(cur, str) else False:
                return "double"
            self._conflict(path)
        return cur

    def infer(self, events: List[Any]) -> Tuple[Dict, List[str]]:
        root = None
        for e in events:
            if isinstance(e, (str, bytes)):
                try:
                    e = json.loads(e)
                except ValueError:
                    self.errors.append("Invalid JSON event skipped")
                    continue
            root = self._merge(root, e, "")
        return _to_spark(root if root is not None else {"type": "struct", "fields": {}}), self.errors


def _to_spark(node):
    if node is None or node == {"__null__": True}:
        return "string"
    if isinstance(node, str):
        return node
    if node["type"] == "struct":
        return {"type": "struct", "fields": [{"name": k, "type": _to_spark(v), "nullable": True, "metadata": {}}
                                             for k, v in node["fields"].items()]}
    return {"type": "array", "elementType": _to_spark(node["elementType"]), "containsNull": True}


def infer_schema(events: List[Any]) -> Dict[str, Any]:
    schema, errors = SchemaInferrer().infer(events)
    return {"Schema": json.dumps(schema), "Errors": errors}
