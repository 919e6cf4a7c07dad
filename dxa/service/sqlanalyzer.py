"""SQL analyser for the query editor's intellisense: table name → columns for every statement of a transform
(reference: Services/DataX.Flow/DataX.Flow.SqlParser/SqlParser.cs:15-391 — regex-based there; here the real parser
computes each view's output columns, expanding ``*`` / ``t.*`` / ``Raw.*`` against the input schema)."""
from __future__ import annotations

import json
from typing import Dict, List, Optional

from ..engine.types import StructType, schema_from_json
from ..sql import ast as A
from ..sql.codegen import generate_code
from ..sql.parser import SqlError, parse_query
from ..sql.transform import parse_transform


def _struct_columns(st: StructType, prefix=()) -> List[str]:
    out = []
    for f in st.fields:
        out.append(".".join(prefix + (f.name,)))
        if isinstance(f.dtype, StructType):
            out += _struct_columns(f.dtype, prefix + (f.name,))
    return out


def analyze(code: str, input_schema: Optional[str] = None, projection: Optional[List[str]] = None,
            rules: str = "[]") -> Dict[str, List[str]]:
    tables: Dict[str, List[str]] = {}
    base: List[str] = []
    if input_schema:
        st = schema_from_json(input_schema)
        base = list(dict.fromkeys(_struct_columns(st)))
    tables["DataXProcessedInput"] = base
    code = generate_code(code, rules).code
    for cmd in parse_transform(code).commands:
        if not cmd.name:
            continue
        try:
            q = parse_query(cmd.text)
        except SqlError:
            tables[cmd.name] = []
            continue
        tables[cmd.name] = _columns(q.body, tables)
    return tables


def _columns(body, tables) -> List[str]:
    if isinstance(body, A.SetOp):
        return _columns(body.left, tables) if body.left is not None else []
    if isinstance(body, A.Query):
        return _columns(body.body, tables)
    out = []
    src_cols: List[str] = []
    for ref in _table_refs(body.from_):
        name = ref.name if not ref.timewindow else "DataXProcessedInput"
        src_cols += tables.get(name, tables.get(name.split("_")[0], []))
    for it in body.items:
        e = it.expr
        if isinstance(e, A.Star):
            top = [c for c in src_cols if "." not in c]
            if e.qualifier and not any(e.qualifier[0].lower() == r.name.lower() or
                                       e.qualifier[0].lower() == (r.alias or "").lower()
                                       for r in _table_refs(body.from_)):
                prefix = ".".join(e.qualifier) + "."
                top = [c[len(prefix):] for c in src_cols if c.startswith(prefix) and "." not in c[len(prefix):]]
            out += top
            continue
        from ..engine.expr import output_name
        out.append(it.alias or output_name(e))
    return out


def _table_refs(src):
    if src is None:
        return []
    if isinstance(src, A.TableRef):
        return [src]
    if isinstance(src, A.Join):
        return _table_refs(src.left) + _table_refs(src.right)
    return []
