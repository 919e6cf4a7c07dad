"""LiveQuery: interactive kernels that run DataX-SQL against sample data of a flow (the reference's
InteractiveQueryManager / KernelService — Services/DataX.Flow/DataX.Flow.InteractiveQuery/KernelService.cs:28-852).

A kernel is created from a flow's GUI definition: the input schema, normalisation snippet (projection), reference
data and functions are loaded; sample events (uploaded, or generated from the schema by the GPU generator) are
parsed and projected into ``DataXProcessedInput``.  ``execute`` follows the reference's rules: a leading
``--DataXQuery--`` is dropped, ``TIMEWINDOW(…)`` is stripped, ``… WITH UPSERT t`` becomes ``t = …``, ``T = SELECT …``
registers view ``T``, ``CREATE TABLE`` registers an empty state table, and at most ``max_rows`` JSON rows come back.
Kernels run in-process on the service's device (GPU when present): a query over the sample is a few milliseconds.
"""
from __future__ import annotations

import json
import re
import threading
import time
import uuid
from typing import Any, Dict, List, Optional

import torch

from ..config.settings import SettingDictionary
from ..engine.column import Table
from ..engine.expr import EvalContext
from ..engine.processor import RawBatch
from ..engine.query import Catalog, run_sql
from ..engine.serialize import table_to_json_lines
from ..engine.types import parse_ddl_schema, schema_from_json
from ..ops.jsonparse import ParsePlan, frame_records, parse
from ..sql.parser import parse_query

QUERY_SEPARATOR = "--DataXQuery--"


class KernelError(Exception):
    pass


class Kernel:
    def __init__(self, kernel_id: str, gui: Dict[str, Any], device, sample_events: Optional[List[str]] = None,
                 sample_size: int = 200, max_rows: int = 100):
        self.id = kernel_id
        self.gui = gui
        self.device = torch.device(device)
        self.max_rows = max_rows
        self.created = time.time()
        self.lock = threading.Lock()
        props = gui.get("input", {}).get("properties", {})
        self.schema = schema_from_json(props["inputSchemaFile"])
        snippet = props.get("normalizationSnippet") or "Raw.*"
        self.projection = [l.strip() for l in snippet.replace("\r\n", "\n").split("\n") if l.strip()]
        from ..udf.registry import build_udfs
        self.udfs, self.udafs, _ = build_udfs(self._function_settings(), {}, {})
        self.catalog = Catalog()
        self.warnings: List[str] = []
        self._load_reference_data()
        self.refresh(sample_events, sample_size)

    def _function_settings(self) -> SettingDictionary:
        d = {}
        for f in self.gui.get("process", {}).get("functions") or []:
            p = f.get("properties") or {}
            t = (f.get("type") or "").lower()
            if t == "jarudf":
                d[f"datax.job.process.jar.udf.{f['id']}.class"] = p.get("class", "")
            elif t == "jarudaf":
                d[f"datax.job.process.jar.udaf.{f['id']}.class"] = p.get("class", "")
            elif t == "azurefunction":
                base = f"datax.job.process.azurefunction.{f['id']}."
                d[base + "serviceendpoint"] = p.get("serviceEndpoint", "")
                d[base + "api"] = p.get("api", "")
                d[base + "code"] = p.get("code", "")
                d[base + "methodtype"] = p.get("methodType", "get")
                d[base + "params"] = ";".join(p.get("params") or [])
        return SettingDictionary(d)

    def _load_reference_data(self):
        from ..io.refdata import load_csv
        for rd in self.gui.get("input", {}).get("referenceData") or []:
            p = rd.get("properties") or {}
            try:
                self.catalog.register(rd["id"], load_csv(p["path"], p.get("delimiter", ","),
                                                         str(p.get("header", True)).lower() == "true", self.device))
            except OSError as e:
                self.warnings.append(f"reference data {rd['id']} not loaded: {e}")

    def refresh(self, sample_events: Optional[List[str]] = None, sample_size: int = 200):
        if sample_events is None:
            from ..simulate.datagen import compile_spark, generate
            buf, offs = generate(compile_spark(self.schema), sample_size, self.device, seed=int(time.time()))
        else:
            buf, offs = frame_records([e.encode() if isinstance(e, str) else e for e in sample_events],
                                      device=self.device)
        raw, _ = parse(buf, offs, ParsePlan(self.schema))
        n = int(offs.shape[0]) - 1
        from ..engine.column import ConstColumn
        from ..engine.types import MapType
        mt = MapType("string", "string")
        t = Table(["Raw", "Properties", "SystemProperties"],
                  [raw, ConstColumn({}, mt, n, self.device), ConstColumn({}, mt, n, self.device)], n, self.device)
        cat = Catalog()
        cat.register("__input", t)
        ctx = self._ctx()
        projected = run_sql("SELECT " + ", ".join(self.projection) + " FROM __input", cat, ctx)
        for name in ("DataXProcessedInput", "DataXProcessedInput_Batch", "DataXProcessedInput_Window"):
            self.catalog.register(name, projected)
        self.sample = projected

    def _ctx(self):
        return EvalContext(now_us=int(time.time() * 1e6), udfs=self.udfs, udafs=self.udafs, device=self.device)

    def execute(self, code: str) -> List[str]:
        if not code or not code.strip():
            raise KernelError("Please select a query in the UI")
        code = code.strip()
        if code.startswith(QUERY_SEPARATOR):
            code = code.replace(QUERY_SEPARATOR, "")
        code = re.sub(r"TIMEWINDOW\s*\(\s*.*?\s*\)", "", code, count=1, flags=re.I)
        m = re.search(r"\s*([^;]*)WITH\s+UPSERT\s*([^;]*)", code, re.I)
        if m:
            code = code.replace(m.group(0), m.group(2).strip() + " = " + m.group(1).strip())
        code = code.strip().rstrip(";").strip()
        with self.lock:
            m3 = re.match(r"\s*CREATE TABLE\s+(\w+)\s*\((.*)\)\s*$", code, re.I | re.S)
            if m3:
                if m3.group(1) not in self.catalog:
                    self.catalog.register(m3.group(1), Table.empty(parse_ddl_schema(m3.group(2)), self.device))
                return ["done"]
            m2 = re.match(r"^\s*([A-Za-z_][A-Za-z0-9_]*)\s*=(.*)$", code, re.S)
            if m2:
                t = run_sql(m2.group(2), self.catalog, self._ctx())
                self.catalog.register(m2.group(1), t)
            else:
                t = run_sql(code, self.catalog, self._ctx())
            return table_to_json_lines(t.slice(0, self.max_rows))

    def sample_input(self, n: Optional[int] = None) -> List[str]:
        return table_to_json_lines(self.sample.slice(0, n or self.max_rows))


class KernelManager:
    def __init__(self, device="cpu", max_kernels: int = 64):
        self.device = device
        self.kernels: Dict[str, Kernel] = {}
        self.max_kernels = max_kernels
        self.lock = threading.Lock()

    def create(self, gui: Dict[str, Any], sample_events: Optional[List[str]] = None, **kw) -> str:
        kid = uuid.uuid4().hex
        k = Kernel(kid, gui, self.device, sample_events, **kw)
        with self.lock:
            if len(self.kernels) >= self.max_kernels:
                oldest = min(self.kernels.values(), key=lambda x: x.created)
                self.kernels.pop(oldest.id, None)
            self.kernels[kid] = k
        return kid

    def get(self, kid: str) -> Kernel:
        k = self.kernels.get(kid)
        if k is None:
            raise KernelError(f"kernel {kid} not found")
        return k

    def delete(self, kid: str) -> bool:
        with self.lock:
            return self.kernels.pop(kid, None) is not None

    def delete_all(self):
        with self.lock:
            self.kernels.clear()
