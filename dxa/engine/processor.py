"""The micro-batch executor: raw events → projected table → windowed views / state tables / transform SQL →
outputs + metrics.  This is the reference's ``CommonProcessorFactory`` (DataProcessing/datax-host/src/main/scala/
datax/processor/CommonProcessorFactory.scala:42-660) re-designed for one MI355X per process:

* the raw batch arrives as ONE device byte buffer + record offsets (``RawBatch``); JSON parsing, projection,
  every transform statement and the window/state bookkeeping run on device columns;
* views are materialised once per batch and dropped at batch end (the reference caches views referenced more than
  once — every view here is already materialised, so that is free);
* outputs serialise on the host thread pool; metrics use the reference's names (``Input_DataXProcessedInput_Events_
  Count``, ``Latency-Process``, ``Latency-Batch``, ``Output_<name>_Sink_*``);
* multi-GPU: ``dxa.parallel`` hooks the group-by / distinct / join operators with RCCL exchanges (see
  ``dxa.parallel.distributed``) — the processor itself is rank-local.
"""
from __future__ import annotations

import collections
import copy
import datetime as _dt
import json
import logging
import os
import re
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch

from .. import parallel as P
from ..config import settings as S
from ..config.secrets import resolve
from ..io import fs
from ..ops.jsonparse import ParsePlan, parse, parse_async
from ..sql.transform import COMMAND_COMMAND, parse_transform
from .column import ConstColumn, DeferredTable, PrimColumn, StructColumn, Table, concat_tables
from .expr import EvalContext, EvalError
from .query import Catalog, _run_prefilters, execute, filter_readers, prefilter, prefilter_result, run_sql
from .serialize import table_to_json_lines
from .state import create_state_tables
from .types import MapType, StructType, schema_from_json
from .windows import TimeWindowConf, WindowStore
from ..telemetry import tracing

log = logging.getLogger("dxa.processor")
_SYNC_STAGES = os.environ.get("DXA_SYNC_STAGES") == "1"


@dataclass
class RawBatch:
    """One micro-batch of raw event payloads resident on the device.  The JSON parse un-escapes string values in
    place (json_parse.hip), so a batch's bytes are consumed by its one parse: re-processing needs fresh bytes."""
    buf: torch.Tensor            # uint8, 16-byte padded
    offs: torch.Tensor           # int64 [n+1]
    n: int
    properties: Optional[Any] = None          # per-event Properties map column (or None → {})
    system_properties: Optional[Any] = None   # per-event SystemProperties map column (or None → {})
    file_info: Optional[Dict[str, Any]] = None
    source_bytes: int = 0
    ends: Optional[torch.Tensor] = None       # int64 [n] record ends when records are not back to back (Kafka
                                              # values in decompressed record batches); offs[n] = end of the bytes
    pending: Optional[Any] = None             # jsonparse.PendingParse started by Processor.prepare
    status: Optional[Any] = None              # source-side decode status (kafka_device.DecodeStatus), checked by
                                              # process_batch before the transform (no row of a corrupt batch
                                              # reaches a sink or an accumulator)
    file_rows: Optional[List[Tuple[Dict[str, str], int]]] = None   # per-file FileInternal + its row count, in row
                                              # order (blob-pointer batches: the FileInfo column varies per row)
    source_metrics: Optional[Dict[str, float]] = None   # e.g. InputBlobs / Latency-Blobs, merged into the batch's


def _read_lines(path: str) -> List[str]:
    return fs.read_lines(resolve(path))


class Processor:
    def __init__(self, settings: S.SettingDictionary, device="cpu", metric_store=None, udfs=None, udafs=None,
                 normalizer=None, pre_projection=None, parse_prune: bool = True,
                 pipeline_outputs: Optional[bool] = None):
        self.settings = settings
        self.device = torch.device(device)
        self.name = settings.job_name()
        d = settings
        # ---- input schema + projection + transform
        schema_ref = d.get(S.INPUT_PREFIX + "blobschemafile")
        if schema_ref is None:
            raise S.SettingError("datax.job.input.default.blobschemafile is required")
        schema_text = resolve(schema_ref)
        if not schema_text.lstrip().startswith("{"):
            schema_text = fs.read_text(schema_text)
        self.raw_schema: StructType = schema_from_json(schema_text)
        self.projections: List[List[str]] = []
        for p in d.get_string_seq(S.PROCESS_PREFIX + "projection") or []:
            lines = [l.strip().rstrip(",") for l in _read_lines(p) if l.strip() and not l.strip().startswith("--")]
            self.projections.append([l.lstrip("﻿") for l in lines])
        self.transform = None
        tpath = d.get(S.PROCESS_PREFIX + "transform")
        if tpath:
            self.transform = parse_transform(_read_lines(tpath))
        self.windows = TimeWindowConf.from_settings(d)
        self.window_store = WindowStore(self.windows) if self.windows.enabled else None
        # ---- independent initialisers run concurrently, as the reference's init futures on an 8-thread pool
        # (CommonProcessorFactory.scala:43-44,58-73): UDF builds (hipRTC compiles of HIP UDFs, plugin imports) and
        # sink construction (connections, logins) overlap each other and the state-table restore and reference-data
        # load, which stay on this thread in this order (at N ranks both run collectives — a restart's key
        # reshuffle, the reference broadcast — whose order must match on every rank).  The first failure is
        # re-raised (the reference's failFast).
        from concurrent.futures import ThreadPoolExecutor
        from ..udf.registry import build_udfs
        from ..io.sinks import build_outputs
        init_pool = ThreadPoolExecutor(max_workers=2, thread_name_prefix="dxa-init")
        f_udfs = init_pool.submit(build_udfs, d, udfs or {}, udafs or {})
        f_outputs = init_pool.submit(build_outputs, d)
        try:
            self.state_tables = create_state_tables(d, self.device)
            self.udfs, self.udafs, self.udf_refreshers = f_udfs.result()
        except BaseException:
            init_pool.shutdown(wait=True, cancel_futures=True)
            raise
        from ..udf.registry import _instantiate
        if normalizer is None and d.get(S.PROCESS_PREFIX + "inputnormalizer"):
            normalizer = _instantiate(d.get(S.PROCESS_PREFIX + "inputnormalizer"))          # InputNormalizerHandler
        if pre_projection is None and d.get(S.PROCESS_PREFIX + "preprojection"):
            pp = _instantiate(d.get(S.PROCESS_PREFIX + "preprojection"))                    # PreProjectionHandler
            init = getattr(pp, "initialize", None)
            pp = init(d) if init is not None else pp
            pre_projection = pp if callable(pp) and not hasattr(pp, "process") else pp.process
        self.normalizer = normalizer
        self.pre_projection = pre_projection
        self.append_props = {k: v for k, v in d.sub_dictionary(S.PROCESS_PREFIX + "appendproperty.").items()}
        # ---- reference data (resident across batches: stream–static joins build their hash tables once)
        try:
            self.reference: Dict[str, Table] = self._load_reference_data()
            # ---- outputs + metrics
            self.outputs = f_outputs.result()
        finally:
            init_pool.shutdown(wait=True)
        from ..telemetry.metrics import MetricLogger
        self.metric_logger = MetricLogger.from_settings(d, metric_store)
        # column pruning (datax.job.process.columnpruning, default on): the parser extracts and windows retain only
        # the raw fields the live statements can read
        parse_prune = parse_prune and d.get_bool(S.PROCESS_PREFIX + "columnpruning", True)
        self.parse_plan = ParsePlan(self.raw_schema, self._needed_raw_paths() if parse_prune else None,
                                    ts_shadow=self._string_to_ts_paths())
        # input rebalance across ranks (reference: datax.job.input.default.eventhub.repartition → rdd.repartition)
        rp = d.get(S.INPUT_PREFIX + "eventhub.repartition") or d.get(S.INPUT_PREFIX + "repartition")
        self.repartition = bool(rp) and rp.strip().lower() not in ("0", "false", "")
        self.batches = 0
        self.last_metrics: Dict[str, float] = {}
        self.last_views: Dict[str, Table] = {}
        self.keep_views = False
        self.stage_times: Dict[str, float] = {}
        # host wall time per phase / statement, summed over batches (no device syncs): where the planning thread
        # spends a batch (bench.py --profile-stages prints it per step)
        self.host_acc: Dict[str, float] = collections.defaultdict(float)
        self._t_route_end = self._c_route_end = 0.0
        self._parsed: Dict[str, object] = {}
        # output pipelining: batch t's sink work overlaps batch t+1's device work (at most one batch in flight)
        self.pipeline_outputs = pipeline_outputs if pipeline_outputs is not None else \
            d.get_bool(S.PROCESS_PREFIX + "pipelineoutputs", False)
        # batches whose outputs may be in flight at once (datax.job.process.outputdepth, env DXA_OUTPUT_DEPTH): 1 =
        # batch t's sinks overlap batch t+1's processing only.  2 also overlaps batch t's D2H / sink writes with
        # batch t+1's rendering — for flows bound by the output copy (every event re-serialised); batches still
        # complete (metrics, state flips, offset commits) in order, but sinks of consecutive batches may finish
        # out of order
        depth = os.environ.get("DXA_OUTPUT_DEPTH") or d.get_or_else(S.PROCESS_PREFIX + "outputdepth", "1") or "1"
        self.output_depth = max(1, int(depth))
        self._inflights: "collections.deque[_InFlight]" = collections.deque()
        self.completed: List = []
        self.on_batch_complete = None
        self.source_metric_names: Tuple[str, ...] = ()
        self.clock: Callable[[], float] = time.time     # current_timestamp() of a batch (tests pin it)

    # ------------------------------------------------------------------------------------------------------------
    def _load_reference_data(self) -> Dict[str, Table]:
        """``datax.job.input.default.referencedata.<name>.{path,format,delimiter,header}`` (ReferenceDataHandler.scala:
        42-60) → resident device tables; ``schema`` (DDL) types columns at load (an extension: Spark reads strings).
        Load statistics land in ``reference_stats``."""
        out = {}
        self.reference_stats: Dict[str, Dict[str, float]] = {}
        for name, sub in self.settings.group_by_sub_namespace(S.INPUT_PREFIX + "referencedata.").items():
            fmt = (sub.get("format") or "csv").lower()
            path = resolve(sub.get_string("path"))
            if fmt not in ("csv", "tsv"):
                raise ValueError(f"unsupported reference data format {fmt}")
            from ..io.refdata import load_csv
            stats: Dict[str, float] = {}
            out[name] = load_csv(path, sub.get("delimiter") or ("\t" if fmt == "tsv" else ","),
                                 (sub.get("header") or "true").lower() == "true", self.device,
                                 schema=sub.get("schema"), stats=stats)
            self.reference_stats[name] = stats
        return out

    def _string_to_ts_paths(self) -> set:
        """Raw string fields a projection line feeds to ``stringToTimestamp`` (the IoT flows' eventTime): the parser
        converts them while their bytes are in cache, and ``stringToTimestamp`` takes that column (dxa_ts.h, the
        same grammar as the string kernel)."""
        import re
        out = set()
        for t in (l for p in self.projections for l in p):
            for m in re.finditer(r"stringToTimestamp\s*\(\s*Raw((?:\s*\.\s*[A-Za-z_`][A-Za-z0-9_`]*)+)\s*\)", t,
                                 flags=re.I):
                out.add(tuple(p.strip().strip("`") for p in m.group(1).split(".") if p.strip()))
        return out

    def _needed_raw_paths(self):
        """Projection pushdown into the JSON parser: which ``Raw`` leaves can any statement reference?

        Conservative: if any projection line / statement / output could see the whole Raw struct (``Raw``,
        ``Raw.*`` followed by ``*`` downstream, to_json of rows, …) we keep everything."""
        import re
        texts = [l for p in self.projections for l in p]
        if not texts:
            return None
        if any(re.search(r"\bRaw\s*\.\s*\*", t) for t in texts):
            # Raw.* expands every field into the projected table: keep all leaves unless SQL proves otherwise
            return self._raw_paths_read_by_sql(texts)
        keep = set()
        for t in texts:
            for m in re.finditer(r"\bRaw((?:\s*\.\s*[A-Za-z_`][A-Za-z0-9_`]*)+)", t):
                parts = tuple(p.strip().strip("`") for p in m.group(1).split(".") if p.strip())
                keep.add(parts)
            if re.search(r"\bRaw\b(?!\s*\.)", t):
                return None
        return keep or None

    def _raw_paths_read_by_sql(self, projection_texts) -> Optional[set]:
        """Column pruning through ``Raw.*``: the Raw leaves any live transform statement can read.

        With ``Raw.*`` every JSON field becomes a column of ``DataXProcessedInput``, but only the columns some
        consumer reads can reach an output.  Demand runs backwards over the live statements: an output or an
        accumulator needs all of its view; a statement needs, from every relation it reads, the identifiers it
        names — plus, where it selects ``*``, whatever its own consumers need (so an alert view ``SELECT *, … FROM
        DataXProcessedInput WHERE …`` read only by ``SELECT DISTINCT <constants> FROM it`` adds nothing).  The
        demand on the input views is matched against the raw schema's paths (at any offset: ``Raw.a.b``, ``a.b``,
        ``t.a.b`` all name ``a.b``; a struct named whole keeps its subtree); the parser then extracts only those
        fields and windows retain only those columns.  Over-keeping is harmless; anything the analysis cannot see
        (``*`` reaching an output, hooks, unparsable text) keeps everything."""
        if self.transform is None or self.pre_projection is not None or self.normalizer is not None:
            return None
        from ..sql import ast as A
        from ..sql.parser import parse_expression, parse_query
        base = f"{S.NAME_PREFIX}ProcessedInput".lower()
        ALL = None
        demand: Dict[str, Optional[set]] = {}
        for op in self.outputs:
            demand[op.name.lower()] = ALL
        for n in self.state_tables:
            demand[n.lower()] = ALL
        live = self._live_statements()
        cmds = self.transform.commands
        for k in range(len(cmds) - 1, -1, -1):
            c = cmds[k]
            if c.command_type == COMMAND_COMMAND or (live is not None and k not in live):
                continue
            try:
                q = parse_query(c.text)
            except Exception:  # noqa: BLE001 — statements the parser rejects fail later, loudly
                return None
            nodes = list(_ast_nodes(q))
            own = demand.get(c.name.lower(), set())
            ids = {tuple(p.lower() for p in n.parts) for n in nodes if isinstance(n, A.Ident)}
            star = any(isinstance(n, A.Star) for n in nodes)
            need = ALL if (star and own is ALL) else (ids | (own if star else set()))
            for r in {n.name.lower() for n in nodes if isinstance(n, A.TableRef)}:
                if r == c.name.lower():
                    continue
                cur = demand.get(r, set())
                demand[r] = ALL if (cur is ALL or need is ALL) else cur | need
        idents = []
        for name, d in demand.items():
            if name == base or name.startswith(base + "_") or name in {w.lower() for w in self.windows.windows}:
                if d is ALL:
                    return None
                idents += list(d)
        # columns the job's settings name rather than its SQL: the window timestamp column (WindowStore reads it
        # from every batch, TimeWindowHandler.scala:41-67) must survive pruning even when no statement names it
        ts_col = getattr(self.windows, "timestamp_column", None)
        if ts_col:
            idents.append(tuple(p.strip().strip("`") for p in str(ts_col).split(".")))
        for t in projection_texts:
            if re.match(r"^\s*Raw\s*\.\s*\*\s*$", t):
                continue
            try:
                e = parse_expression(re.sub(r"\s+AS\s+`?[A-Za-z_][A-Za-z0-9_]*`?\s*$", "", t, flags=re.I))
            except Exception:  # noqa: BLE001
                return None
            idents += [n.parts for n in A.walk(e) if isinstance(n, A.Ident)]
        tree = _schema_tree(self.raw_schema)
        keep = set()
        for parts in idents:
            low = [p.lower() for p in parts]
            for i in range(len(low)):
                node, path = tree, ()
                for p in low[i:]:
                    if node is None or p not in node:
                        break
                    name, node = node[p]
                    path += (name,)
                if path:
                    keep.add(path)
        return keep or None

    # ------------------------------------------------------------------------------------------------------------
    def prepare(self, raw: RawBatch, stream=None) -> RawBatch:
        """Queue the batch's JSON parse now, so that ``project`` finds the per-field null counts already on the
        host instead of waiting for the parse.  A no-op off the GPU and with an input normalizer (which rewrites
        the bytes first).

        ``stream=None``: on the current stream (call it right after the previous batch's ``process_batch``; the
        parse then runs behind that batch's kernels).  A side ``stream`` (its own parse stream, already ordered after
        the batch's ingest): call it BEFORE the previous batch's ``process_batch`` — the parse then overlaps that
        batch's query kernels, which leave most of the chip idle (profiles/round4: the ``full`` flow's kernels keep
        the GPU busy ~35 % of the step), and ``project`` no longer waits a whole parse per batch."""
        if raw.pending is None and self.normalizer is None and raw.buf.device.type == "cuda":
            with torch.inference_mode():
                self._prepare(raw, stream)
        return raw

    def _prepare(self, raw: RawBatch, stream) -> None:
        if stream is None:
            raw.pending = parse_async(raw.buf, raw.offs, self.parse_plan, raw.ends)
        else:
            with torch.cuda.stream(stream):
                raw.pending = parse_async(raw.buf, raw.offs, self.parse_plan, raw.ends)

    def project(self, raw: RawBatch, batch_time_us: int, ctx: EvalContext) -> Table:
        t0 = time.perf_counter()
        buf = raw.buf
        offs = raw.offs
        ends = raw.ends
        if self.normalizer is not None:
            if ends is not None:                  # normalizers take back-to-back records: pack the values first
                from .column import StrColumn
                starts = offs[:-1]
                packed = StrColumn(buf, starts, (ends - starts).to(torch.int32)).compact()
                buf = packed.arena
                offs = torch.cat([packed.starts, (packed.starts[-1:] + packed.lens[-1:].to(torch.int64))
                                  if raw.n else torch.zeros(1, dtype=torch.int64, device=buf.device)])
                ends = None
            buf, offs = self.normalizer(buf, offs)
        with tracing.stage("parse"):
            if raw.pending is not None and self.normalizer is None:
                raw_col, row_ok = raw.pending.result()
                raw.pending = None
            else:
                raw_col, row_ok = parse(buf, offs, self.parse_plan, ends)
        self._sync()
        self.stage_times["parse"] = time.perf_counter() - t0
        n = raw.n
        dev = self.device
        empty_map = MapType("string", "string")
        props = raw.properties if raw.properties is not None else ConstColumn({}, empty_map, n, dev)
        sysprops = raw.system_properties if raw.system_properties is not None else ConstColumn({}, empty_map, n, dev)
        pp = dict(self.append_props)
        pp.update({"BatchTime": _fmt_ts(batch_time_us), "CPTime": _fmt_ts(int(time.time() * 1e6)),
                   "CPExecutor": str(torch.cuda.current_device() if dev.type == "cuda" else "driver")})
        if raw.file_info:
            pp["InputTime"] = str(raw.file_info.get("fileTime", ""))
            pp["Partition"] = str(raw.file_info.get("outputFileName", ""))
        names = ["Raw", "Properties", "SystemProperties", f"{S.NAME_PREFIX}Properties"]
        internal = f"__{S.NAME_PREFIX}_"
        targets = {i.get("target") for i, _c in raw.file_rows or []} or {(raw.file_info or {}).get("target")}
        self._batch_target = next(iter(targets)) if len(targets) == 1 else None      # ${target} of blob outputs
        self._source_metrics = dict(raw.source_metrics or {})
        if raw.file_rows:
            # one FileInternal per file: per-row map columns gathered from a k-row table (k = files)
            from .column import column_from_pylist
            infos = [dict(i) for i, _c in raw.file_rows]
            idx = torch.repeat_interleave(torch.arange(len(infos), device=dev),
                                          _h2d([c for _i, c in raw.file_rows], torch.int64, dev))
            pps = [dict(pp, InputTime=str(i.get("fileTime", "")), Partition=str(i.get("outputFileName", "")))
                   for i in infos]
            cols = [raw_col, props, sysprops, column_from_pylist(pps, empty_map, dev).take(idx)]
            names.append(f"{internal}FileInfo")
            cols.append(column_from_pylist(infos, empty_map, dev).take(idx))
        else:
            cols = [raw_col, props, sysprops, ConstColumn(pp, empty_map, n, dev)]
            if raw.file_info:
                names.append(f"{internal}FileInfo")
                cols.append(ConstColumn(dict(raw.file_info), empty_map, n, dev))
        table = Table(names, cols, n, dev)
        if self.pre_projection is not None:
            table = self.pre_projection(table, ctx)
        for step in self.projections:
            preserved = [nm for nm in table.names if nm.startswith(internal)]
            cat = Catalog()
            cat.register("__dxa_input", table)
            items = step + [f"`{p}`" for p in preserved if not any(p in s for s in step)]
            table = run_sql("SELECT " + ", ".join(items) + " FROM __dxa_input", cat, ctx)
        if self.repartition and P.active():
            with tracing.stage("repartition", self.stage_times):
                table = P.rebalance_table(table)
        self._sync()
        self.stage_times["project"] = time.perf_counter() - t0
        return table

    def route(self, projected: Table, batch_time_us: int, interval_us: int, ctx: EvalContext,
              partition_time: _dt.datetime, t_start: Optional[float] = None) -> Dict[str, float]:
        t_start = time.perf_counter() if t_start is None else t_start
        metrics: Dict[str, float] = {}
        base = f"{S.NAME_PREFIX}ProcessedInput"
        cat = Catalog()
        for name, t in self.reference.items():
            t.static = True
            cat.register(name, t)
        cat._built = getattr(self, "_ref_built", {})
        self._ref_built = cat._built
        metrics["Input_Normalized_Events_Count"] = projected.length
        metrics.update(self._batch_source_metrics())
        part = P.PARTITIONED if P.active() else P.REPLICATED
        projected.dist = part
        if self.window_store is not None:
            tw = time.perf_counter()
            with tracing.stage("windows", self.stage_times):
                views, cnt = self.window_store.process(projected, batch_time_us, interval_us)
            self.host_acc["windows"] += time.perf_counter() - tw
            for k, v in views.items():
                v.dist = part
                cat.register(k, v)
            metrics[f"Input_{base}_Events_Count"] = cnt
        else:
            cat.register(base, projected)
            metrics[f"Input_{base}_Events_Count"] = projected.length
        for name, st in self.state_tables.items():
            cat.register(name, st.active)
        views: Dict[str, Table] = {}
        t0 = time.perf_counter()
        if self.transform is not None:
            live = None if self.keep_views else self._live_statements()
            cmds = self.transform.commands
            schedule = list(self._view_schedule(live))
            # windowed GROUP BYs may complete lazily (one rank, sequential views): see query._deferred_select
            defer_ok = self.device.type == "cuda" and not P.active() and not self._concurrent_views()
            readers = {}
            if self.device.type == "cuda":
                # the WHERE masks of statements over tables present now, with one count read for all of them
                # (command statements change nothing a predicate reads: _run_command)
                # with a window (sequential views): every such mask is queued right now, ahead of the windowed
                # statements' kernels (which the schedule starts first), so the count read finds them done
                eager = self.window_store is not None and not self._concurrent_views()
                with tracing.host_section("prefilter"):
                    prefilter([self._query(cmds[k]) for step in schedule for k in step
                               if cmds[k].command_type != COMMAND_COMMAND], cat, ctx, min_group=1 if eager else 2)
                    if eager:
                        for group in list(ctx.prefilter_cands.values()):
                            _run_prefilters(group, ctx)
                        ctx.prefilter_cands = {}
                if not self._concurrent_views():
                    # statements filtering a view this batch produces: their masks start when the view is registered
                    order = [k for step in schedule for k in step if cmds[k].command_type != COMMAND_COMMAND]
                    key = ("readers", tuple(order))
                    if getattr(self, "_readers", (None,))[0] != key:
                        self._readers = (key, filter_readers([(k, self._query(cmds[k])) for k in order], ctx))
                    readers = self._readers[1]
                    step_of = {k: i for i, k in enumerate(order)}
            for step in schedule:
                if len(step) > 1:
                    # independent views: each on a side HIP stream, forked from and joined back to this stream
                    results = self._run_concurrent([cmds[k] for k in step], cat, ctx)
                else:
                    cmd = cmds[step[0]]
                    if cmd.command_type == COMMAND_COMMAND:
                        self._run_command(cmd.text)
                        continue
                    ts = time.perf_counter()
                    q = self._query(cmd)
                    ctx.defer_dense = defer_ok and not (q.order_by or q.limit is not None or q.sort_by or
                                                        q.distribute_by)
                    with tracing.stage(f"sql:{cmd.name}"):
                        results = [execute(q, cat, ctx)]
                    ctx.defer_dense = False
                    self.host_acc[f"sql:{cmd.name}"] += time.perf_counter() - ts
                    if _SYNC_STAGES:
                        self._sync()
                        self.stage_times[f"sql:{cmd.name}"] = time.perf_counter() - ts
                for k, result in zip(step, results):
                    cmd = cmds[k]
                    st = self.state_tables.get(cmd.name)
                    if st is not None:
                        # the device-side state moves on now; the standby write waits for the previous batch's
                        # flip (StateTable.release in _complete_inflight), not this batch
                        with tracing.host_section("state:overwrite"):
                            result = st.overwrite(result, tag=batch_time_us)
                    cat.register(cmd.name, result)
                    views[cmd.name] = result
                    later = readers.get(cmd.name.lower()) if readers else None
                    if later and not isinstance(result, DeferredTable):
                        later = [r for r in later if step_of.get(r[0], -1) > step_of.get(k, -1)]
                        if later:
                            with tracing.host_section("prefilter"):
                                prefilter_result(result, later, ctx)
            with tracing.host_section("deferred:finish"):
                while ctx.pending:                  # results no later statement read: complete them now
                    d = ctx.pending.pop(0)
                    if isinstance(d, DeferredTable):
                        d.resolve()
        self._sync()
        self.stage_times["transform"] = time.perf_counter() - t0
        # outputs: device half staged here (filters + async D2H into pinned memory), host half (JSON rendering +
        # sink writes) on the output pool — pipelined, it overlaps the next batch's GPU work
        t1 = time.perf_counter()
        staged = []
        for op in self.outputs:
            t = views.get(op.name) or cat.get(op.name)
            if t is None:
                raise EvalError(f"could not find data set name '{op.name}' for output '{op.name}'")
            if P.active() and P.dist_of(t) == P.REPLICATED and P.rank() != 0:
                t = t.slice(0, 0)      # replicated results are written once, by rank 0
            staged.append((op.name, op.stage(t, ctx)))
        from ..ops.serialize import link_render_groups
        link_render_groups([p for _, st in staged for p in st.payloads()])    # one render launch pair per batch
        if self.window_store is not None:
            # the new pane's compaction: queued behind the statements AND the outputs' staging, so neither the
            # statements' status reads nor the outputs' renders wait for it
            self.window_store.settle()
        t2 = time.perf_counter()
        self.host_acc["outputs:stage"] += t2 - t1
        while len(self._inflights) >= self.output_depth:
            self._complete_inflight()
        t3 = time.perf_counter()
        self.host_acc["outputs:complete_previous"] += t3 - t2
        from ..io.sinks import _pool
        target = getattr(self, "_batch_target", None)
        local = [k for k, (_, st) in enumerate(staged) if st.op.local]
        futs = {}
        if len(local) > 1:
            together = _pool.submit(_finish_local, [staged[k][1] for k in local], partition_time, target)
            futs = {k: _Part(together, j) for j, k in enumerate(local)}
        fl = _InFlight(batch_time_us, metrics, [(name, futs.get(k) or _pool.submit(_timed, st.finish, partition_time,
                                                                                   target))
                                                for k, (name, st) in enumerate(staged)], t_start)
        fl.t_staged = time.perf_counter()
        fl.stages = dict(self.stage_times)
        self._inflights.append(fl)
        self.stage_times["output_stage"] = time.perf_counter() - t1
        self.host_acc["outputs:submit"] += fl.t_staged - t3
        if self.keep_views:
            self.last_views = {**{k: cat.get(k) for k in cat.names()}, **views}
        if not self.pipeline_outputs:
            while self._inflights:
                self._complete_inflight()
            self._sync()
            self.stage_times["output"] = time.perf_counter() - t1
        self._t_route_end = time.perf_counter()
        self._c_route_end = time.thread_time()
        return fl.metrics

    def declare_source_metrics(self, names) -> None:
        """The metric names the source may attach to a batch (``Source.metric_names``).  Every batch carries all of
        them — zero, or ``-inf`` for a latency (dropped after the reduction when no rank measured it) — so the key
        set every rank all-reduces does not depend on its data: an empty batch or a batch without file times on one
        rank still matches the others."""
        self.source_metric_names = tuple(names or ())

    def _batch_source_metrics(self) -> Dict[str, float]:
        got = dict(getattr(self, "_source_metrics", None) or {})
        declared = getattr(self, "source_metric_names", ())
        out = {k: (float("-inf") if P.is_max_metric(k) else 0.0) for k in declared}
        undeclared = sorted(set(got) - set(declared))
        if undeclared and P.active():
            raise EvalError(f"source metrics {undeclared} were not declared (Source.metric_names): at N ranks the "
                            f"batch metric key set must not depend on the data")
        out.update(got)
        return out

    def _query(self, cmd):
        q = self._parsed.get(cmd.text)
        if q is None:
            from ..sql.parser import parse_query
            q = self._parsed[cmd.text] = parse_query(cmd.text)         # parsed once, reused every batch
        return q

    def _concurrent_views(self) -> Optional[str]:
        """How independent views run (``datax.job.process.concurrentviews``, env ``DXA_VIEW_STREAMS``):
        ``None`` — one after another on the batch stream; ``"streams"`` — one after another on this thread, each on
        its own side HIP stream (a view's synchronising reads wait only for its own kernels, and its kernels overlap
        the next view's planning); ``"threads"`` — a worker thread per view as well (each thread's collectives on
        its own communicator at N ranks).  ``true`` selects ``streams``."""
        env = os.environ.get("DXA_VIEW_STREAMS")
        v = (env if env is not None else self.settings.get(S.PROCESS_PREFIX + "concurrentviews") or "false")
        v = v.strip().lower()
        if v in ("0", "false", "off", "no", ""):
            return None
        return "threads" if v == "threads" else "streams"

    def _view_schedule(self, live: Optional[set]) -> List[List[int]]:
        """The transform's statements as steps; a step of several statements runs them concurrently.

        Sequential mode: one statement per step, in text order.  Concurrent mode (the reference runs outputs and
        init work in parallel futures, CommonProcessorFactory.scala:43-73,114-117; here independent *views* also
        overlap, each on its own HIP stream): a statement's level is one more than the levels of the earlier
        statements whose names it reads (read-after-write) and of the earlier statements that read its own name
        (write-after-read: a statement that reads an accumulator's previous state runs before the accumulator is
        overwritten).  Steps run level by level; the views of a level run together, and accumulator (state-table)
        statements — whose overwrite completes the in-flight batch — run alone after them.  Commands (SET, CREATE
        TABLE) keep their place ahead of everything (they produce no view)."""
        key = ("sched", None if live is None else tuple(sorted(live)), self._concurrent_views())
        if getattr(self, "_sched", (None,))[0] == key:
            return self._sched[1]
        cmds = self.transform.commands
        if not key[2] and self.window_store is None:
            steps = [[k] for k, c in enumerate(cmds)
                     if c.command_type == COMMAND_COMMAND or live is None or k in live]
            self._sched = (key, steps)
            return steps
        import re
        level: Dict[str, int] = {}
        reads: List[Tuple[int, set]] = []
        lv: Dict[int, int] = {}
        commands = []
        # statements that read a time window directly run first in their level (a windowed GROUP BY completes lazily,
        # DeferredTable: its kernels start soonest), and the statements reading their results run last in theirs, so
        # the status read finds the kernels finished.  The WHERE masks over the batch's tables are queued before all
        # of it (route: prefilter), so their count reads do not wait for the window's kernels
        wnames = {"timewindow", f"{S.NAME_PREFIX}ProcessedInput_Window".lower()} | (
            {n.lower() for n in self.window_store.conf.windows} if self.window_store is not None else set())
        windowed: set = set()
        direct: set = set()
        for k, c in enumerate(cmds):
            if c.command_type == COMMAND_COMMAND:
                commands.append(k)
                continue
            if live is not None and k not in live:
                continue
            nm = c.name.lower()
            words = {w.lower() for w in re.findall(r"[A-Za-z_][A-Za-z0-9_]*", c.text)}
            lk = 0
            for w in words:
                if w in level and w != nm:
                    lk = max(lk, level[w] + 1)
            for j, wj in reads:
                if nm in wj:
                    lk = max(lk, lv[j] + 1)
            if nm in level:                       # a redefinition: after the earlier definition
                lk = max(lk, level[nm] + 1)
            lv[k] = lk
            level[nm] = lk
            reads.append((k, words))
            if words & wnames:
                direct.add(nm)
            if words & wnames or any(w in windowed and w != nm for w in words):
                windowed.add(nm)
        steps = [[k] for k in commands]
        for L in sorted(set(lv.values())):
            ks = [k for k in sorted(lv) if lv[k] == L]
            plain = [k for k in ks if cmds[k].name not in self.state_tables]
            if not key[2]:
                # windowed statements first (their kernels start soonest), their readers last; stable otherwise
                plain.sort(key=lambda k: 0 if cmds[k].name.lower() in direct else
                           2 if cmds[k].name.lower() in windowed else 1)
            if plain:
                # sequential mode with a window: one statement per step, level by level — a windowed statement's
                # readers run after the statements that do not read it, while its kernels finish (DeferredTable)
                steps += [plain] if key[2] else [[k] for k in plain]
            steps += [[k] for k in ks if cmds[k].name in self.state_tables]
        self._sched = (key, steps)
        return steps

    def _run_concurrent(self, cmds, cat, ctx) -> List[Table]:
        """Fork-join of independent views: each statement runs on its own side HIP stream (``threads`` mode: on a
        worker thread too).  The side streams first wait for this stream (the views' inputs), and this stream waits
        for every side stream before any result is used; so blocks a side stream allocates are reused only behind
        those waits.  Worker threads overlap one view's Python planning with another's synchronising reads (the GIL
        is released while a thread waits on the device) — measured slower than ``streams`` on the full flow
        (profiles/view_streams), as every PyTorch call hands the GIL over.  At N ranks branch ``i`` of a threaded
        level issues its collectives (key shuffles, broadcasts) on communicator ``i``, so every communicator sees
        the same sequence on every rank."""
        dev = self.device
        cuda = dev.type == "cuda"
        nslots = 4
        threads = self._concurrent_views() == "threads"
        if getattr(self, "_view_pool", None) is None:
            from concurrent.futures import ThreadPoolExecutor
            self._view_pool = ThreadPoolExecutor(max_workers=nslots, thread_name_prefix="dxa-view")
            self._view_streams = [torch.cuda.Stream(dev) for _ in range(nslots)] if cuda else []
        groups = P.branch_groups(nslots) if P.active() and threads else [None] * nslots
        main = torch.cuda.current_stream(dev) if cuda else None
        fork = None
        if cuda:
            fork = torch.cuda.Event()
            fork.record(main)
        times = self.stage_times

        def run(slot, cmd):
            import contextlib
            s = self._view_streams[slot] if cuda else None
            with contextlib.ExitStack() as es:
                if cuda:
                    torch.cuda.set_device(dev)
                    s.wait_event(fork)
                    es.enter_context(torch.cuda.stream(s))
                if groups[slot] is not None:
                    es.enter_context(P.use_branch(groups[slot]))
                ts = time.perf_counter()
                with tracing.stage(f"sql:{cmd.name}"):
                    # a context per branch: execute() swaps ctx.catalog for WITH / sub-query scopes
                    out = execute(self._query(cmd), cat, copy.copy(ctx))
                if _SYNC_STAGES and cuda:
                    s.synchronize()
                    times[f"sql:{cmd.name}"] = time.perf_counter() - ts
            return out

        for cmd in cmds:
            self._query(cmd)                      # parse on this thread (the cache is a plain dict)
        results, err = [], None
        if not threads:
            try:
                results = [run(i % nslots, cmd) for i, cmd in enumerate(cmds)]
            finally:
                if cuda:
                    for s in self._view_streams[:len(cmds)]:
                        main.wait_stream(s)
            return results
        for base in range(0, len(cmds), nslots):  # at most one branch per slot (stream, communicator) at a time
            chunk = cmds[base:base + nslots]
            futures = [self._view_pool.submit(run, i, cmd) for i, cmd in enumerate(chunk)]
            for f in futures:
                try:
                    results.append(f.result())
                except BaseException as e:  # noqa: BLE001 — join every branch before re-raising
                    err = err or e
            if err is not None:
                break
        if cuda:
            for s in self._view_streams[:len(cmds)]:
                main.wait_stream(s)
        if err is not None:
            raise err
        return results

    def _live_statements(self) -> Optional[set]:
        """Indices of the transform's query statements whose results can reach an output or a state table.
        Spark temp views are lazy: the reference registers each statement as ``spark.sql(statement)`` +
        ``createOrReplaceTempView`` (CommonProcessorFactory.scala:270-288) and only the outputs run actions
        (:297-305) and state tables write (:258-264), so a view that no output, accumulator or later live statement
        reads is never computed (the generated ``sa2_*`` copies, a ``Tagged`` view whose only consumers are the per-rule alert
        views, …), so skipping it changes no output.  Liveness runs backwards over the statements; a statement's
        reads are over-approximated by every statement name appearing as a word in its text."""
        if getattr(self, "_live", None) is not None:
            return getattr(self, "_live", None)
        import re
        cmds = self.transform.commands
        names = {c.name.lower() for c in cmds if c.command_type != COMMAND_COMMAND and c.name}
        needed = {op.name.lower() for op in self.outputs} | {n.lower() for n in self.state_tables}
        live = set()
        for k in range(len(cmds) - 1, -1, -1):
            c = cmds[k]
            if c.command_type == COMMAND_COMMAND or not c.name:
                continue
            nm = c.name.lower()
            if nm not in needed:
                continue
            live.add(k)
            needed.discard(nm)
            words = {w.lower() for w in re.findall(r"[A-Za-z_][A-Za-z0-9_]*", c.text)}
            needed |= (words & names) | ({nm} & words)
        self._live = live
        skipped = [c.name for k, c in enumerate(cmds) if c.command_type != COMMAND_COMMAND and k not in live]
        if skipped:
            log.info("views no output reads (not evaluated): %s", ", ".join(skipped))
        return live

    def _complete_inflight(self):
        """Finish the in-flight batch: collect sink counts, all-reduce the batch metrics across ranks, persist state
        tables (after outputs, as the reference), stamp latencies, emit metrics and fire ``on_batch_complete``."""
        if not self._inflights:
            return None
        fl = self._inflights.popleft()
        metrics = fl.metrics
        t_done = fl.t_staged
        for name, f in fl.futures:
            res, t_end = f.result()
            t_done = max(t_done, t_end)
            for k, v in res.items():
                metrics[f"Output_{name}_{k}"] = float(v)
        for st in self.state_tables.values():
            st.flush(fl.batch_time_us)  # this rank's standby part is durable before the all-reduce (= the barrier)
        # batch metrics are job-wide: counts summed, latencies maxed over ranks, key sets checked first (timings
        # stay per-rank)
        metrics = fl.metrics = P.reduce_metrics(metrics, self.device)
        flipped = False
        for st in self.state_tables.values():
            flipped |= st.persist(fl.batch_time_us)
        if flipped and P.active():
            # rank 0 flipped metadata.info just now: no rank may overwrite the copy the old metadata named (its next
            # standby) before that flip is on disk — the next batch's standby writes are ordered after this point
            P.order_point(self.device)
        for st in self.state_tables.values():
            st.release()               # the next batch's deferred standby writes may start
        metrics.update(tracing.stage_metrics(fl.stages))          # per-rank stage timings (not all-reduced)
        # processing latency = batch start → its last sink write finished (measured where the write finished, not
        # where the completion was observed)
        metrics["Latency-Process"] = t_done - fl.t0
        metrics["Latency-Batch"] = (time.time() * 1e6 - fl.batch_time_us) / 1e6
        self.last_done_perf = t_done            # perf_counter() when the batch's last sink write finished
        if P.rank() == 0:
            self.metric_logger.send_batch_metrics(metrics, fl.batch_time_us // 1000)
        self.last_metrics = metrics
        self.completed.append((fl.batch_time_us, metrics))
        del self.completed[:-64]
        if self.on_batch_complete is not None:
            self.on_batch_complete(fl.batch_time_us, metrics)
        return metrics

    def drain(self) -> Optional[Dict[str, float]]:
        """Complete the in-flight batch (pipelined mode); returns its metrics."""
        m = None
        while self._inflights:
            m = self._complete_inflight()
        self._sync()
        return m

    def _sync(self):
        """Stage attribution (DXA_SYNC_STAGES=1): make per-stage wall times include their device work."""
        if _SYNC_STAGES and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def _run_command(self, text: str):
        low = text.strip().lower()
        if low.startswith(("set ", "cache ", "uncache ", "refresh ", "clear cache")) or not low:
            return
        if low.startswith("create table"):
            # accumulator DDL: the state table itself is configured (datax.job.process.statetable.*) and loaded at
            # start-up, so the statement is a no-op here — as Spark's CREATE TABLE IF NOT EXISTS on an existing table
            import re
            m = re.match(r"create\s+table\s+(?:if\s+not\s+exists\s+)?([A-Za-z_][A-Za-z0-9_]*)", low)
            if m and any(n.lower() == m.group(1) for n in self.state_tables):
                return
            raise EvalError(f"CREATE TABLE for an unconfigured accumulator: {text.strip()[:80]}")
        raise EvalError(f"unsupported command statement: {text}")

    def process_batch(self, raw: RawBatch, batch_time_us: int, interval_us: int,
                      partition_time: Optional[_dt.datetime] = None) -> Dict[str, float]:
        """Run one micro-batch.  Synchronous mode returns the batch's complete metrics.  Pipelined mode
        (``pipeline_outputs``) returns as soon as the batch's outputs are staged — its metrics (with sink counts and
        ``Latency-Process`` measured to output completion) arrive through ``on_batch_complete`` / ``completed``
        when the next batch (or ``drain()``) completes it.

        Runs under ``torch.inference_mode``: nothing here is differentiated, and without the autograd / version-
        counter dispatch every tensor op costs ~1 us less host time (hundreds of ops per batch on the planning
        thread, which bounds the device-resident flows)."""
        with torch.inference_mode():
            return self._process_batch(raw, batch_time_us, interval_us, partition_time)

    def _process_batch(self, raw: RawBatch, batch_time_us: int, interval_us: int,
                       partition_time: Optional[_dt.datetime] = None) -> Dict[str, float]:
        t0 = time.perf_counter()
        ctx = EvalContext(now_us=int(self.clock() * 1e6), udfs=self.udfs, udafs=self.udafs, device=self.device)
        for refresh in self.udf_refreshers:
            refresh(batch_time_us)
        try:
            _maybe_inject_fault(self.batches)
            tp = time.perf_counter()
            projected = self.project(raw, batch_time_us, ctx)
            self.host_acc["project"] += time.perf_counter() - tp
            # a device-side decode failure (corrupt LZ4 block, bad CRC) must stop the batch before any of its rows
            # reach an accumulator or a sink — the host decoder raises at the same point (before processing).  The
            # status word sits in pinned memory behind the decode, which the parse above already waited for
            check = getattr(raw.status, "raise_if_failed", None)
            if check is not None:
                check(f"batch {batch_time_us}")
            tr = time.perf_counter()
            metrics = self.route(projected, batch_time_us, interval_us, ctx,
                                 partition_time or _dt.datetime.utcnow(), t0)
            t_ret = time.perf_counter()
            self.host_acc["route"] += t_ret - tr
            # from route's return to here: the batch thread waiting for the GIL an output thread took (wall) and
            # the release of route's locals (CPU)
            self.host_acc["route:release"] += t_ret - self._t_route_end
            self.host_acc["route:release_cpu"] += time.thread_time() - self._c_route_end
            self.batches += 1
            return metrics
        except Exception:
            log.exception("batch %s failed", batch_time_us)
            try:
                while self._inflights:
                    self._complete_inflight()   # the previous batches still get their outputs and metrics
            except Exception:  # noqa: BLE001
                self._inflights.clear()
            from ..telemetry.appinsights import track_exception
            track_exception("ProcessDataFrame", _fmt_ts(batch_time_us))
            raise


def _maybe_inject_fault(batch_index: int):
    """Fault injection for recovery tests: ``DXA_FAULT_INJECT=batch=<k>[,once=<marker file>]`` fails the k-th batch of
    this process (with ``once``: only until the marker exists, i.e. the first attempt)."""
    spec = os.environ.get("DXA_FAULT_INJECT")
    if not spec:
        return
    opts = dict(kv.split("=", 1) for kv in spec.split(",") if "=" in kv)
    if int(opts.get("batch", -1)) != batch_index:
        return
    marker = opts.get("once")
    if marker:
        if os.path.exists(marker):
            return
        with open(marker, "w") as f:
            f.write("injected\n")
    raise RuntimeError(f"injected fault at batch {batch_index}")


OUTPUT_CPU = [0.0]             # output threads' CPU time (time.thread_time) in the outputs' host halves, summed


def _timed(fn, *args):
    c0 = time.thread_time()
    out = fn(*args)
    OUTPUT_CPU[0] += time.thread_time() - c0
    return out, time.perf_counter()


def _finish_local(items, partition_time, target):
    """The host halves of a batch's outputs whose sinks never block (``OutputOperator.local``), on one thread."""
    return [_timed(st.finish, partition_time, target) for st in items]


class _Part:
    """One output's (metrics, end time) out of a ``_finish_local`` future."""
    __slots__ = ("fut", "k")

    def __init__(self, fut, k):
        self.fut, self.k = fut, k

    def result(self):
        return self.fut.result()[self.k]


class _InFlight:
    __slots__ = ("batch_time_us", "metrics", "futures", "t0", "t_staged", "stages")

    def __init__(self, batch_time_us, metrics, futures, t0):
        self.batch_time_us = batch_time_us
        self.metrics = metrics
        self.futures = futures
        self.t0 = t0
        self.t_staged = t0
        self.stages = {}


def _fmt_ts(us: int) -> str:
    t = _dt.datetime(1970, 1, 1) + _dt.timedelta(microseconds=int(us))
    return t.strftime("%Y-%m-%d %H:%M:%S.") + f"{t.microsecond // 1000:03d}"


def _h2d(data, dtype, device):
    from ..ops.native import h2d
    return h2d(data, dtype, device)


def _schema_tree(st: StructType):
    """lower-case field name → (field name, subtree or None) for a struct schema."""
    out = {}
    for f in st.fields:
        out[f.name.lower()] = (f.name, _schema_tree(f.dtype) if isinstance(f.dtype, StructType) else None)
    return out


def _ast_nodes(obj):
    """Every AST node (expressions, select items, relations) reachable from a parsed query."""
    from dataclasses import fields, is_dataclass
    stack = [obj]
    seen = set()
    while stack:
        o = stack.pop()
        if id(o) in seen:
            continue
        seen.add(id(o))
        if isinstance(o, (list, tuple)):
            stack.extend(o)
            continue
        if is_dataclass(o):
            yield o
            for f in fields(o):
                stack.append(getattr(o, f.name))
