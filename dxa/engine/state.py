"""Accumulator ("state") tables — ``CREATE TABLE`` / ``WITH UPSERT`` targets that survive across batches.

Reference: DataProcessing/datax-host/src/main/scala/datax/handler/StateTableHandler.scala:17-129 — double-buffered
(A/B) Parquet tables plus a ``metadata.info`` file naming the active copy; a query assigning to the table overwrites
the standby copy and flips; the flip is persisted after the batch's outputs (CommonProcessorFactory.scala:318-320).

Here the active copy is a device-resident columnar table (queried straight from HBM every batch); the standby copy
is written to ``<location>/<A|B>/part-0.parquet`` (pyarrow) and ``metadata.info`` is rewritten atomically after
outputs, so a restarted engine resumes from the last committed accumulator state.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from ..io import fs
from .column import Table
from .types import StructType, parse_ddl_schema


from concurrent.futures import ThreadPoolExecutor

_writer = ThreadPoolExecutor(max_workers=2, thread_name_prefix="dxa-state")


class StateTable:
    def __init__(self, name: str, schema: StructType, location: str, device):
        self.name = name
        self.schema = schema
        self.location = location.rstrip("/") + "/"
        self.device = torch.device(device)
        self.meta_file = self.location + "metadata.info"
        self.params = self._read_meta()
        self.modified = False
        self.active: Table = self._load(self.params["active"])

    def _read_meta(self) -> Dict[str, str]:
        if fs.exists(self.meta_file):
            out = {}
            for line in fs.read_lines(self.meta_file):
                pos = line.find("=")
                if pos <= 0:
                    raise ValueError(f"Invalid content in '{self.meta_file}': '{line}'")
                out[line[:pos]] = line[pos + 1:]
            return out
        return {"active": "A", "standby": "B"}

    def _path(self, suffix: str) -> str:
        return self.location + suffix + "/part-0.parquet"

    def _load(self, suffix: str) -> Table:
        p = self._path(suffix)
        if not fs.exists(p):
            return Table.empty(self.schema, self.device)
        import pyarrow.parquet as pq
        from ..io.arrow import table_from_arrow
        return table_from_arrow(pq.read_table(str(fs.local_path(p))), self.schema, self.device)

    def overwrite(self, t: Table):
        """INSERT OVERWRITE standby + flip (returns the new active table).  The standby Parquet copy is written by
        a background writer from pinned host buffers; ``persist`` (after the batch's outputs) waits for it before
        it flips ``metadata.info``, so the metadata never names a partially written copy."""
        from ..io.arrow import to_host_async
        t = _conform(t, self.schema)
        self._wait_write()
        host, ev = to_host_async(t)
        self._pending = _writer.submit(self._write, self.params["standby"], host, ev)
        self.params = {"active": self.params["standby"], "standby": self.params["active"]}
        self.modified = not self.modified
        self.active = t
        return t

    def _wait_write(self):
        p = getattr(self, "_pending", None)
        if p is not None:
            self._pending = None
            p.result()

    def _write(self, suffix: str, t: Table, event=None):
        import pyarrow.parquet as pq
        from ..io.arrow import table_to_arrow
        if event is not None:
            event.synchronize()
        p = fs.local_path(self._path(suffix))
        p.parent.mkdir(parents=True, exist_ok=True)
        tmp = p.with_suffix(".tmp")
        # uncompressed, no dictionary pages or statistics: the standby copy is rewritten every batch and read back
        # only on restart (2 ms instead of 6.7 ms for a 10 K-row state table; still a Parquet file Spark can read)
        pq.write_table(table_to_arrow(t, self.schema), str(tmp), compression="none", use_dictionary=False,
                       write_statistics=False)
        tmp.replace(p)

    def persist(self):
        self._wait_write()
        if self.modified:
            fs.write_atomic(self.meta_file, "\n".join(f"{k}={v}" for k, v in self.params.items()))
            self.modified = False


def _conform(t: Table, schema: StructType) -> Table:
    from .expr import cast_column
    cols = []
    names = []
    for f in schema.fields:
        c = t.column(f.name)
        if c is None:
            raise ValueError(f"state table result is missing column {f.name}")
        if c.dtype != f.dtype and isinstance(f.dtype, str):
            c = cast_column(c, f.dtype)
        cols.append(c)
        names.append(f.name)
    return Table(names, cols, t.length, t.device)


def create_state_tables(d, device) -> Dict[str, StateTable]:
    from ..config.settings import PROCESS_PREFIX
    out = {}
    for name, sub in d.group_by_sub_namespace(PROCESS_PREFIX + "statetable.").items():
        schema = parse_ddl_schema(sub.get_string("schema"))
        out[name] = StateTable(name, schema, sub.get_string("location"), device)
    return out
