"""Accumulator ("state") tables — ``CREATE TABLE`` / ``WITH UPSERT`` targets that survive across batches.

Reference: DataProcessing/datax-host/src/main/scala/datax/handler/StateTableHandler.scala:17-129 — double-buffered
(A/B) Parquet tables plus a ``metadata.info`` file naming the active copy; a query assigning to the table overwrites
the standby copy and flips; the flip is persisted after the batch's outputs (CommonProcessorFactory.scala:318-320).

Here the active copy is a device-resident columnar table (queried straight from HBM every batch); the standby copy
is written to ``<location>/<A|B>/part-<rank>.parquet`` (pyarrow) and ``metadata.info`` is rewritten atomically after
outputs, so a restarted engine resumes from the last committed accumulator state.

Multi-GPU (SURVEY §2.G X10 — Spark writes the state table as one Parquet part per partition): every rank keeps and
persists ITS share of the table, as the query produced it — a ``GROUP BY`` result lives on the key's owner rank
(``hashed``), a global aggregate is identical everywhere (``replicated``).  The distribution tag survives the
overwrite, so the next batch's ``UNION ALL <state> … GROUP BY`` treats the state rows as rank-local rows again rather
than as a replicated copy (which ``_set_op`` would keep on rank 0 only).  ``metadata.info`` is flipped once per batch
by rank 0, after every rank's part is durable (the batch-metrics all-reduce in ``Processor._complete_inflight`` is
the barrier), and records ``parts`` (the world size that wrote the copy) and ``dist``.  On restart with the same
world size each rank reads its own part; with a different one, rank r reads parts ``p ≡ r (mod W)`` and the table
is tagged ``partitioned`` (the next GROUP BY re-shuffles it by key hash).
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor
from typing import Any, Callable, Dict, List, Optional

import torch

from .. import parallel as P
from ..io import fs
from .column import StrColumn, Table, concat_tables
from .types import StructType, parse_ddl_schema

_writer = ThreadPoolExecutor(max_workers=2, thread_name_prefix="dxa-state")


class _Write:
    """One batch's overwrite of a state table: the standby-part write (submitted, or deferred until the previous
    batch's flip is released) and the metadata that batch's ``persist`` flips to."""

    def __init__(self, tag, params: Dict[str, str]):
        self.tag = tag
        self.params = params
        self.fut = None
        self.job: Optional[Callable[[], Any]] = None
        self.persisted = False

    def wait(self):
        if self.job is not None:            # never released: nothing may still reference its copy
            self.fut, self.job = _writer.submit(self.job), None
        if self.fut is not None:
            self.fut.result()


class StateTable:
    def __init__(self, name: str, schema: StructType, location: str, device):
        self.name = name
        self.schema = schema
        self.location = location.rstrip("/") + "/"
        self.device = torch.device(device)
        self.meta_file = self.location + "metadata.info"
        self.rank, self.world = P.rank(), P.world()
        self.params = self._read_meta()
        self._writes: List[_Write] = []      # overwrites not yet released, oldest first
        self.active: Table = self._load(self.params["active"])

    # ---- metadata ------------------------------------------------------------------------------------------------
    def _read_meta(self) -> Dict[str, str]:
        if fs.exists(self.meta_file):
            out = {}
            for line in fs.read_lines(self.meta_file):
                if not line.strip():
                    continue
                pos = line.find("=")
                if pos <= 0:
                    raise ValueError(f"Invalid content in '{self.meta_file}': '{line}'")
                out[line[:pos]] = line[pos + 1:]
            if "active" not in out or "standby" not in out:
                raise ValueError(f"'{self.meta_file}' names no active/standby copy")
            return out
        return {"active": "A", "standby": "B"}

    @property
    def dist(self) -> str:
        """Distribution of the active copy across ranks (``replicated`` on a single rank)."""
        return P.dist_of(self.active) if P.active() else P.REPLICATED

    def _path(self, suffix: str, part: int) -> str:
        return f"{self.location}{suffix}/part-{part}.parquet"

    # ---- load ----------------------------------------------------------------------------------------------------
    def _read_part(self, suffix: str, part: int):
        p = self._path(suffix, part)
        if not fs.exists(p):
            return None
        import pyarrow.compute as pc
        import pyarrow.parquet as pq
        from ..io.arrow import table_from_arrow
        at = pq.read_table(str(fs.local_path(p)))
        t = table_from_arrow(at, self.schema, self.device)
        # the string columns' longest value, read here on the host once: the per-batch UNION with this table then
        # bounds its bytes without waiting for a device scan (strings.concat_multi)
        arrow_name = {n.lower(): n for n in at.column_names}
        for name, c in zip(t.names, t.columns):
            src = arrow_name.get(name.lower())
            if type(c) is StrColumn and src is not None and c.length:
                try:
                    m = pc.max(pc.binary_length(at.column(src))).as_py()
                except Exception:  # noqa: BLE001 — e.g. a dictionary-encoded column: leave it unbounded
                    continue
                c.max_len = int(m or 0)
        return t

    def _load(self, suffix: str) -> Table:
        parts_written = int(self.params.get("parts", "1"))
        dist = self.params.get("dist", P.REPLICATED if parts_written == 1 else P.PARTITIONED)
        if not P.active():
            # one rank owns everything: a replicated copy is any one part, a partitioned one is all parts
            mine = [0] if dist == P.REPLICATED else list(range(parts_written))
            tag = P.REPLICATED
        elif dist == P.REPLICATED:
            mine, tag = [0], P.REPLICATED
        else:
            mine = [p for p in range(parts_written) if p % self.world == self.rank]
            # same world: the rows are exactly the ones this rank produced (HASHED stays valid but nothing downstream
            # distinguishes it from PARTITIONED); a different world: any key may now sit on any rank
            tag = P.PARTITIONED
        tables: List[Table] = [t for t in (self._read_part(suffix, p) for p in mine) if t is not None]
        t = concat_tables(tables) if tables else Table.empty(self.schema, self.device)
        if len(tables) > 1:
            t = Table(t.names, t.columns, t.length, t.device)
        t.dist = tag if P.active() else P.REPLICATED
        if P.active() and not tables and dist != P.REPLICATED:
            t.dist = P.PARTITIONED       # an empty share of a partitioned table
        return t

    # ---- update --------------------------------------------------------------------------------------------------
    def overwrite(self, t: Table, tag=None):
        """INSERT OVERWRITE standby + flip (returns the new active table).  The device work (conform, one packed
        D2H) starts here; the standby Parquet part is written by a background writer from the pinned host copy.
        ``persist(tag)`` (after the batch's outputs) waits for that write before it flips ``metadata.info``, so the
        metadata never names a partially written copy.

        The next batch may overwrite before this one is persisted (outputs are pipelined): its write goes to the
        copy the on-disk metadata still names active, so it is deferred until ``release`` of this batch's flip —
        the batch itself (the device-side state) does not wait."""
        from ..io.arrow import to_host_async
        dist = P.dist_of(t)
        t = _conform(t, self.schema)
        t.dist = dist if P.active() else P.REPLICATED
        job = None
        if not (P.active() and dist == P.REPLICATED and self.rank != 0):   # replicated: rank 0's part-0 is the copy
            host, ev = to_host_async(t)
            suffix, rank = self.params["standby"], self.rank
            job = lambda: self._write(suffix, rank, host, ev)             # noqa: E731
        self.params = {"active": self.params["standby"], "standby": self.params["active"],
                       "parts": str(self.world), "dist": t.dist}
        w = _Write(tag, dict(self.params))
        if job is not None:
            if self._writes:
                w.job = job
            else:
                w.fut = _writer.submit(job)
        self._writes.append(w)
        self.active = t
        return t

    @property
    def modified(self) -> bool:
        return any(not w.persisted for w in self._writes)

    def _entry(self, tag) -> Optional[_Write]:
        for w in self._writes:
            if not w.persisted and (tag is None or w.tag == tag):
                return w
        return None

    def _write(self, suffix: str, part: int, t: Table, event=None):
        import pyarrow.parquet as pq
        from ..io.arrow import table_to_arrow
        if event is not None:
            event.synchronize()
        p = fs.local_path(self._path(suffix, part))
        p.parent.mkdir(parents=True, exist_ok=True)
        tmp = p.with_name(p.name + ".tmp")
        # uncompressed, no dictionary pages or statistics: the standby copy is rewritten every batch and read back
        # only on restart (2 ms instead of 6.7 ms for a 10 K-row state table; still a Parquet file Spark can read)
        pq.write_table(table_to_arrow(t, self.schema), str(tmp), compression="none", use_dictionary=False,
                       write_statistics=False)
        tmp.replace(p)

    def flush(self, tag=None):
        """Make this rank's standby part of batch ``tag`` durable (call on every rank before the barrier that
        precedes ``persist``)."""
        w = self._entry(tag)
        if w is not None:
            w.wait()

    def persist(self, tag=None) -> bool:
        """Flip ``metadata.info`` to batch ``tag``'s copy (rank 0 only; every rank's part must already be durable —
        see ``flush``).  At N ranks the processor follows the flips with ``parallel.order_point`` and then
        ``release``: the next batch's standby write (into the copy the previous metadata named active) starts only
        after rank 0's flip.  Returns whether there was a flip."""
        w = self._entry(tag)
        if w is None:
            return False
        w.wait()
        if self.rank == 0:
            fs.write_atomic(self.meta_file, "\n".join(f"{k}={v}" for k, v in w.params.items()))
        w.persisted = True
        return True

    def release(self) -> None:
        """The persisted flips are ordered (after ``order_point`` at N ranks): drop them and start the next
        batch's deferred standby write."""
        while self._writes and self._writes[0].persisted:
            self._writes.pop(0)
        if self._writes and self._writes[0].job is not None:
            w = self._writes[0]
            w.fut, w.job = _writer.submit(w.job), None


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
