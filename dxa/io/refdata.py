"""Reference data loading (CSV/TSV → device table).  Reference: DataProcessing/datax-host/src/main/scala/datax/
handler/ReferenceDataHandler.scala:16-61 and datax-utility/.../CSVUtil.scala:15-41 — Spark reads with the given
delimiter/header and no schema inference, so every column is a string; stream–static joins cast as needed.

Reference tables stay resident in HBM for the life of the job (sized for 288 GB); joins against them reuse one
cached hash table (``Catalog.cached_build``)."""
from __future__ import annotations

import csv
import io

import torch

from ..engine.column import Table, strings_from_pylist
from . import fs


def load_csv(path: str, delimiter: str = ",", header: bool = True, device="cpu") -> Table:
    text = fs.read_text(path)
    rows = list(csv.reader(io.StringIO(text), delimiter=delimiter))
    rows = [r for r in rows if r]
    if not rows:
        return Table([], [], 0, device)
    if header:
        names, rows = [c.strip() for c in rows[0]], rows[1:]
    else:
        names = [f"_c{i}" for i in range(len(rows[0]))]
    cols = []
    for j, _ in enumerate(names):
        cols.append(strings_from_pylist([r[j] if j < len(r) else None for r in rows], device))
    return Table(names, cols, len(rows), device)
