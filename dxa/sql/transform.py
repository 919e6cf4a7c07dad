"""Transform-file splitter: ``--DataXQuery--`` separated statements → named views / commands.

Behavioural parity with the reference's ``TransformSQLParser``
(DataProcessing/datax-host/src/main/scala/datax/sql/TransformSqlParser.scala:15-105):

* a line matching ``^--DataXQuery--`` closes the current statement (ProductConstant.scala:18);
* ``name = SELECT …`` on the first line of a statement names it (a *Query*); otherwise it is a *Command*;
* lines starting with ``--`` are comments and blank lines are dropped; remaining lines are trimmed and joined by
  a single space;
* a duplicated view name is an error;
* ``view_reference_count[name]`` counts how many later statements mention ``\\bname\\b`` — the executor keeps
  views referenced more than once materialised (TransformHandler.scala:21-23, CommonProcessorFactory.scala:282-286);
* ``replace_table_names`` rewrites table names on word boundaries.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional

QUERY_SEPARATOR = re.compile(r"^--DataXQuery--")
COMMAND_QUERY = "Query"
COMMAND_COMMAND = "Command"

_NAMED = re.compile(r"^\s*([a-zA-Z0-9_]+)\s*=(.*)$")
_COMMENT = re.compile(r"^\s*--")


class TransformError(Exception):
    pass


@dataclass
class SqlCommand:
    text: str
    name: Optional[str]
    command_type: str


@dataclass
class ParsedResult:
    commands: List[SqlCommand] = field(default_factory=list)
    view_reference_count: Dict[str, int] = field(default_factory=dict)


def parse_transform(lines: Iterable[str] | str) -> ParsedResult:
    if isinstance(lines, str):
        lines = lines.replace("\r\n", "\n").split("\n")
    result = ParsedResult()
    buf: List[str] = []
    name: Optional[str] = None

    def flush(nm):
        sql = " ".join(l for l in buf if l)
        result.commands.append(SqlCommand(sql, nm, COMMAND_COMMAND if nm is None else COMMAND_QUERY))
        if nm:
            if nm in result.view_reference_count:
                raise TransformError(f"dataset name '{nm}' has been created, please check the query to make sure "
                                     f"it is not created again")
            result.view_reference_count[nm] = 0
            for k in list(result.view_reference_count):
                if re.search(r"\b" + re.escape(k) + r"\b", sql):
                    result.view_reference_count[k] += 1

    for raw in lines:
        line = raw.rstrip("\r")
        if not line.strip():
            continue
        if QUERY_SEPARATOR.match(line):
            if buf:
                flush(name)
            name = None
            buf = []
            continue
        if _COMMENT.match(line):
            continue
        if not buf:
            m = _NAMED.match(line)
            if m:
                name = m.group(1)
                buf.append(m.group(2).strip())
                continue
        buf.append(line.strip())
    if buf and name is not None:
        flush(name)
    return result


def replace_table_names(statement: str, mapping: Dict[str, str]) -> str:
    for k, v in mapping.items():
        statement = re.sub(r"\b" + re.escape(k) + r"\b", v.replace("\\", "\\\\"), statement)
    return statement
