"""DataX-SQL macro expansion: no-code rules / alerts / metrics / outputs / accumulators / time windows → plain
transform statements the engine executes.

Behavioural parity with the reference's rules code generator
(Services/DataX.Flow/DataX.Flow.CodegenRules/Engine.cs:18-644, Rule.cs:16-294, Metrics.cs, and the templates in
Resources/defaultQueryTemplate.xml / defaultOutputTemplate.xml):

* ``T = ProcessRules(X)``            → ``T = SELECT *, filterNull(Array(IF(cond, MAP(rule…), NULL), …)) AS Rules FROM X``
* ``T = ProcessAggregateRules(X)``   → per rule ar1 (GROUP BY pivots with aggregates) / ar2 (rule object) /
                                        ar3 (output template) and an ar4 UNION, then ``T = SELECT * FROM ar4``
* ``ProcessAlerts(X)`` / ``ProcessAggregateAlerts(X)`` → alert tables + ``<Tag>Alert`` metric rows + OUTPUTs
  (auto-inserted for ``$isAlert`` rules whose call is missing)
* ``M = CreateMetric(X, expr)``      → metric row statement
* ``OUTPUT a, b TO s1, s2;``          → removed, returned as (table, sink) pairs
* ``CREATE TABLE n (schema);``        → removed, returned as accumulation tables
* ``… FROM DataXProcessedInput TIMEWINDOW('5 minutes')`` → ``FROM DataXProcessedInput_5minutes`` (+ window spec)
* ``--DataXQuery-- <query> WITH UPSERT n`` → ``n = <query>``

The reference pretty-prints the result with its SQL formatter; we emit one statement per ``--DataXQuery--`` block
(whitespace differs, tokens are identical — the golden tests compare token streams).
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple
from xml.etree import ElementTree

DEFAULT_TARGET = "DataXProcessedInput"

DEFAULT_QUERY_TEMPLATES = {
    "SimpleRule": """
--DataXQuery--
$return = SELECT *, $arrayConditions AS Rules FROM DataXProcessedInput;
""",
    "SimpleAlert": """
--DataXQuery--
sa1_$ruleCounter = SELECT *, '$ruleId' AS ruleId, '$ruleDescription' AS ruleDescription, '$severity' AS severity, '$tag' AS Tag FROM DataXProcessedInput
WHERE $condition;

--DataXQuery--
sa2_$ruleCounter = ApplyTemplate(sa1_$ruleCounter, $outputTemplate);

--DataXQuery--
$tagAlert = SELECT DISTINCT DATE_TRUNC('second', current_timestamp()) AS EventTime, '$tagAlert' AS MetricName, 0 as Metric,  '$productId' AS Product, '$ruleDescription' AS Pivot1 FROM sa1_$ruleCounter;

OUTPUT sa2_$ruleCounter TO $alertsinks;
OUTPUT $tagAlert TO Metrics;
""",
    "AggregateRule": """
--DataXQuery--
ar1_$ruleCounter = SELECT $aggs, $pivots, COUNT(*) AS Count
FROM DataXProcessedInput
GROUP BY $pivots;

--DataXQuery--
ar2_$ruleCounter = SELECT *, IF($condition,$ruleObject,NULL) AS RuleObject
FROM ar1_$ruleCounter;

--DataXQuery--
ar3_$ruleCounter = ApplyTemplate(ar2_$ruleCounter, defaultAggOutputTemplate);
""",
    "AggregateAlert": """
--DataXQuery--
aa1_$ruleCounter = SELECT $aggs, $pivots, COUNT(*) AS Count
FROM DataXProcessedInput
GROUP BY $pivots;

--DataXQuery--
aa2_$ruleCounter = SELECT *, $ruleObject AS RuleObject FROM aa1_$ruleCounter WHERE $condition;

--DataXQuery--
aa3_$ruleCounter = ApplyTemplate(aa2_$ruleCounter, $outputTemplate);

--DataXQuery--
$tagAlert = SELECT DISTINCT DATE_TRUNC('second', current_timestamp()) AS EventTime, '$tagAlert' AS MetricName, 0 as Metric, '$productId' AS Product, RuleObject.ruleDescription AS Pivot1 FROM aa2_$ruleCounter;

OUTPUT aa3_$ruleCounter TO $alertsinks;
OUTPUT $tagAlert TO Metrics;
""",
}

DEFAULT_OUTPUT_TEMPLATES = {
    "defaultAggOutputTemplate": """
  MAP(
    $pivotstemplate
  ) AS pivots,
  $aggstemplate,
  Count AS count,
  MAP(
    'ruleId', '$ruleId',
    '$tagname', '$tag',
    'description', '$ruleDescription',
    'severity', '$severity'
  ) AS result""",
}


class CodegenError(Exception):
    pass


def loads_lenient(text: str):
    """JSON with // and /* */ comments and trailing commas (the reference's rule fixtures use both)."""
    out = []
    i, n = 0, len(text)
    in_str = False
    while i < n:
        c = text[i]
        if in_str:
            out.append(c)
            if c == "\\" and i + 1 < n:
                out.append(text[i + 1])
                i += 2
                continue
            if c == '"':
                in_str = False
            i += 1
            continue
        if c == '"':
            in_str = True
            out.append(c)
            i += 1
            continue
        if text.startswith("//", i):
            while i < n and text[i] != "\n":
                i += 1
            continue
        if text.startswith("/*", i):
            j = text.find("*/", i + 2)
            i = n if j < 0 else j + 2
            continue
        out.append(c)
        i += 1
    s = re.sub(r",(\s*[}\]])", r"\1", "".join(out)).lstrip("﻿")
    return json.loads(s) if s.strip() else []


_AGG_RE = re.compile(r"(.*)\((.*?)\)")


@dataclass
class Rule:
    rule_id: str = ""
    product_id: str = ""
    rule_type: str = "SimpleRule"
    rule_description: str = ""
    rule_category: str = ""
    severity: str = ""
    condition: str = ""
    aggs: List[str] = field(default_factory=list)
    pivots: List[str] = field(default_factory=list)
    tagname: str = "Tag"
    tag: str = ""
    fact: str = ""
    id: str = ""
    output_template: str = ""
    sinks: List[str] = field(default_factory=list)
    alert_sinks: Optional[List[str]] = None
    is_alert: bool = False
    target_table: str = DEFAULT_TARGET

    @staticmethod
    def from_json(d: dict) -> "Rule":
        low = {k.lower(): v for k, v in d.items()}

        def g(k, default=None):
            return low.get(k.lower(), default)
        return Rule(g("$ruleId", "") or "", g("$productId", "") or "", g("$ruleType", "SimpleRule") or "SimpleRule",
                    g("$ruleDescription", "") or "", g("$ruleCategory", "") or "", g("$severity", "") or "",
                    g("$condition", "") or "", list(g("$aggs") or []), list(g("$pivots") or []),
                    g("$tagname", "") or "", g("$tag", "") or "", g("$fact", "") or "", g("$id", "") or "",
                    g("$outputTemplate", "") or "", list(g("$sinks") or []), g("$alertsinks"),
                    bool(g("$isAlert", False)), g("schemaTableName", DEFAULT_TARGET) or DEFAULT_TARGET)

    # -- Rule.cs helpers --------------------------------------------------------------------------------------------
    @staticmethod
    def _agg_alias(agg: str) -> str:
        m = _AGG_RE.search(agg)
        op, col = m.group(1), m.group(2)
        if col.endswith("`"):
            return col.rstrip("`") + "_" + op + "`"
        return col.replace(".", "") + "_" + op

    def aggs_to_select(self) -> str:
        if not self.aggs:
            return ""
        return ", ".join(f"{a} AS {self._agg_alias(a)}" for a in self.aggs)

    def condition_to_sql(self) -> str:
        if not self.aggs:
            return self.condition
        out = self.condition
        for a in self.aggs:
            out = out.replace(a, self._agg_alias(a))
        for p in self.pivots:
            if not p.startswith("`") and "." in p:
                out = out.replace(p, p.split(".")[-1])
        return out

    def aggs_to_template(self) -> str:
        if not self.aggs:
            return ""
        groups: Dict[str, List[str]] = {}
        for a in self.aggs:
            m = _AGG_RE.search(a)
            groups.setdefault(m.group(2), []).append(m.group(1))
        parts = []
        for col, ops in groups.items():
            inner = []
            for op in ops:
                if col.endswith("`"):
                    inner.append(f"'{op}', {col.rstrip('`')}_{op}`")
                else:
                    inner.append(f"'{op}', {col.replace('.', '')}_{op}")
            parts.append(f"'{col}', MAP(\n" + ",".join(inner) + ")")
        return "MAP(\n" + ", \n".join(parts) + "\n) AS aggs"

    def pivots_to_template(self) -> str:
        if not self.pivots:
            return ""
        parts = []
        for p in self.pivots:
            if p.strip().endswith("`"):
                parts.append(f"'{p}', {p}")
            else:
                parts.append(f"'{p}', {p.split('.')[-1]}")
        return ",\n".join(parts)

    @staticmethod
    def list_to_string(xs: Optional[List[str]]) -> str:
        return ", ".join(xs) if xs else ""

    def rules_object(self) -> str:
        return (f"MAP('ruleId', '{self.rule_id}', 'ruleDescription', '{self.rule_description}', "
                f"'severity', '{self.severity}', '{self.tagname}', '{self.tag}')")


@dataclass
class RulesCode:
    code: str
    outputs: List[Tuple[str, str]]
    accumulation_tables: Dict[str, str]
    time_windows: Dict[str, str]
    metrics: Dict


def metrics_config(outputs: List[Tuple[str, str]]) -> Dict:
    """Dashboard config for tables output to Metrics (reference Metrics.cs)."""
    sources, widgets = [], []
    for table, sink in outputs:
        if sink.strip().lower() != "metrics":
            continue
        alert = "alert" in table.lower() and "," not in table
        names = [n.strip() for n in table.split(",")]
        sources.append({"name": table, "input": {"type": "MetricDetailsApi" if alert else "MetricApi",
                                                  "pollingInterval": 60000,
                                                  "metricKeys": [{"name": f"_FLOW_:{n}", "displayName": n}
                                                                 for n in names]},
                        "output": {"type": "DirectTable" if alert else "DirectTimeChart",
                                   "data": {"timechart": not alert, "current": False, "table": alert},
                                   "chartTimeWindowInMs": 3600000}})
        widgets.append({"name": table, "data": table + ("_table" if alert else "_timechart"), "displayName": table,
                        "position": "TimeCharts", "type": "DetailsList" if alert else "MultiLineChart"})
    return {"sources": sources, "widgets": widgets,
            "initParameters": {"widgetSets": ["direct"], "jobNames": {"type": "getCPSparkJobNames"}}}


def _templates_from_xml(text: Optional[str], tag: str, key: str) -> Optional[Dict[str, str]]:
    if not text:
        return None
    root = ElementTree.fromstring(text.lstrip("﻿").encode())
    return {el.get(key): (el.text or "") for el in root.iter(tag)}


class Engine:
    def __init__(self, query_templates: Optional[str] = None, output_templates: Optional[str] = None):
        self.qt = _templates_from_xml(query_templates, "query", "type") or dict(DEFAULT_QUERY_TEMPLATES)
        self.ot = _templates_from_xml(output_templates, "outputTemplate", "id") or dict(DEFAULT_OUTPUT_TEMPLATES)

    def generate(self, code: str, rules_json, product_id: str = "") -> RulesCode:
        rules = rules_json if isinstance(rules_json, list) else loads_lenient(rules_json or "[]")
        self.rules = [r if isinstance(r, Rule) else Rule.from_json(r) for r in rules]
        self.code = code.lstrip("﻿")
        self.stmt = 0
        self.rule_counter = 1
        self.product = product_id
        self._auto_alerts()
        self._alerts()
        self._rules()
        self._aggregate_rules()
        self._aggregate_alerts()
        self._create_metrics()
        outputs = self._outputs()
        acc = self._accumulation_tables()
        windows = self._time_windows()
        metrics = metrics_config(outputs)
        self._upsert()
        return RulesCode(_normalise(self.code), outputs, acc, windows, metrics)

    # -- selection --------------------------------------------------------------------------------------------------
    def _select(self, rule_type: str, target: str, alert: Optional[bool]):
        out = []
        for r in self.rules:
            if self.product and r.product_id != self.product:
                continue
            if r.rule_type != rule_type or r.target_table != target:
                continue
            if alert and not r.is_alert:
                continue
            out.append(r)
        return out

    def _auto_alerts(self):
        kinds: Dict[str, List[str]] = {}
        for r in self.rules:
            if (self.product and r.product_id != self.product) or not r.is_alert:
                continue
            kinds.setdefault(r.target_table, [])
            if r.rule_type not in kinds[r.target_table]:
                kinds[r.target_table].append(r.rule_type)
        for table, types in kinds.items():
            for t in types:
                if t == "SimpleRule":
                    if not re.search(r"ProcessAlerts\s*\(\s*" + re.escape(table) + r"\s*\)", self.code, re.I):
                        self.code += f"\nProcessAlerts({table});"
                else:
                    if not re.search(r"ProcessAggregateAlerts\s*\(\s*" + re.escape(table) + r"\s*\)", self.code, re.I):
                        self.code += f"\nProcessAggregateAlerts({table});"

    def _alerts(self):
        for m in list(re.finditer(r"ProcessAlerts\s*\(\s*(.*?)\s*\)", self.code, re.I)):
            self.stmt += 1
            target = m.group(1) or DEFAULT_TARGET
            rules = self._select("SimpleRule", target, True)
            s = self._expand(rules, self.qt["SimpleAlert"], target)
            self.code = self.code.replace(m.group(0), s, 1)

    def _rules(self):
        for m in list(re.finditer(r"(.*?)\s*=\s*ProcessRules\s*\(\s*(.*?)\s*\)", self.code, re.I)):
            self.stmt += 1
            target = m.group(2) or DEFAULT_TARGET
            rules = self._select("SimpleRule", target, None)
            s = self.qt["SimpleRule"].replace("$arrayConditions", self._array_conditions(rules))
            s = s.replace("$return", m.group(1))
            s = s.replace(DEFAULT_TARGET, target)
            self.code = self.code.replace(m.group(0), s, 1)

    def _aggregate_rules(self):
        for m in list(re.finditer(r"(.*?)\s*=\s*ProcessAggregateRules\s*\(\s*(.*?)\s*\)", self.code, re.I)):
            self.stmt += 1
            target = m.group(2) or DEFAULT_TARGET
            rules = self._select("AggregateRule", target, None)
            s = self._expand(rules, self.qt["AggregateRule"], target)
            s += f"\n\n--DataXQuery--\nar4_{self.stmt} = "
            parts = [f"SELECT * FROM ar3_{self.stmt}_{i}" for i in range(1, self.rule_counter)]
            s += " UNION ".join(parts)
            s += f"\n\n--DataXQuery--\n$return = SELECT * FROM ar4_{self.stmt}"
            s = s.replace("$return", m.group(1))
            self.code = self.code.replace(m.group(0), s, 1)

    def _aggregate_alerts(self):
        for m in list(re.finditer(r"ProcessAggregateAlerts\s*\(\s*(.*?)\s*\)", self.code, re.I)):
            self.stmt += 1
            target = m.group(1) or DEFAULT_TARGET
            rules = self._select("AggregateRule", target, True)
            s = self._expand(rules, self.qt["AggregateAlert"], target)
            self.code = self.code.replace(m.group(0), s, 1)

    def _create_metrics(self):
        for m in list(re.finditer(r"(.*?)\s*=\s*CreateMetric\s*\(\s*(.*?)\s*,\s*(.*?)\s*\)", self.code, re.I)):
            out_table, from_table, metric = m.group(1), m.group(2), m.group(3)
            s = (f"\n\n--DataXQuery--\n{out_table} = SELECT DISTINCT DATE_TRUNC('second', current_timestamp()) AS "
                 f"EventTime, '{out_table}' AS MetricName, {metric} AS Metric, '{self.product}' AS Product, '' AS "
                 f"Pivot1 FROM {from_table} GROUP BY EventTime, MetricName, Metric, Product, Pivot1;")
            self.code = self.code.replace(m.group(0), s, 1)

    def _array_conditions(self, rules: List[Rule]) -> str:
        if not rules:
            return "'NULL'"
        body = ",\n".join(f"IF({r.condition}, {r.rules_object()}, NULL)" for r in rules)
        return "filterNull(Array(\n" + body + "\n))"

    def _expand(self, rules: List[Rule], template: str, target: str) -> str:
        if not rules:
            return ""
        self.rule_counter = 1
        result = ""
        for r in rules:
            result += template.strip()
            for m in list(re.finditer(r"ApplyTemplate\s*\(\s*(.*?)\s*,\s*(.*?)\s*\)", result, re.I)):
                o = None
                if m.group(2) == "$outputTemplate":
                    if r.output_template:
                        o = self.ot.get(r.output_template)
                    elif "aggregate" in r.rule_type.lower():
                        o = self.ot.get("defaultAggOutputTemplate")
                else:
                    o = self.ot.get(m.group(2))
                if o is None:
                    result = result.replace(m.group(0), f"SELECT * FROM {m.group(1)}")
                else:
                    tv = o.replace("$aggstemplate", r.aggs_to_template()).replace("$pivotstemplate",
                                                                                 r.pivots_to_template())
                    result = result.replace(m.group(0), f"SELECT {tv} FROM {m.group(1)}")
            if r.alert_sinks is None or (len(r.alert_sinks) == 1 and r.alert_sinks[0] == "Metrics"):
                result = result.replace("OUTPUT aa3_$ruleCounter TO $alertsinks;", "")
                result = result.replace("OUTPUT sa2_$ruleCounter TO $alertsinks;", "")
            else:
                result = result.replace("$alertsinks", r.list_to_string([s for s in r.alert_sinks if s != "Metrics"]))
            # replacement order matters ($tagname before $tag turns "$tagAlert" into "<Tag>Alert")
            for k, v in [("$productId", r.product_id), ("$ruleId", r.rule_id),
                         ("$ruleCounter", f"{self.stmt}_{self.rule_counter}"),
                         ("$ruleDescription", r.rule_description), ("$ruleCategory", r.rule_category),
                         ("$ruleType", r.rule_type), ("$severity", r.severity), ("$aggs", r.aggs_to_select()),
                         ("$condition", r.condition_to_sql()), ("$tagname", r.tagname), ("$tag", r.tag),
                         ("$sinks", r.list_to_string(r.sinks)), ("$ruleObject", r.rules_object()), ("$id", r.id),
                         ("$fact", r.fact), (DEFAULT_TARGET, target)]:
                result = result.replace(k, v)
            if not r.pivots:
                result = result.replace("GROUP BY $pivots", "").replace("$pivots,", "")
            else:
                result = result.replace("$pivots", r.list_to_string(r.pivots))
            self.rule_counter += 1
        return result

    # -- post-processing --------------------------------------------------------------------------------------------
    def _outputs(self) -> List[Tuple[str, str]]:
        out = []
        for m in list(re.finditer(r"OUTPUT\s+(.*?)\s+TO\s+([^;]*);", self.code, re.I)):
            for sink in m.group(2).split(","):
                out.append((m.group(1), sink.strip()))
            self.code = self.code.replace(m.group(0), "", 1)
        return out

    def _accumulation_tables(self) -> Dict[str, str]:
        acc = {}
        for m in list(re.finditer(r"CREATE TABLE\s+(.*?)\s*\((.*?)\)\s*;", self.code, re.I)):
            acc[m.group(1)] = m.group(2)
            self.code = self.code.replace(m.group(0), "", 1)
        self.code = self.code.replace("--DataXStates--", "")
        return acc

    def _time_windows(self) -> Dict[str, str]:
        out = {}
        pat = re.compile(r"\s*--DataXQuery--\s*([^;]*?)FROM\s+([^\s]+)(\s+)TIMEWINDOW\s*\(\s*(.*?)\s*\)\s*([^;]*?)",
                         re.I)
        for m in list(pat.finditer(self.code)):
            spec = m.group(4).strip().replace("'", "")
            new_table = m.group(2).strip() + "_" + spec.replace(" ", "")
            if m.group(2).strip().lower() != DEFAULT_TARGET.lower():
                raise CodegenError("'DataXProcessedInput' is the only table for which the TIMEWINDOW can be specified")
            q = re.sub(r"\bDataXProcessedInput\b", new_table, m.group(0), flags=re.I)
            q = q.replace(m.group(4).strip(), "")
            q = re.sub(r"(TIMEWINDOW\s*\(\s*\)\s*)", "", q, flags=re.I)
            out.setdefault(new_table, spec)
            self.code = self.code.replace(m.group(0), q, 1)
        return out

    def _upsert(self):
        pat = re.compile(r"\s*--DataXQuery--\s*([^;]*)WITH\s+UPSERT\s+([^;]*)", re.I)
        for m in list(pat.finditer(self.code)):
            nq = "\n\n--DataXQuery--\n" + m.group(2).strip() + " = " + m.group(1).strip() + "\n"
            self.code = self.code.replace(m.group(0), nq, 1)


def _normalise(code: str) -> str:
    """The reference's final pass minus pretty-printing: separator lines, no ';', no empty statements."""
    code = code.replace("\r\n", "\n").replace(";", "")
    code = code.replace("--DataXQuery--", "\n--DataXQuery--\n")
    code = code.strip().strip("\n\r\t")
    code = re.sub(r"--DataXQuery--\s*(?=--DataXQuery--)", "", code)
    code = re.sub(r"--DataXQuery--\s*$", "", code).strip()
    lines = [l.rstrip() for l in code.split("\n")]
    out = []
    for l in lines:
        if not l.strip() and (not out or not out[-1].strip()):
            continue
        out.append(l)
    return "\n".join(out).strip() + "\n"


def generate_code(code: str, rules_json="[]", product_id: str = "", query_templates: Optional[str] = None,
                  output_templates: Optional[str] = None) -> RulesCode:
    return Engine(query_templates, output_templates).generate(code, rules_json, product_id)
