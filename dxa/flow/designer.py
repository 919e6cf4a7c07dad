"""Flow-designer model: the rule condition builder and the designer-flow ⇄ product-config conversion.

The reference does this in the browser (Website/Packages/datax-pipeline/src/modules/flowDefinition/
flowHelpers.js:35-530, enums flowModels.js:114-157): a rule's condition is edited as a tree of groups and
conditions, turned into the SQL text that rules codegen consumes (``$condition``), and aggregate rules derive their
``$aggs`` / ``$pivots`` lists from the tree.  Here the same model runs server-side (REST ``designer/*`` routes), so
the console, scripts and tests share one implementation.

Condition tree::

    {"type": "group", "conjunction": "and", "conditions": [
        {"type": "condition", "conjunction": "and", "field": "temperature", "operator": "greater",
         "value": "90", "aggregate": "none"},
        {"type": "group", "conjunction": "or", "conditions": [...]}]}
"""
from __future__ import annotations

import re
from typing import Any, Dict, List, Optional

# flowModels.js:114-157
RULE_TAG = "tag"
SIMPLE_RULE, AGGREGATE_RULE = "SimpleRule", "AggregateRule"
AGGREGATES = ("MIN", "MAX", "AVG", "SUM", "COUNT", "DCOUNT", "none")
GROUP, CONDITION = "group", "condition"
OPERATORS = {
    "equal": "=", "notEqual": "<>", "greater": ">", "lessThan": "<", "greaterThanOrEqual": ">=",
    "lessThanOrEqual": "<=", "stringEqual": "=", "stringNotEqual": "<>", "contains": "LIKE",
    "notContains": "NOT LIKE", "startsWith": "LIKE", "endsWith": "LIKE",
}
NUMBER_OPERATORS = {"equal", "notEqual", "greater", "lessThan", "greaterThanOrEqual", "lessThanOrEqual"}
SEVERITIES = ("Critical", "Medium", "Low")


class ConditionError(ValueError):
    pass


def default_group() -> Dict[str, Any]:
    return {"type": GROUP, "conjunction": "and", "conditions": [default_condition()]}


def default_condition() -> Dict[str, Any]:
    return {"type": CONDITION, "conjunction": "and", "field": "", "operator": "equal", "value": "",
            "aggregate": "none"}


def is_number_operator(op: str) -> bool:
    return op in NUMBER_OPERATORS


def _is_number(v) -> bool:
    # flowHelpers.js:15-18: !isNaN(parseFloat(v)) && isFinite(v)
    try:
        x = float(str(v).strip())
    except ValueError:
        return False
    return x == x and x not in (float("inf"), float("-inf"))


def format_operator(op: str) -> str:
    return OPERATORS.get(op, "")


def format_value(op: str, value) -> str:
    """flowHelpers.js:142-164: numbers verbatim; text quoted with '' escaping and LIKE wildcards."""
    value = "" if value is None else str(value)
    if is_number_operator(op):
        return value
    value = value.replace("'", "''")
    if op in ("contains", "notContains"):
        return f"'%{value}%'"
    if op == "startsWith":
        return f"'{value}%'"
    if op == "endsWith":
        return f"'%{value}'"
    return f"'{value}'"


def format_aggregate_field(aggregate: str, field: str) -> str:
    if aggregate == "DCOUNT":
        return f"COUNT(DISTINCT {field})"
    if aggregate == "none" or not aggregate:
        return field
    return f"{aggregate}({field})"


def _conj(c: str) -> str:
    return f" {(c or 'and').upper()} "


def _condition_text(c: Dict, index: int, aggregate: bool) -> str:
    text = _conj(c.get("conjunction")) if index > 0 else ""
    field = format_aggregate_field(c.get("aggregate", "none"), c.get("field", "")) if aggregate else c.get("field", "")
    op = c.get("operator", "equal")
    return text + f"{field} {format_operator(op)} {format_value(op, c.get('value'))}"


def _group_text(g: Dict, index: int, aggregate: bool) -> str:
    text = _conj(g.get("conjunction")) if index > 0 else ""
    text += "("
    for i, c in enumerate(g.get("conditions", [])):
        text += _group_text(c, i, aggregate) if c.get("type") == GROUP else _condition_text(c, i, aggregate)
    return text + ")"


def conditions_to_sql(conditions: Optional[Dict], aggregate: bool = False) -> str:
    """flowHelpers.js:93-130 ``formatRuleConditionsToString``: the outer group's parentheses are dropped."""
    if not conditions:
        return ""
    return _group_text(conditions, 0, aggregate)[1:-1]


def validate_conditions(conditions: Dict, rule_type: str = SIMPLE_RULE, ignore_empty_field_and_value: bool = False,
                        ignore_empty_group: bool = False) -> Optional[str]:
    """flowHelpers.js:39-91: the first violated rule's message, or None."""
    def check_condition(c):
        if rule_type == AGGREGATE_RULE and c.get("aggregate", "none") != "none" and \
                not is_number_operator(c.get("operator")):
            raise ConditionError("Text operators cannot be used with Aggregate conditions")
        if not ignore_empty_field_and_value:
            if not c.get("field"):
                raise ConditionError("All conditions need to have column name specified")
            if c.get("value") in (None, ""):
                raise ConditionError("All conditions need to have a value specified")
        v = c.get("value")
        if is_number_operator(c.get("operator")) and v not in (None, "") and not _is_number(v):
            raise ConditionError("Value field must be a number when a numeric operator is used")

    def check_group(g):
        if not ignore_empty_group and not g.get("conditions"):
            raise ConditionError("All groups need to have at least 1 condition")
        for c in g.get("conditions", []):
            (check_group if c.get("type") == GROUP else check_condition)(c)

    try:
        check_group(conditions)
        return None
    except ConditionError as e:
        return str(e)


def _walk(g: Dict):
    for c in g.get("conditions", []):
        if c.get("type") == GROUP:
            yield from _walk(c)
        else:
            yield c


def _unique(xs):
    seen, out = set(), []
    for x in xs:
        if x not in seen:
            seen.add(x)
            out.append(x)
    return out


def config_aggregates(aggregate: bool, conditions: Dict, extra: List[Dict]) -> List[str]:
    """flowHelpers.js:219-247: aggregates used in the conditions, then the user's extra ones, de-duplicated."""
    if not aggregate:
        return []
    xs = [format_aggregate_field(c.get("aggregate"), c.get("field", "")) for c in _walk(conditions)
          if c.get("aggregate", "none") != "none"]
    xs += [format_aggregate_field(a.get("aggregate"), a.get("column", "")) for a in extra or []]
    return _unique(xs)


def config_pivots(aggregate: bool, conditions: Dict, extra: List[str]) -> List[str]:
    """flowHelpers.js:297-325: non-aggregated condition fields, then the user's extra GROUP BY columns."""
    if not aggregate:
        return []
    return _unique([c.get("field", "") for c in _walk(conditions) if c.get("aggregate", "none") == "none"]
                   + list(extra or []))


_AGG_RE = re.compile(r"^(\S+)\((.+)\)$")
_DISTINCT_RE = re.compile(r"^DISTINCT (.+)$")


def flow_aggregates(aggregate: bool, conditions: Dict, aggs: List[str]) -> List[Dict[str, str]]:
    """flowHelpers.js:249-295: the config's aggregate list minus those the conditions imply."""
    if not aggregate or not aggs:
        return []
    implied = {format_aggregate_field(c.get("aggregate"), c.get("field", "")) for c in _walk(conditions)
               if c.get("aggregate", "none") != "none"}
    out = []
    for a in aggs:
        m = _AGG_RE.match(a)
        if not m:
            continue
        cand = {"aggregate": m.group(1), "column": m.group(2)}
        d = _DISTINCT_RE.match(cand["column"])
        if cand["aggregate"] == "COUNT" and d:
            cand = {"aggregate": "DCOUNT", "column": d.group(1)}
        if format_aggregate_field(cand["aggregate"], cand["column"]) not in implied:
            out.append(cand)
    return out


def flow_pivots(aggregate: bool, conditions: Dict, pivots: List[str]) -> List[str]:
    """flowHelpers.js:327-357."""
    if not aggregate or not pivots:
        return []
    implied = {c.get("field", "") for c in _walk(conditions) if c.get("aggregate", "none") == "none"}
    return [p for p in pivots if p not in implied]


def flow_rules_to_config(rules: List[Dict]) -> List[Dict]:
    """flowHelpers.js:359-393 ``convertFlowToConfigRules``."""
    out = []
    for r in rules or []:
        if r.get("type") != RULE_TAG:
            continue
        p = r.get("properties", {})
        agg = p.get("ruleType") == AGGREGATE_RULE
        conds = p.get("conditions") or default_group()
        out.append({"id": r.get("id"), "type": r.get("type"), "properties": {
            "$productId": p.get("productId"), "$ruleType": p.get("ruleType"), "$ruleId": p.get("ruleId"),
            "$ruleDescription": p.get("ruleDescription"), "$condition": conditions_to_sql(conds, agg),
            "$tagName": p.get("tagName"), "$tag": p.get("tag"),
            "$aggs": config_aggregates(agg, conds, p.get("aggs") or []),
            "$pivots": config_pivots(agg, conds, p.get("pivots") or []),
            "$isAlert": p.get("isAlert"), "$severity": p.get("severity"), "$alertSinks": p.get("alertSinks"),
            "$outputTemplate": p.get("outputTemplate"),
            "schemaTableName": p.get("schemaTableName"), "conditions": conds}})
    return out


def config_rules_to_flow(rules: List[Dict]) -> List[Dict]:
    """flowHelpers.js:395-432 ``convertConfigToFlowRules``.  Accepts ``$`` keys or the stored ``_S_`` form."""
    out = []
    for r in rules or []:
        if r.get("type") != RULE_TAG:
            continue
        p = {("$" + k[3:]) if k.startswith("_S_") else k: v for k, v in r.get("properties", {}).items()}
        agg = p.get("$ruleType") == AGGREGATE_RULE
        conds = p.get("conditions") or default_group()
        out.append({"id": r.get("id"), "type": r.get("type"), "properties": {
            "productId": p.get("$productId"), "ruleType": p.get("$ruleType"), "ruleId": p.get("$ruleId"),
            "ruleDescription": p.get("$ruleDescription"), "condition": p.get("$condition"),
            "tagName": p.get("$tagName"), "tag": p.get("$tag"),
            "aggs": flow_aggregates(agg, conds, p.get("$aggs") or []),
            "pivots": flow_pivots(agg, conds, p.get("$pivots") or []),
            "isAlert": p.get("$isAlert"), "severity": p.get("$severity"), "alertSinks": p.get("$alertSinks"),
            "outputTemplate": p.get("$outputTemplate"),
            "schemaTableName": p.get("schemaTableName"), "conditions": conds}})
    return out


def flow_to_config(flow: Dict, query: str) -> Dict:
    """flowHelpers.js:438-475 ``convertFlowToConfig``: the designer's flow → the product config flow/save takes."""
    by_id = lambda xs: sorted(xs or [], key=lambda x: str(x.get("id", "")))  # noqa: E731
    props = flow.get("input", {}).get("properties", {})
    batch_inputs = flow.get("batchInputs") or [default_batch_input()]
    return {
        "name": flow.get("name"), "flowId": flow.get("flowId"), "displayName": (flow.get("displayName") or "").strip(),
        "owner": flow.get("owner"), "databricksToken": flow.get("databricksToken"),
        "input": {**flow.get("input", {}), "referenceData": flow.get("referenceData", []), "batch": batch_inputs},
        "process": {"timestampColumn": props.get("timestampColumn"),
                    "watermark": f"{props.get('watermarkValue')} {props.get('watermarkUnit')}",
                    "functions": by_id(flow.get("functions")), "queries": [query],
                    "jobconfig": flow.get("scale")},
        "outputs": by_id(flow.get("outputs")),
        "outputTemplates": by_id(flow.get("outputTemplates")),
        "rules": flow_rules_to_config(by_id(flow.get("rules"))),
        "batchList": sorted(flow.get("batchList") or [], key=lambda b: str(b.get("type", "")), reverse=True),
    }


def config_to_flow(config: Dict) -> Dict:
    """flowHelpers.js:477-509 ``convertConfigToFlow``."""
    inp = dict(config.get("input", {}))
    props = dict(inp.get("properties", {}))
    props.setdefault("inputSubscriptionId", "")
    props.setdefault("inputResourceGroup", "")
    inp["properties"] = props
    proc = config.get("process", {})
    return {
        "name": config.get("name"), "flowId": config.get("flowId"), "displayName": config.get("displayName"),
        "owner": config.get("owner"), "databricksToken": config.get("databricksToken"), "input": inp,
        "batchInputs": inp.get("batch") or [default_batch_input()],
        "batchList": config.get("batchList") or [],
        "referenceData": inp.get("referenceData") or [],
        "functions": proc.get("functions") or [],
        "query": (proc.get("queries") or [""])[0],
        "scale": proc.get("jobconfig"),
        "outputs": config.get("outputs"),
        "outputTemplates": config.get("outputTemplates") or [],
        "rules": config_rules_to_flow(config.get("rules")),
    }


def default_batch_input() -> Dict[str, Any]:
    return {"type": "blob", "properties": {"connection": "", "path": "", "formatType": "json",
                                           "compressionType": "none"}}
