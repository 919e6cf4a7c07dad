"""Flow-designer model (dxa.flow.designer) against the semantics of the reference's browser helpers
(Website/Packages/datax-pipeline/src/modules/flowDefinition/flowHelpers.js).  The reference has no tests for these
helpers, so the expected strings below are worked out from that file (parity unpinned by a reference fixture)."""
import pytest

from dxa.flow import designer as D
from dxa.sql.codegen import generate_code


def C(field, op, value, conj="and", agg="none"):
    return {"type": "condition", "conjunction": conj, "field": field, "operator": op, "value": value,
            "aggregate": agg}


def G(*conds, conj="and"):
    return {"type": "group", "conjunction": conj, "conditions": list(conds)}


def test_simple_conditions_to_sql():
    g = G(C("temperature", "greater", "90"), C("deviceType", "stringEqual", "Heat'er", conj="or"))
    assert D.conditions_to_sql(g) == "temperature > 90 OR deviceType = 'Heat''er'"


def test_like_operators_and_nested_groups():
    g = G(C("name", "contains", "abc"),
          G(C("name", "startsWith", "x"), C("name", "endsWith", "y", conj="or"), conj="and"),
          C("name", "notContains", "z", conj="or"))
    assert D.conditions_to_sql(g) == ("name LIKE '%abc%' AND (name LIKE 'x%' OR name LIKE '%y') "
                                      "OR name NOT LIKE '%z%'")


def test_aggregate_conditions_and_derived_lists():
    g = G(C("temperature", "greater", "50", agg="AVG"), C("deviceId", "equal", "3"),
          C("homeId", "greater", "1", agg="DCOUNT"))
    assert D.conditions_to_sql(g, aggregate=True) == \
        "AVG(temperature) > 50 AND deviceId = 3 AND COUNT(DISTINCT homeId) > 1"
    # a simple rule ignores the aggregate column
    assert D.conditions_to_sql(g, aggregate=False) == "temperature > 50 AND deviceId = 3 AND homeId > 1"
    assert D.config_aggregates(True, g, [{"aggregate": "MAX", "column": "t"}, {"aggregate": "AVG",
                                                                                "column": "temperature"}]) == \
        ["AVG(temperature)", "COUNT(DISTINCT homeId)", "MAX(t)"]
    assert D.config_pivots(True, g, ["deviceType", "deviceId"]) == ["deviceId", "deviceType"]
    assert D.config_aggregates(False, g, []) == [] and D.config_pivots(False, g, ["x"]) == []
    # config → designer: only the extra aggregates / pivots come back
    assert D.flow_aggregates(True, g, ["AVG(temperature)", "COUNT(DISTINCT homeId)", "MAX(t)",
                                       "COUNT(DISTINCT x)"]) == \
        [{"aggregate": "MAX", "column": "t"}, {"aggregate": "DCOUNT", "column": "x"}]
    assert D.flow_pivots(True, g, ["deviceId", "deviceType"]) == ["deviceType"]


@pytest.mark.parametrize("g,rule_type,msg", [
    (G(C("t", "contains", "1", agg="AVG")), D.AGGREGATE_RULE, "Text operators cannot be used with Aggregate conditions"),
    (G(C("", "equal", "1")), D.SIMPLE_RULE, "All conditions need to have column name specified"),
    (G(C("t", "equal", "")), D.SIMPLE_RULE, "All conditions need to have a value specified"),
    (G(C("t", "greater", "abc")), D.SIMPLE_RULE, "Value field must be a number when a numeric operator is used"),
    (G(C("t", "equal", "1"), G()), D.SIMPLE_RULE, "All groups need to have at least 1 condition"),
    (G(C("t", "stringEqual", "abc")), D.SIMPLE_RULE, None),
])
def test_validate_conditions(g, rule_type, msg):
    assert D.validate_conditions(g, rule_type) == msg


def _designer_flow():
    cond = G(C("telemetry.temperature", "greater", "44.5"))
    return {"name": "iot", "displayName": " IoT flow ", "owner": "me",
            "input": {"type": "local", "mode": "streaming",
                      "properties": {"timestampColumn": "eventTimeStamp", "watermarkValue": "0",
                                     "watermarkUnit": "second"}},
            "referenceData": [], "functions": [{"id": "b"}, {"id": "a"}], "scale": {"jobNumGpus": "1"},
            "outputs": [{"id": "Metrics", "type": "metric", "properties": {}}],
            "rules": [{"id": "r1", "type": "tag", "properties": {
                "productId": "iot", "ruleType": "SimpleRule", "ruleId": "r1", "ruleDescription": "hot",
                "conditions": cond, "tagName": "Tag", "tag": "Hot", "aggs": [], "pivots": [], "isAlert": True,
                "severity": "Critical", "alertSinks": ["Metrics"], "outputTemplate": "",
                "schemaTableName": "DataXProcessedInput"}}]}


def test_flow_config_round_trip_and_codegen():
    flow = _designer_flow()
    cfg = D.flow_to_config(flow, "--DataXQuery--\nT = ProcessRules(DataXProcessedInput);\nOUTPUT T TO Metrics;")
    assert cfg["displayName"] == "IoT flow"
    assert [f["id"] for f in cfg["process"]["functions"]] == ["a", "b"]
    assert cfg["process"]["watermark"] == "0 second"
    r = cfg["rules"][0]["properties"]
    assert r["$condition"] == "telemetry.temperature > 44.5" and r["$tag"] == "Hot"
    back = D.config_to_flow(cfg)
    assert back["rules"][0]["properties"]["conditions"] == flow["rules"][0]["properties"]["conditions"]
    assert back["query"].startswith("--DataXQuery--")
    assert back["input"]["properties"]["inputSubscriptionId"] == ""
    # the generated condition feeds the rules codegen unchanged
    rc = generate_code(cfg["process"]["queries"][0], [x["properties"] for x in cfg["rules"]], "iot")
    assert "telemetry.temperature > 44.5" in rc.code


def test_designer_routes(tmp_path, monkeypatch):
    from fastapi.testclient import TestClient
    from dxa.service.app import create_app
    monkeypatch.setenv("DXA_SECRETS_DIR", str(tmp_path / "secrets"))
    monkeypatch.setenv("DXA_SUPERVISE", "0")
    c = TestClient(create_app(str(tmp_path / "root")))
    r = c.post("/api/designer/conditions/sql", json={
        "ruleType": "AggregateRule", "pivots": ["deviceType"],
        "conditions": G(C("temperature", "greater", "50", agg="MAX"), C("deviceId", "equal", "1"))}).json()
    assert not r["error"]
    assert r["result"]["condition"] == "MAX(temperature) > 50 AND deviceId = 1"
    assert r["result"]["aggs"] == ["MAX(temperature)"] and r["result"]["pivots"] == ["deviceId", "deviceType"]
    assert r["result"]["error"] is None
    bad = c.post("/api/designer/conditions/sql", json={"conditions": G(C("t", "greater", "x"))}).json()
    assert bad["result"]["error"] == "Value field must be a number when a numeric operator is used"
    cfg = c.post("/api/designer/flow/toconfig", json={"flow": _designer_flow(), "query": "q"}).json()["result"]
    assert cfg["rules"][0]["properties"]["$condition"] == "telemetry.temperature > 44.5"
    fl = c.post("/api/designer/flow/fromconfig", json={"config": cfg}).json()["result"]
    assert fl["rules"][0]["properties"]["ruleId"] == "r1"
