"""Deployment assets: the ARM template's expressions reference only declared parameters / variables, its
dependsOn entries name resources the template creates, and the k8s manifests parse."""
import json
import os
import re

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _strings(o):
    if isinstance(o, str):
        yield o
    elif isinstance(o, dict):
        for k, v in o.items():
            yield from _strings(k)
            yield from _strings(v)
    elif isinstance(o, list):
        for v in o:
            yield from _strings(v)


def test_arm_template_references_resolve():
    t = json.load(open(os.path.join(ROOT, "deploy", "arm", "azuredeploy.json")))
    assert t["$schema"].endswith("deploymentTemplate.json#")
    params, variables = set(t["parameters"]), set(t["variables"])
    types = {r["type"].lower() for r in t["resources"]}
    for s in _strings(t):
        if not s.startswith("["):
            continue
        assert s.endswith("]") and s.count("(") == s.count(")") and s.count("'") % 2 == 0, s
        for p in re.findall(r"parameters\('([^']+)'\)", s):
            assert p in params, p
        for v in re.findall(r"variables\('([^']+)'\)", s):
            assert v in variables, v
    for r in t["resources"]:
        for dep in r.get("dependsOn", []):
            m = re.match(r"\[resourceId\('([^']+)'", dep)
            assert m and m.group(1).lower() in types, dep
    p = json.load(open(os.path.join(ROOT, "deploy", "arm", "azuredeploy.parameters.json")))
    assert set(p["parameters"]) <= params
    required = {k for k, v in t["parameters"].items() if "defaultValue" not in v}
    assert required <= set(p["parameters"]), required


def test_k8s_manifests_parse():
    d = os.path.join(ROOT, "deploy", "k8s")
    for f in os.listdir(d):
        docs = [x for x in yaml.safe_load_all(open(os.path.join(d, f))) if x]
        assert docs and all("kind" in x for x in docs), f
