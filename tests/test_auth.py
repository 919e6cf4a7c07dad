"""Control-plane auth (GatewayController.cs / RolesCheck.cs): JWT bearer tokens verified here — RS256 against a
JWKS (AAD's published-keys format) and HS256 — with exp / nbf / aud / iss and the DataXReader / DataXWriter roles;
loopback-only onebox mode; a trusted gateway's roles header."""
import json
import subprocess
import time

import pytest
from fastapi.testclient import TestClient

from dxa.service import auth as A


@pytest.fixture(scope="module")
def rsa_key(tmp_path_factory):
    d = tmp_path_factory.mktemp("k")
    key = d / "k.pem"
    r = subprocess.run(["openssl", "genrsa", "-out", str(key), "2048"], capture_output=True)
    if r.returncode != 0:
        pytest.skip("openssl unavailable")
    txt = subprocess.run(["openssl", "rsa", "-in", str(key), "-text", "-noout"], capture_output=True,
                         text=True).stdout

    def field(name):
        lines = txt.split(name + ":")[1].splitlines()[1:]
        hexs = []
        for l in lines:
            if not l.startswith("    "):
                break
            hexs.append(l.strip().replace(":", ""))
        return int("".join(hexs), 16)
    n, d_ = field("modulus"), field("privateExponent")
    jwks = {"keys": [{"kty": "RSA", "use": "sig", "kid": "k1", "n": A.b64url_encode(n.to_bytes(256, "big")),
                      "e": A.b64url_encode((65537).to_bytes(3, "big"))}]}
    path = d / "jwks.json"
    path.write_text(json.dumps(jwks))
    return n, d_, str(path)


def _claims(roles, **kw):
    now = int(time.time())
    c = {"aud": "api://datax", "iss": "https://sts.windows.net/tid/", "exp": now + 600, "nbf": now - 60,
         "roles": roles, "oid": "o1", "tid": "t1"}
    c.update(kw)
    return c


def test_rsa_verify_roundtrip(rsa_key):
    n, d, _ = rsa_key
    sig = A.rsa_sign_sha256(n, d, b"hello")
    assert A.rsa_verify_sha256(n, 65537, b"hello", sig)
    assert not A.rsa_verify_sha256(n, 65537, b"hellO", sig)


def test_jwt_rs256_roles_and_claims(rsa_key, tmp_path, monkeypatch):
    n, d, jwks = rsa_key
    from dxa.service.app import create_app
    monkeypatch.setenv("DXA_AUTH", "jwt")
    monkeypatch.setenv("DXA_AUTH_JWKS", jwks)
    monkeypatch.setenv("DXA_AUTH_AUDIENCE", "api://datax")
    monkeypatch.setenv("DXA_AUTH_ISSUER", "https://sts.windows.net/tid/")
    monkeypatch.setenv("DXA_SUPERVISE", "0")
    client = TestClient(create_app(str(tmp_path / "svc")))

    def tok(claims, **kw):
        return {"Authorization": "Bearer " + A.make_token(claims, "RS256", rsa=(n, d), kid="k1", **kw)}
    flow = {"name": "f1", "displayName": "f1", "gui": {"name": "f1", "displayName": "f1"}}
    assert client.post("/api/flow/getall", json={}).status_code == 401                   # no token
    assert client.post("/api/flow/getall", json={}, headers=tok(_claims(["DataXReader"]))).status_code == 200
    r = client.post("/api/flow/save", json=flow, headers=tok(_claims(["DataXReader"])))
    assert r.status_code == 403 and "DataXWriter" in r.json()["detail"]
    assert client.post("/api/flow/save", json=flow, headers=tok(_claims(["DataXWriter"]))).status_code == 200
    assert client.post("/api/kernel/executequery", json={}, headers=tok(_claims(["DataXReader"]))).status_code == 403
    # expired, wrong audience, wrong issuer, tampered payload
    assert client.post("/api/flow/getall", json={},
                       headers=tok(_claims(["DataXReader"], exp=int(time.time()) - 3600))).status_code == 401
    assert client.post("/api/flow/getall", json={}, headers=tok(_claims(["DataXReader"], aud="x"))).status_code == 401
    assert client.post("/api/flow/getall", json={}, headers=tok(_claims(["DataXReader"], iss="x"))).status_code == 401
    h, p, s = tok(_claims(["DataXReader"]))["Authorization"][7:].split(".")
    forged = A.b64url_encode(json.dumps(_claims(["DataXWriter"])).encode())
    assert client.post("/api/flow/save", json=flow,
                       headers={"Authorization": f"Bearer {h}.{forged}.{s}"}).status_code == 401
    # the roles header is NOT trusted in jwt mode
    assert client.post("/api/flow/save", json=flow, headers={"X-DXA-Roles": "Writer"}).status_code == 401


def test_hs256_whitelist_and_local_mode():
    secret = b"s3cret"
    a = A.Authenticator({"DXA_AUTH_HS256_SECRET": "s3cret", "DXA_AUTH_CLIENT_WHITELIST": "o9.t9"})
    assert a.mode == "jwt"
    good = "Bearer " + A.make_token(_claims(["DataXWriter"]), secret=secret)
    assert a.check(True, good, None, "10.0.0.1")["roles"] == ["DataXWriter"]
    wl = "Bearer " + A.make_token(_claims([], oid="o9", tid="t9"), secret=secret)
    assert a.check(True, wl, None, "10.0.0.1")["oid"] == "o9"            # whitelisted client, no roles
    with pytest.raises(A.AuthError):
        a.check(False, "Bearer " + A.make_token(_claims(["DataXReader"]), secret=b"other"), None, "10.0.0.1")
    local = A.Authenticator({})
    assert local.mode == "local"
    assert local.check(True, None, None, "127.0.0.1") == {}
    with pytest.raises(A.AuthError) as e:
        local.check(False, None, None, "10.1.2.3")
    assert e.value.status == 401


def test_jwks_requires_audience_and_exact_roles(rsa_key, tmp_path):
    """A tenant's JWKS also signs other applications' tokens: JWKS mode refuses to run without an audience, and only
    the configured role names (DataXReader / DataXWriter) grant access — a generic "Writer" role does not."""
    n, d, jwks = rsa_key
    with pytest.raises(ValueError):
        A.Authenticator({"DXA_AUTH_JWKS": jwks})
    assert A.Authenticator({"DXA_AUTH_JWKS": jwks, "DXA_AUTH_ANY_AUDIENCE": "1"}).mode == "jwt"
    a = A.Authenticator({"DXA_AUTH_HS256_SECRET": "k"})
    with pytest.raises(A.AuthError) as e:
        a.check(True, "Bearer " + A.make_token(_claims(["Writer"]), secret=b"k"), None, "10.0.0.1")
    assert e.value.status == 403


def test_unknown_kid_does_not_refetch_per_request(rsa_key):
    n, d, jwks = rsa_key
    ks = A.KeySet(jwks)
    calls = []
    real = ks._fetch
    ks._fetch = lambda: calls.append(1) or real()
    ks.get("k1")
    for _ in range(5):
        with pytest.raises(A.AuthError):
            ks.get("forged-kid")
    assert len(calls) == 1


def test_metrics_upload_and_batches_routes_need_roles(tmp_path, monkeypatch):
    """Every route of the app is authenticated: the metrics reads (Reader), metric ingestion and the Livy-style
    ``/batches`` job submission (Writer) answer 401 without a token; ``/batches`` also takes the Basic credentials
    of ``DXA_BATCHES_BASIC`` (what a fleet's LivyClient sends)."""
    import base64
    from dxa.service.app import create_app
    monkeypatch.setenv("DXA_AUTH", "jwt")
    monkeypatch.setenv("DXA_AUTH_HS256_SECRET", "k3y")
    monkeypatch.setenv("DXA_SUPERVISE", "0")
    monkeypatch.setenv("DXA_BATCHES_BASIC", "fleet:pw")
    client = TestClient(create_app(str(tmp_path / "svc")))

    def tok(roles):
        return {"Authorization": "Bearer " + A.make_token(_claims(roles, aud=None, iss=None), "HS256",
                                                           secret=b"k3y")}
    reader, writer = tok(["DataXReader"]), tok(["DataXWriter"])
    item = [{"app": "DATAX-x", "met": "m1", "val": 3}]
    # no token: 401 everywhere
    assert client.get("/api/metrics/get", params={"m": "DATAX-x:m1"}).status_code == 401
    assert client.get("/api/metrics/DATAX-x:m1/freshness").status_code == 401
    assert client.post("/api/data/upload", json=item).status_code == 401
    assert client.post("/api/metrics/ingest", content='{"app":"p","met":"m","val":2}',
                       headers={"Content-Type": "text/plain"}).status_code == 401
    assert client.post("/batches", json={"file": "x", "args": []}).status_code == 401
    assert client.get("/batches").status_code == 401
    assert client.get("/batches/1").status_code == 401
    assert client.delete("/batches/1").status_code == 401
    # readers read, writers write
    assert client.post("/api/data/upload", json=item, headers=reader).status_code == 403
    assert client.post("/api/data/upload", json=item, headers=writer).json() == "done"
    assert client.get("/api/metrics/get", params={"m": "DATAX-x:m1"}, headers=reader).json()[0]["val"] == 3
    assert client.get("/api/metrics/DATAX-x:m1/freshness", headers=reader).status_code == 200
    assert client.post("/batches", json={"file": "x"}, headers=reader).status_code == 403
    assert client.get("/batches", headers=reader).json()["total"] == 0
    # Livy Basic credentials
    basic = {"Authorization": "Basic " + base64.b64encode(b"fleet:pw").decode()}
    bad = {"Authorization": "Basic " + base64.b64encode(b"fleet:nope").decode()}
    assert client.get("/batches", headers=basic).status_code == 200
    assert client.get("/batches", headers=bad).status_code == 401
