"""keyvault:// resolution through Azure Key Vault REST against an in-process fake (MSI and client-credential
tokens), after the local sources miss — the reference's KeyVaultClient + MSI authenticator behaviour."""
import json
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from dxa.config import keyvault, secrets


@pytest.fixture()
def fake_kv():
    calls = []

    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def _send(self, code, obj):
            b = json.dumps(obj).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(b)))
            self.end_headers()
            self.wfile.write(b)

        def do_GET(self):
            u = urllib.parse.urlsplit(self.path)
            calls.append(("GET", u.path, dict(self.headers)))
            if u.path == "/msi/token":
                q = urllib.parse.parse_qs(u.query)
                assert self.headers.get("Metadata") == "true" and q["resource"] == ["https://vault.azure.net"]
                return self._send(200, {"access_token": "msi-tok", "expires_in": "3600"})
            if u.path.startswith("/kv/myvault/secrets/"):
                if self.headers.get("Authorization") not in ("Bearer msi-tok", "Bearer sp-tok"):
                    return self._send(401, {"error": "unauthorized"})
                name = urllib.parse.unquote(u.path.rsplit("/", 1)[1])
                if name == "missing":
                    return self._send(404, {"error": {"code": "SecretNotFound"}})
                return self._send(200, {"value": f"secret-of-{name}", "id": name})
            self._send(404, {})

        def do_POST(self):
            u = urllib.parse.urlsplit(self.path)
            n = int(self.headers.get("Content-Length") or 0)
            form = urllib.parse.parse_qs(self.rfile.read(n).decode())
            calls.append(("POST", u.path, form))
            if u.path == "/aad/tenant1/oauth2/token" and form["client_secret"] == ["s3"]:
                return self._send(200, {"access_token": "sp-tok", "expires_on": "9999999999"})
            self._send(401, {})

    srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    yield f"http://127.0.0.1:{srv.server_address[1]}", calls
    srv.shutdown()
    srv.server_close()


def _clear(monkeypatch, tmp_path):
    monkeypatch.setenv("DXA_SECRETS_DIR", str(tmp_path / "nosecrets"))
    for k in ("DXA_SECRETS_FILE", "DXA_KEYVAULT_TENANT", "DXA_KEYVAULT_CLIENT_ID", "DXA_KEYVAULT_CLIENT_SECRET"):
        monkeypatch.delenv(k, raising=False)
    secrets._cache.clear()


def test_msi_token_and_secret_read(fake_kv, monkeypatch, tmp_path):
    base, calls = fake_kv
    _clear(monkeypatch, tmp_path)
    monkeypatch.setenv("DXA_KEYVAULT_URL", base + "/kv/{vault}")
    monkeypatch.setenv("DXA_KEYVAULT_MSI_ENDPOINT", base + "/msi/token")
    assert secrets.resolve("keyvault://myvault/eh-conn") == "secret-of-eh-conn"
    assert secrets.resolve("keyvault://myvault/other") == "secret-of-other"
    assert [c[1] for c in calls].count("/msi/token") == 1            # token cached
    with pytest.raises(secrets.SecretError):
        secrets.resolve("keyvault://myvault/missing")
    # local sources still win over Key Vault
    monkeypatch.setenv("DXA_SECRET_MYVAULT_LOCAL", "from-env")
    assert secrets.resolve("keyvault://myvault/local") == "from-env"


def test_client_credentials_token(fake_kv, monkeypatch, tmp_path):
    base, calls = fake_kv
    _clear(monkeypatch, tmp_path)
    monkeypatch.setenv("DXA_KEYVAULT_URL", base + "/kv/{vault}")
    monkeypatch.setenv("DXA_KEYVAULT_TENANT", "tenant1")
    monkeypatch.setenv("DXA_KEYVAULT_CLIENT_ID", "app1")
    monkeypatch.setenv("DXA_KEYVAULT_CLIENT_SECRET", "s3")
    monkeypatch.setenv("DXA_KEYVAULT_AUTHORITY", base + "/aad")
    assert secrets.resolve("keyvault://myvault/x") == "secret-of-x"
    post = [c for c in calls if c[0] == "POST"][0]
    assert post[2]["grant_type"] == ["client_credentials"] and post[2]["client_id"] == ["app1"]


def test_no_keyvault_configured_raises(monkeypatch, tmp_path):
    _clear(monkeypatch, tmp_path)
    monkeypatch.delenv("DXA_KEYVAULT_URL", raising=False)
    assert keyvault.default_client() is None
    with pytest.raises(secrets.SecretError):
        secrets.resolve("keyvault://v/none")
