"""Azure Key Vault secret reads for ``keyvault://<vault>/<secret>`` references (the reference's KeyVaultClient +
MSI authenticator: DataProcessing/datax-host/src/main/scala/datax/securedsetting/KeyVaultClient.scala:31-110,
datax-keyvault/src/main/scala/datax/keyvault/KeyVaultMsiAuthenticatorClient.scala:16-48).

``secrets.resolve`` consults Key Vault after the local sources when ``DXA_KEYVAULT_URL`` is set (a template such
as ``https://{vault}.vault.azure.net``).  The bearer token comes from, in order:

* a client-credentials grant when ``DXA_KEYVAULT_TENANT`` / ``_CLIENT_ID`` / ``_CLIENT_SECRET`` are set
  (``DXA_KEYVAULT_AUTHORITY`` overrides ``https://login.microsoftonline.com``);
* a managed-identity endpoint: ``DXA_KEYVAULT_MSI_ENDPOINT`` (default: the HDInsight-style
  ``http://localhost:40381/oauth2/token`` the reference used, else Azure IMDS
  ``http://169.254.169.254/metadata/identity/oauth2/token``).

Tokens are cached until 5 minutes before they expire.
"""
from __future__ import annotations

import json
import os
import threading
import time
import urllib.error
import urllib.parse
import urllib.request
from typing import Optional, Tuple

RESOURCE = "https://vault.azure.net"
API_VERSION = "7.0"
REFERENCE_MSI = "http://localhost:40381/oauth2/token"
IMDS = "http://169.254.169.254/metadata/identity/oauth2/token"


class KeyVaultError(RuntimeError):
    pass


def _get_json(url: str, headers=None, data: Optional[bytes] = None, timeout: float = 10.0):
    req = urllib.request.Request(url, data=data, headers=headers or {}, method="POST" if data else "GET")
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return json.loads(r.read())
    except urllib.error.HTTPError as e:
        raise KeyVaultError(f"{url} → HTTP {e.code}: {e.read()[:200]!r}") from None
    except (urllib.error.URLError, OSError, ValueError) as e:
        raise KeyVaultError(f"{url}: {e}") from None


class TokenProvider:
    def __init__(self):
        self._tok: Optional[Tuple[str, float]] = None
        self._lock = threading.Lock()

    def _fetch(self) -> Tuple[str, float]:
        raise NotImplementedError

    def token(self) -> str:
        with self._lock:
            if self._tok is None or self._tok[1] - 300 < time.time():
                self._tok = self._fetch()
            return self._tok[0]


def _expiry(body) -> float:
    for k in ("expires_on", "expires_in"):
        if k in body:
            v = float(body[k])
            return v if k == "expires_on" else time.time() + v
    return time.time() + 3600


class MsiTokenProvider(TokenProvider):
    def __init__(self, endpoint: str):
        super().__init__()
        self.endpoint = endpoint

    def _fetch(self):
        sep = "&" if "?" in self.endpoint else "?"
        q = urllib.parse.urlencode({"resource": RESOURCE, "api-version": "2018-02-01"})
        body = _get_json(f"{self.endpoint}{sep}{q}", {"Metadata": "true"})
        return body["access_token"], _expiry(body)


class ClientSecretTokenProvider(TokenProvider):
    def __init__(self, tenant: str, client_id: str, secret: str, authority: str = "https://login.microsoftonline.com"):
        super().__init__()
        self.url = f"{authority.rstrip('/')}/{tenant}/oauth2/token"
        self.form = urllib.parse.urlencode({"grant_type": "client_credentials", "client_id": client_id,
                                            "client_secret": secret, "resource": RESOURCE}).encode()

    def _fetch(self):
        body = _get_json(self.url, {"Content-Type": "application/x-www-form-urlencoded"}, self.form)
        return body["access_token"], _expiry(body)


class KeyVaultClient:
    def __init__(self, url_template: str, tokens: TokenProvider):
        self.url_template = url_template
        self.tokens = tokens

    def get_secret(self, vault: str, name: str) -> str:
        base = self.url_template.format(vault=vault).rstrip("/")
        body = _get_json(f"{base}/secrets/{urllib.parse.quote(name)}?api-version={API_VERSION}",
                         {"Authorization": f"Bearer {self.tokens.token()}"})
        if "value" not in body:
            raise KeyVaultError(f"secret {vault}/{name}: no value in response")
        return body["value"]


_CLIENT: Optional[KeyVaultClient] = None
_CLIENT_KEY = None


def default_client() -> Optional[KeyVaultClient]:
    """Client configured from the environment, or None when ``DXA_KEYVAULT_URL`` is unset."""
    global _CLIENT, _CLIENT_KEY
    url = os.environ.get("DXA_KEYVAULT_URL")
    if not url:
        return None
    env = tuple(os.environ.get(k) for k in ("DXA_KEYVAULT_URL", "DXA_KEYVAULT_TENANT", "DXA_KEYVAULT_CLIENT_ID",
                                            "DXA_KEYVAULT_CLIENT_SECRET", "DXA_KEYVAULT_AUTHORITY",
                                            "DXA_KEYVAULT_MSI_ENDPOINT"))
    if _CLIENT is not None and _CLIENT_KEY == env:
        return _CLIENT
    _, tenant, cid, secret, authority, msi = env
    if tenant and cid and secret:
        tp: TokenProvider = ClientSecretTokenProvider(tenant, cid, secret,
                                                      authority or "https://login.microsoftonline.com")
    else:
        tp = MsiTokenProvider(msi or REFERENCE_MSI)
    _CLIENT, _CLIENT_KEY = KeyVaultClient(url, tp), env
    return _CLIENT
